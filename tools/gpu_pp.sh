cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
SKIP_T=${SKIP_T:-0}; [ "$SKIP_T" = 1 ] || timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "attn_prefill" -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_pp.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/pytest_pp.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/attn_pp_ab.py > gpurun_out/attn_pp_ab.log 2>&1
rc=$?; echo "ab rc=$rc"; grep -v amdgpu.ids gpurun_out/attn_pp_ab.log; [ $rc -eq 0 ] || exit $rc
AP_STAMP=0 AP_LENS=2048,2048 AP_CTX=3000,0 timeout -k 10 300 python -u tools/attn_pp_ab.py > gpurun_out/attn_pp_ab2.log 2>&1
rc=$?; echo "ab2 rc=$rc"; grep -v amdgpu.ids gpurun_out/attn_pp_ab2.log; exit $rc
