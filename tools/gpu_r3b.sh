cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
AP_STAMP=0 timeout -k 10 300 python -u tools/attn_pp_ab.py > gpurun_out/attn_pp_ab.log 2>&1
rc=$?; echo "ab rc=$rc"; grep -v amdgpu.ids gpurun_out/attn_pp_ab.log; [ $rc -eq 0 ] || exit $rc
STEP=suite,bench BSTEPS=3 bash tools/gpu_r3.sh
