#!/bin/bash
# Re-run the kernel tests that follow the new defaults, then the TP engine tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "attn_oproj or test_gemm_part or part_tail or stream_part" > gpurun_out/pytest_r4p.log 2>&1
rc=$?; echo "kernels rc=$rc"; tail -3 gpurun_out/pytest_r4p.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_tp_gpu.py -v -rf --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_tp_r4.log 2>&1
rc=$?; echo "tp rc=$rc"; grep -E "PASSED|FAILED|passed|failed" gpurun_out/pytest_tp_r4.log | tail -6
