#!/bin/bash
# The TP engine tests (2 / 4 / 8 processes on one GPU) and the peer-mapped collective tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1000 python3 -u -m pytest ${TP_FILES:-tests/test_ipc_allreduce_gpu.py tests/test_tp_gpu.py} ${TP_X--x} -v \
  -p no:cacheprovider --timeout 900 --timeout-method thread -m gpu > gpurun_out/tp_once.log 2>&1
rc=$?
echo "tp tests rc=$rc"
grep -E "PASSED|FAILED|passed|failed|never arrived" gpurun_out/tp_once.log | tail -30
exit $rc
