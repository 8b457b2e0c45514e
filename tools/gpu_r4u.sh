#!/bin/bash
# TP engine tests alone, verbose, progress in gpurun_out/tp_test_progress.log.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_tp_gpu.py -v -rf --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_tp_r4u.log 2>&1
rc=$?; echo "tp rc=$rc"; grep -E "PASSED|FAILED|passed|failed" gpurun_out/pytest_tp_r4u.log | tail -6
cat gpurun_out/tp_test_progress.log | awk '{print $1, $2, $3, $4, $5, $6}' | sort -k3 | tail -30
