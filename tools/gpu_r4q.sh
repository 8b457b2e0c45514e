#!/bin/bash
# TP engine tests (2 / 4 / 8 ranks on one GPU) after the warm-up barrier, then the stream-slab count sweep.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_tp_gpu.py -v -rf --timeout 600 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_tp_r4.log 2>&1
rc=$?; echo "tp rc=$rc"; grep -E "PASSED|FAILED|passed|failed" gpurun_out/pytest_tp_r4.log | tail -6; [ $rc -le 1 ] || exit $rc
DA_NATIVE=STREAM_PART_MAX_S:4,64,4,64 DA_STEPS=40 timeout -k 10 300 python -u tools/decode_anatomy.py 32 > gpurun_out/r4q_maxs.log 2>&1 || exit $?
grep -E "^--|ms/step" gpurun_out/r4q_maxs.log | grep -v replay
