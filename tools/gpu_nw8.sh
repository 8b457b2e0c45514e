#!/bin/bash
# 8-wave single-partition decode attention (no merge launch) at batch 32: tests, then decode A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "attn_decode" > gpurun_out/nw8_tests.log 2>&1 || exit $?
tail -1 gpurun_out/nw8_tests.log
DA_NATIVE=DECODE_NW8_MIN_PAIRS:256,0,256,0 DA_STEPS=40 timeout -k 10 400 python -u tools/decode_anatomy.py 32 > gpurun_out/nw8_da.log 2>&1 || exit $?
grep -E "^--|ms/step" gpurun_out/nw8_da.log | grep -v replay
