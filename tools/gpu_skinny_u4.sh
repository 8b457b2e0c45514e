#!/bin/bash
# Batch-1 skinny GEMM: 4 vs 2 K blocks in flight per wave (tests, then decode_anatomy in one process).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
RAGK_SKINNY_UNROLL=4 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "skinny or test_gemm_small or gemm_dec" > gpurun_out/sku4_tests.log 2>&1 || exit $?
tail -1 gpurun_out/sku4_tests.log
DA_SKU=4,2,4,2 DA_STEPS=40 timeout -k 10 400 python -u tools/decode_anatomy.py 1 4 > gpurun_out/sku4_da.log 2>&1 || exit $?
grep -E "^--|ms/step" gpurun_out/sku4_da.log | grep -v replay
