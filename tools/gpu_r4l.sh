#!/bin/bash
# Batch-1 skinny GEMM with two K blocks in flight per wave + nt weights: kernel tests, decode A/B, then
# the idle-gap profile of a short bench run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "skinny or gemm_small or test_gemm_" > gpurun_out/r4l_tests.log 2>&1 || exit $?
tail -1 gpurun_out/r4l_tests.log
DA_SKU=2,1,2,1 DA_STEPS=48 timeout -k 10 400 python -u tools/decode_anatomy.py 1 > gpurun_out/r4l_sku.log 2>&1 || exit $?
grep -E "^--|ms/step" gpurun_out/r4l_sku.log | grep -v replay
bash tools/gpu_r4j.sh
