#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "skinny or test_gemm_small or gemm_dec or vocab" > gpurun_out/skc_tests.log 2>&1 || exit $?
tail -1 gpurun_out/skc_tests.log
for r in 1 2; do
  C1_N=4 timeout -k 10 300 python tools/c1_probe.py > gpurun_out/skc_c1_$r.log 2>&1 || exit $?
  echo "default: $(tail -1 gpurun_out/skc_c1_$r.log)"
done
