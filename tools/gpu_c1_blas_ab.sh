#!/bin/bash
# C=1: qkv (no-epilogue GEMM) on hipBLASLt too (RAGK_PREFILL_BLAS=all) vs gemm_w4 (resid, default).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  for m in resid all; do
    RAGK_PREFILL_BLAS=$m C1_N=4 timeout -k 10 300 python tools/c1_probe.py > gpurun_out/c1blas_${m}_$r.log 2>&1 || exit $?
    echo "blas=$m: $(tail -1 gpurun_out/c1blas_${m}_$r.log)"
  done
done
