#!/bin/bash
# C=1: batch-1 skinny GEMM with 2 K blocks in flight (default) vs 1 (the round-3 kernel), both default-policy loads.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  for u in 2 1; do
    RAGK_SKINNY_UNROLL=$u C1_N=4 timeout -k 10 300 python tools/c1_probe.py > gpurun_out/c1su_${u}_$r.log 2>&1 || exit $?
    echo "unroll=$u: $(tail -1 gpurun_out/c1su_${u}_$r.log)"
  done
done
