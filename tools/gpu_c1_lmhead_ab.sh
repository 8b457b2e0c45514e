#!/bin/bash
# C=1: vocab projection skinny GEMM unrolled too (max blocks 0 = no limit) vs only the few-block shapes (2048).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  for mb in 2048 0; do
    RAGK_SKINNY_UNROLL_MAX_BLOCKS=$mb C1_N=4 timeout -k 10 300 python tools/c1_probe.py > gpurun_out/c1lm_${mb}_$r.log 2>&1 || exit $?
    echo "max_blocks=$mb: $(tail -1 gpurun_out/c1lm_${mb}_$r.log)"
  done
done
