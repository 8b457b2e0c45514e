#!/bin/bash
# C=1 with the batch-1 skinny GEMM unrolled (2 K blocks in flight, default) vs the round-3 form (1), in
# separate processes, alternating; then the same in one process (decode_anatomy).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  for u in 2 1; do
    RAGK_SKINNY_UNROLL=$u C1_N=4 timeout -k 10 300 python tools/c1_probe.py > gpurun_out/r4v_c1_${u}_$r.log 2>&1 || exit $?
    echo "unroll=$u: $(tail -1 gpurun_out/r4v_c1_${u}_$r.log)"
  done
done
