#!/bin/bash
# C=1: batch-1 skinny GEMM (down) with nt weight loads (default) vs default-policy loads; the vocab GEMM
# keeps the 1-block plain form in both. Separate processes, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  for nt in 1 0; do
    RAGK_SKINNY_NT=$nt C1_N=4 timeout -k 10 300 python tools/c1_probe.py > gpurun_out/c1snt_${nt}_$r.log 2>&1 || exit $?
    echo "skinny_nt=$nt: $(tail -1 gpurun_out/c1snt_${nt}_$r.log)"
  done
done
