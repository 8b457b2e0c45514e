#!/bin/bash
# C=1 and batch 4: split-K decode GEMM (gemm_part) with nt weight loads (default) vs default policy; separate
# processes, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  for nt in 1 0; do
    RAGK_PART_NT=$nt C1_N=4 timeout -k 10 300 python tools/c1_probe.py > gpurun_out/c1pnt_${nt}_$r.log 2>&1 || exit $?
    echo "part_nt=$nt: $(tail -1 gpurun_out/c1pnt_${nt}_$r.log)"
  done
done
