#!/bin/bash
# C=1 prefill of one 5.2k-token prompt: split-K gemm_w4c + add_partials_rmsnorm (default) vs the plain
# residual-add route (hipBLASLt addmm) for o_proj / down; separate processes, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  for sk in 1 0; do
    RAGK_PREFILL_SPLITK=$sk C1_N=4 timeout -k 10 300 python tools/c1_probe.py > gpurun_out/c1sk_${sk}_$r.log 2>&1 || exit $?
    echo "splitk=$sk: $(tail -1 gpurun_out/c1sk_${sk}_$r.log)"
  done
done
