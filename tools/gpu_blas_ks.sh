#!/bin/bash
# Bench A/B of the per-projection hipBLASLt route for the residual-add prefill GEMMs (RAGK_PREFILL_BLAS_KS):
# all (default: o_proj K=4096 and down K=14336 on hipBLASLt), o only, down only. Same box, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  for ks in all 4096 14336; do
    v=$ks; [ "$ks" = all ] && v=
    RAGK_PREFILL_BLAS_KS=$v timeout -k 10 400 python -u bench.py --steps ${BSTEPS:-10} --warmup 3 --c1 0 > gpurun_out/blasks_${ks}_$r.log 2>&1 || exit $?
    echo "ks=$ks run $r: $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/blasks_${ks}_$r.log | tr '\n' ' ')"
  done
done
