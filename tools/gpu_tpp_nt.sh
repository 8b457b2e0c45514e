#!/bin/bash
# TP=8 8B shard at batch 32: nt decode attention (default from batch 8) vs never; separate processes, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  for nt in 8 100000; do
    RAGK_DECODE_NT_MIN_BH=$nt timeout -k 10 300 python -u tools/tp_decode_probe.py 32 > gpurun_out/tppnt_${nt}_$r.log 2>&1 || exit $?
    echo "nt_min_b=$nt: $(grep 'replay' gpurun_out/tppnt_${nt}_$r.log)"
  done
done
