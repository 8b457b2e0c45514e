#!/bin/bash
# nt rule by batch x KV heads: TP=1 batch 32 (256 -> nt) and the TP=8 shard at batch 32 (32 -> no nt),
# each vs the opposite setting; decode tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q --timeout 120 --timeout-method thread -k "attn_decode" > gpurun_out/ntrule_tests.log 2>&1 || exit $?
tail -1 gpurun_out/ntrule_tests.log
for r in 1 2; do
  for bh in 64 100000; do
    RAGK_DECODE_NT_MIN_BH=$bh timeout -k 10 300 python -u tools/tp_decode_probe.py 32 > gpurun_out/ntrule_tp_${bh}_$r.log 2>&1 || exit $?
    echo "tp shard min_bh=$bh: $(grep 'replay' gpurun_out/ntrule_tp_${bh}_$r.log)"
  done
done
