#!/bin/bash
# TP=8 rank-0 shard decode probe (8B and 70B shards) on the current tree.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/tp_decode_probe.py 1 4 32 > gpurun_out/tpp_final.log 2>&1 || exit $?
grep "ms/step" gpurun_out/tpp_final.log
TPP_MODEL=70b timeout -k 10 400 python -u tools/tp_decode_probe.py 1 32 > gpurun_out/tpp70_final.log 2>&1 || exit $?
grep "ms/step" gpurun_out/tpp70_final.log
