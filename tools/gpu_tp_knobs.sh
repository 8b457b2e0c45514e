#!/bin/bash
# TP=8-shard decode probe A/B (gpurun): fused-reduction fences, stream GEMM for the shard's gate/up.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for cfg in "light:" "fences:RAGK_AR_FENCES=1" "stream:RAGK_STREAM_MIN_ROWS=2048"; do
  name=${cfg%%:*}; envs=${cfg#*:}
  echo "== $name $envs"
  timeout -k 10 300 env $envs TPP_STEPS=32 python -u tools/tp_decode_probe.py 1 32 2>&1 | grep -E "^B=.*replay" || { echo "failed"; exit 1; }
done
