#!/bin/bash
# Decode knob A/B on one MI355X (gpurun): batch 1 and 32 decode step time under a few settings.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for cfg in "base:" "mt2:RAGK_DECODE_MIN_TILES=2" "blk1024:RAGK_DECODE_BLOCKS=1024" "nomerge:RAGK_DECODE_OPROJ_MERGE=0" "mt8:RAGK_DECODE_MIN_TILES=8"; do
  name=${cfg%%:*}; envs=${cfg#*:}
  echo "== $name $envs"
  timeout -k 10 240 env $envs DA_STEPS=48 python -u tools/decode_anatomy.py ${BS:-1 32} 2>&1 | grep -E "^B=" || { echo "failed"; exit 1; }
done
