#!/bin/bash
# TP=8-shard decode probe with / without the fused decode launches (8B and 70B shards), then the
# round-3 bench regression A/B and the served path (tools/gpu_r4c.sh).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for mode in "unfused:X=1" "ao:RAGK_DECODE_ATTN_OPROJ=1 RAGK_DECODE_QAO=0" "qao:RAGK_DECODE_ATTN_OPROJ=1"; do
  name=${mode%%:*}; envs=${mode#*:}
  env $envs timeout -k 10 300 python -u tools/tp_decode_probe.py 1 4 32 > gpurun_out/tpp_$name.log 2>&1 || exit $?
  echo "$name: $(grep -h 'ms/step' gpurun_out/tpp_$name.log | tr '\n' ' ')"
done
env RAGK_DECODE_ATTN_OPROJ=1 TPP_MODEL=70b TPP_PREFILL=32768 timeout -k 10 400 python -u tools/tp_decode_probe.py 1 32 \
  > gpurun_out/tpp70_qao.log 2>&1 || exit $?
TPP_MODEL=70b timeout -k 10 400 python -u tools/tp_decode_probe.py 1 32 > gpurun_out/tpp70_unfused.log 2>&1 || exit $?
bash tools/gpu_r4c.sh
