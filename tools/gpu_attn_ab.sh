#!/bin/bash
# Prefill attention A/B (tools/attn_pp_ab.py, AP_VARIANTS) on the bench workloads: one 32k-token step of
# 6 x 5.4k prompts, one 5.2k prompt, a 2k chunk over 3k of context.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out

{ timeout -k 10 120 python3 -u tools/attn_pp_ab.py &&
  AP_LENS=5200 timeout -k 10 120 python3 -u tools/attn_pp_ab.py &&
  AP_LENS=2048 AP_CTX=3072 timeout -k 10 120 python3 -u tools/attn_pp_ab.py; } > gpurun_out/attn_ab.log 2>&1
rc=$?
cat gpurun_out/attn_ab.log | grep -v amdgpu.ids
exit $rc
