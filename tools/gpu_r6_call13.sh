#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
AP_CHECK=1 AP_VARIANTS=base,kl,base,kl timeout -k 10 200 python3 -u tools/attn_decode_probe.py > gpurun_out/ap7.log 2>&1 || { tail -5 gpurun_out/ap7.log; exit 1; }
grep -v amdgpu.ids gpurun_out/ap7.log
