#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
AP_CHECK=1 AP_VARIANTS=base,kl,diag_dma,base,kl timeout -k 10 200 python3 -u tools/attn_decode_probe.py > gpurun_out/ap5.log 2>&1 || { tail -5 gpurun_out/ap5.log; exit 1; }
grep -v amdgpu.ids gpurun_out/ap5.log
AP_JITTER=150 AP_VARIANTS=base,kl,base,kl timeout -k 10 200 python3 -u tools/attn_decode_probe.py > gpurun_out/ap6.log 2>&1 || { tail -5 gpurun_out/ap6.log; exit 1; }
grep -v amdgpu.ids gpurun_out/ap6.log
