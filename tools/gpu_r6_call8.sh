#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
AP_VARIANTS=base,diag,nt0,base,diag timeout -k 10 200 python3 -u tools/attn_decode_probe.py > gpurun_out/ap1.log 2>&1 || { tail -5 gpurun_out/ap1.log; exit 1; }
cat gpurun_out/ap1.log | grep -v amdgpu.ids
AP_JITTER=150 AP_VARIANTS=base,diag timeout -k 10 200 python3 -u tools/attn_decode_probe.py > gpurun_out/ap2.log 2>&1 || { tail -5 gpurun_out/ap2.log; exit 1; }
cat gpurun_out/ap2.log | grep -v amdgpu.ids
TAG=r6 WHICH=fp8 bash tools/gpu_configs.sh
