#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
AP_VARIANTS=base,diag,diag_dma,base,diag,diag_dma timeout -k 10 200 python3 -u tools/attn_decode_probe.py > gpurun_out/ap3.log 2>&1 || { tail -5 gpurun_out/ap3.log; exit 1; }
grep -v amdgpu.ids gpurun_out/ap3.log
AP_B=256 AP_HKV=1 AP_VARIANTS=base,diag,diag_dma,base,diag,diag_dma timeout -k 10 200 python3 -u tools/attn_decode_probe.py > gpurun_out/ap4.log 2>&1 || { tail -5 gpurun_out/ap4.log; exit 1; }
grep -v amdgpu.ids gpurun_out/ap4.log
