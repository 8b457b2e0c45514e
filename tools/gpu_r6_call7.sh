#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
RAGK_DECODE_TIMING=1 DA_MID=30 DA_STEPS=96 timeout -k 10 300 python3 -u tools/decode_anatomy.py 32 > gpurun_out/da32_mid.log 2>&1 || { tail -5 gpurun_out/da32_mid.log; exit 1; }
grep "B=" gpurun_out/da32_mid.log
RAGK_DECODE_TIMING=1 DA_NT=0 DA_STEPS=64 timeout -k 10 300 python3 -u tools/decode_anatomy.py 32 > gpurun_out/da32_nt0.log 2>&1 || { tail -5 gpurun_out/da32_nt0.log; exit 1; }
grep "B=\|--" gpurun_out/da32_nt0.log
