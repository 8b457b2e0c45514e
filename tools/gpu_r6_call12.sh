#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_canary_gpu.py -x -q -k "decode or attn" --timeout 120 --timeout-method thread > gpurun_out/pt_attn.log 2>&1
rc=$?; tail -4 gpurun_out/pt_attn.log; [ $rc = 0 ] || exit $rc
DA_NATIVE=DECODE_KL:0,1,0,1 DA_STEPS=48 timeout -k 10 400 python3 -u tools/decode_anatomy.py 32 > gpurun_out/da32_kl.log 2>&1 || { tail -5 gpurun_out/da32_kl.log; exit 1; }
grep "B=\|--" gpurun_out/da32_kl.log
