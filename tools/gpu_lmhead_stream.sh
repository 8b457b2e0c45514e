#!/bin/bash
# Vocab projection on the stream GEMM with nt weights (STREAM_MAX_ROWS 200000) vs gemm_dec / skinny (32768).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
DA_NATIVE=STREAM_MAX_ROWS:200000,32768,200000,32768 DA_STEPS=40 timeout -k 10 400 python -u tools/decode_anatomy.py 32 4 > gpurun_out/lmh_nt.log 2>&1 || exit $?
grep -E "^--|ms/step" gpurun_out/lmh_nt.log | grep -v replay
