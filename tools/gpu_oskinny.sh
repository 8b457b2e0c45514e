#!/bin/bash
# TP=1 small-batch o_proj as skinny GEMM + residual epilogue + plain norm vs split-K slabs (+ merge) + consumer.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
DA_LLAMA=DECODE_OPROJ_SKINNY_MAX_M:4,0,4,0 DA_STEPS=40 timeout -k 10 400 python -u tools/decode_anatomy.py 1 4 > gpurun_out/oskinny.log 2>&1 || exit $?
grep -E "^--|ms/step" gpurun_out/oskinny.log | grep -v replay
