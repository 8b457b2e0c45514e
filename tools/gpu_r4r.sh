#!/bin/bash
# Decode attention split at batch 32 with nt loads: 256 / 512 / 1024 target blocks (max_parts 1 / 2 / 4).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
DA_NATIVE=DECODE_TARGET_BLOCKS:256,512,1024,256,512,1024 DA_STEPS=40 timeout -k 10 400 python -u tools/decode_anatomy.py 32 > gpurun_out/r4r_blocks.log 2>&1 || exit $?
grep -E "^--|ms/step" gpurun_out/r4r_blocks.log | grep -v replay
