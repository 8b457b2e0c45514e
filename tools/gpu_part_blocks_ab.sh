#!/bin/bash
# A/B of the split-K decode GEMM slice choice at batch 32 (RAGK_PART_MIN_BLOCKS: 512 -> down uses
# 28-step slices, 512 blocks of 131 VGPRs = 2 rounds on 256 CUs; 1024 -> 14-step slices, 1024 blocks).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for mb in 512 1024 512 1024; do
  timeout -k 10 300 env RAGK_PART_MIN_BLOCKS=$mb python -u tools/decode_anatomy.py 32 16 > gpurun_out/pb_$mb.log 2>&1 || exit $?
  echo "min_blocks=$mb"; grep "graph replay" gpurun_out/pb_$mb.log
done
