#!/bin/bash
# C=1: decode-attention partition size (RAGK_DECODE_MIN_TILES: 4 default, 2, 1 = more, shorter KV partitions);
# separate processes, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  for mb in ${TILES:-4 2 1}; do
    RAGK_DECODE_MIN_TILES=$mb C1_N=4 timeout -k 10 300 python tools/c1_probe.py > gpurun_out/c1dmt_${mb}_$r.log 2>&1 || exit $?
    echo "decode_min_tiles=$mb: $(tail -1 gpurun_out/c1dmt_${mb}_$r.log)"
  done
done
