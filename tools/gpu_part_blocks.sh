#!/bin/bash
# C=1: split-K slice policy (RAGK_PART_MIN_BLOCKS: 512 default, 256 = fewer/longer slabs, 1024 = more/shorter);
# separate processes, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  for mb in 512 256 1024; do
    RAGK_PART_MIN_BLOCKS=$mb C1_N=4 timeout -k 10 300 python tools/c1_probe.py > gpurun_out/c1pmb_${mb}_$r.log 2>&1 || exit $?
    echo "part_min_blocks=$mb: $(tail -1 gpurun_out/c1pmb_${mb}_$r.log)"
  done
done
