#!/bin/bash
# C=1: stream-GEMM row floor (RAGK_STREAM_MIN_ROWS 16384 default vs 4096: the 4096-row down projection on the stream GEMM);
# separate processes, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  for mb in 16384 4096; do
    RAGK_STREAM_MIN_ROWS=$mb C1_N=4 timeout -k 10 300 python tools/c1_probe.py > gpurun_out/c1smr_${mb}_$r.log 2>&1 || exit $?
    echo "stream_min_rows=$mb: $(tail -1 gpurun_out/c1smr_${mb}_$r.log)"
  done
done
