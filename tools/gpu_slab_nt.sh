#!/bin/bash
# Stream-GEMM decode slabs with nt weights (default) vs default-policy loads at batch 32; separate processes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  for nt in 1 0; do
    RAGK_STREAM_PART_NT=$nt DA_STEPS=40 timeout -k 10 300 python -u tools/decode_anatomy.py 32 > gpurun_out/slabnt_${nt}_$r.log 2>&1 || exit $?
    echo "slab_nt=$nt: $(grep 'decode steps' gpurun_out/slabnt_${nt}_$r.log)"
  done
done
