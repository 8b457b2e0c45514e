#!/bin/bash
# batch-32 decode in situ: async (timing events), sync decode path, async with a host delay per step
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
run() { local tag=$1; shift; env "$@" DA_STEPS=96 timeout -k 10 300 python3 -u tools/decode_anatomy.py 32 > gpurun_out/da32_$tag.log 2>&1 || { tail -5 gpurun_out/da32_$tag.log; exit 1; }; echo "== $tag"; grep "B=" gpurun_out/da32_$tag.log; }
run base RAGK_DECODE_TIMING=1
run sync RAGK_ASYNC_DECODE=0
run delay RAGK_DECODE_TIMING=1 RAGK_FAULTS=step_delay_ms=3
