#!/bin/bash
# Stream-slab policy sweeps (tools/decode_anatomy.py DA_NATIVE, same process, alternating): batch threshold,
# tile rows for the 48-tile qkv, and the vocab projection on the stream GEMM.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
DA_NATIVE=STREAM_PART_MIN_M:1,17,1,17 DA_STEPS=40 timeout -k 10 400 python -u tools/decode_anatomy.py 4 8 16 > gpurun_out/r4n_minm.log 2>&1 || exit $?
grep -E "^--|ms/step" gpurun_out/r4n_minm.log | grep -v replay
DA_NATIVE=STREAM_PART_ROWS:64,0,64,0 DA_STEPS=40 timeout -k 10 300 python -u tools/decode_anatomy.py 32 > gpurun_out/r4n_rows.log 2>&1 || exit $?
grep -E "^--|ms/step" gpurun_out/r4n_rows.log | grep -v replay
DA_NATIVE=STREAM_MAX_ROWS:200000,32768,200000,32768 DA_STEPS=40 timeout -k 10 400 python -u tools/decode_anatomy.py 1 32 > gpurun_out/r4n_lmh.log 2>&1 || exit $?
grep -E "^--|ms/step" gpurun_out/r4n_lmh.log | grep -v replay
