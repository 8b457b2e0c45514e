#!/bin/bash
# gate/up SiLU*up stream GEMM tile rows: 128 (one block per CU, deeper ring) vs 64 (two per CU, default).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
DA_PAIR=128,64,128,64 DA_STEPS=40 timeout -k 10 400 python -u tools/decode_anatomy.py 1 32 > gpurun_out/pair_da.log 2>&1 || exit $?
grep -E "^--|ms/step" gpurun_out/pair_da.log | grep -v replay
