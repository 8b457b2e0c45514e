#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "stream or gemm_part" --timeout 120 --timeout-method thread > gpurun_out/pt_stream.log 2>&1
rc=$?; tail -4 gpurun_out/pt_stream.log; [ $rc = 0 ] || exit $rc
DA_PAIR=64,0 DA_NATIVE=STREAM_PART_ROWS:128,0,128,0 DA_STEPS=48 timeout -k 10 400 python3 -u tools/decode_anatomy.py 32 > gpurun_out/da32_tiles.log 2>&1 || { tail -5 gpurun_out/da32_tiles.log; exit 1; }
grep "B=\|--" gpurun_out/da32_tiles.log
