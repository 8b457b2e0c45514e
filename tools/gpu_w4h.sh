#!/bin/bash
# gemm_w4: bit-exactness / numerics tests, then the M = 32768 probe of the four Llama-8B prefill shapes
# (+ the residual shapes without their epilogue) against hipBLASLt (torch.mm and the in-place addmm the
# library route uses), interleaved in one process.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "w4 or pingpong or large_m or splitk or gemm_plain" > gpurun_out/w4h_tests.log 2>&1 || { tail -30 gpurun_out/w4h_tests.log; exit 1; }
tail -3 gpurun_out/w4h_tests.log
PROBE_M=32768 PROBE_SHAPES=${PROBE_SHAPES:-0,1,2,3,4,5} PROBE_PATHS=${PROBE_PATHS:-6,torch,blas} PROBE_ROUNDS=5 \
  timeout -k 10 300 python3 -u tools/gemm_probe.py > gpurun_out/w4h_probe.log 2>&1 || { tail -30 gpurun_out/w4h_probe.log; exit 1; }
grep TF gpurun_out/w4h_probe.log
