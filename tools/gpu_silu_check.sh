#!/bin/bash
# Kernel tests touching SiLU epilogues and decode attention, then the gate/up probe vs hipBLASLt.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python3 -u -m pytest tests/test_kernels_gpu.py tests/test_e2e_gpu.py tests/test_realshape_gpu.py -x -q --timeout 200 \
  --timeout-method thread -k "silu or w4 or pingpong or decode or stream or part or e2e or realshape or engine" > gpurun_out/silu_tests.log 2>&1 \
  || { tail -30 gpurun_out/silu_tests.log; exit 1; }
tail -2 gpurun_out/silu_tests.log
PROBE_M=32768 PROBE_SHAPES=2,0 PROBE_PATHS=6,blas PROBE_ROUNDS=5 timeout -k 10 200 python3 -u tools/gemm_probe.py > gpurun_out/silu_probe.log 2>&1 || exit 1
grep TF gpurun_out/silu_probe.log
