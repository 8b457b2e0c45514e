#!/bin/bash
# gemm_w4 (4-wave prefill GEMM) numerics + interleaved A/B vs the ping-pong kernel and hipBLASLt.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "pingpong" > gpurun_out/w4_test.log 2>&1 &&
PROBE_PATHS=2,6,torch timeout -k 10 180 python tools/gemm_probe.py > gpurun_out/w4_probe.log 2>&1 &&
PROBE_PATHS=2,6 PROBE_M=32768 timeout -k 10 180 python tools/gemm_probe.py >> gpurun_out/w4_probe.log 2>&1
rc=$?
tail -3 gpurun_out/w4_test.log; grep TF gpurun_out/w4_probe.log
exit $rc
