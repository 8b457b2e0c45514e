#!/bin/bash
# Fused decode launch timelines (stamp build) and the 8-rank TP engine test with 2 HW queues per process.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "attn_oproj" > gpurun_out/r4e_fused.log 2>&1 || exit $?
FS_MODE=ao timeout -k 10 200 python -u tools/fused_stamps.py > gpurun_out/r4e_stamps_ao_b1.log 2>&1 || exit $?
FS_MODE=qao timeout -k 10 200 python -u tools/fused_stamps.py > gpurun_out/r4e_stamps_qao_b1.log 2>&1 || exit $?
FS_MODE=qao FS_B=4 timeout -k 10 200 python -u tools/fused_stamps.py > gpurun_out/r4e_stamps_qao_b4.log 2>&1 || exit $?
timeout -k 10 600 python -u -m pytest tests/test_tp_gpu.py -x -v --timeout 500 --timeout-method thread \
  -k "8" > gpurun_out/r4e_tp8.log 2>&1
