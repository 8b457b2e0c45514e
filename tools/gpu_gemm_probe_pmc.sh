#!/bin/bash
# GEMM probe (gemm_w4 vs torch.mm / hipBLASLt at M = 32768) and its PMC passes, round 4.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
PROBE_M=32768 PROBE_PATHS=6,torch timeout -k 10 300 python3 -u tools/gemm_probe.py > gpurun_out/gemm_probe_r4.log 2>&1 || exit $?
cat gpurun_out/gemm_probe_r4.log
PROBE_M=32768 PROBE_PATHS=6,torch bash tools/gpu_pmc_gemm.sh || exit $?
python3 tools/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc_summary_r4.txt 2>&1; head -40 gpurun_out/pmc_summary_r4.txt
