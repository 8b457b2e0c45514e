#!/bin/bash
# gemm_w4 (path 6: continuous K-stream kernel for K < 8192, spread schedule for K >= 8192) vs
# hipBLASLt (torch.matmul) on the Llama-3.1-8B prefill shapes at M=32768: interleaved timing, then
# one PMC pass (MFMA busy / issue waits / clock). Summaries: tools/pmc_summary.py gpurun_out/pmc.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
export PROBE_M=32768 PROBE_PATHS=6,torch
timeout -k 10 300 python3 -u tools/gemm_probe.py > gpurun_out/gemm_probe.log 2>&1 &&
cat gpurun_out/gemm_probe.log &&
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT" &&
PROBE_ROUNDS=1 PROBE_ITERS=3 timeout -s KILL 180 rocprofv3 --pmc $P1 --kernel-trace --output-format csv -d gpurun_out/pmc/p1 -o run -- python3 tools/gemm_probe.py > gpurun_out/pmc/p1.log 2>&1
rc=$?
python3 tools/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc_summary.txt 2>&1
exit $rc
