#!/bin/bash
# PMC passes (one rocprofv3 run per counter set, kernel-trace only) over tools/gemm_probe.py.
# Analyse with: python tools/pmc_summary.py gpurun_out/pmc
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
export PROBE_ROUNDS=1 PROBE_ITERS=3
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
timeout -s KILL 120 rocprofv3 --pmc $P1 --kernel-trace --output-format csv -d gpurun_out/pmc/p1 -o run -- python3 tools/gemm_probe.py > gpurun_out/pmc/p1.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc $P2 --kernel-trace --output-format csv -d gpurun_out/pmc/p2 -o run -- python3 tools/gemm_probe.py > gpurun_out/pmc/p2.log 2>&1
rc=$?
grep TF gpurun_out/pmc/p1.log
exit $rc
