#!/bin/bash
# Round-3 closing run on one MI355X: GPU test suite, smoke(), the headline bench, then the GEMM probe
# (gemm_w4 vs torch.mm at M=32768) with one PMC pass. Each GPU step has its own limit; stop at the first
# step that dies of anything but test failures.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -4 gpurun_out/pytest_gpu.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
tail -1 gpurun_out/smoke.log
timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 --json-out gpurun_out/bench_final.json > gpurun_out/bench_final.log 2>&1 || exit $?
tail -1 gpurun_out/bench_final.log
export PROBE_M=32768 PROBE_PATHS=6,torch
timeout -k 10 300 python3 -u tools/gemm_probe.py > gpurun_out/gemm_probe.log 2>&1 || exit $?
cat gpurun_out/gemm_probe.log
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT"
PROBE_ROUNDS=1 PROBE_ITERS=3 timeout -s KILL 180 rocprofv3 --pmc $P1 --kernel-trace --output-format csv -d gpurun_out/pmc/p1 -o run -- python3 tools/gemm_probe.py > gpurun_out/pmc/p1.log 2>&1
rc=$?
python3 tools/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc_summary.txt 2>&1
cat gpurun_out/pmc_summary.txt | head -30
exit $rc
