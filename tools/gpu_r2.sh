#!/bin/bash
# Round-2 GPU validation on one MI355X (run via gpurun): new TP tests, the full GPU suite, the
# headline bench and a rocprofv3 kernel-trace summary of it. Every GPU step has its own limit and
# the steps are chained with &&.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
STEP=${STEP:-all}
if [ "$STEP" = "tp" ] || [ "$STEP" = "all" ]; then
timeout -k 10 600 python -u -m pytest tests/test_tp_gpu.py tests/test_ipc_allreduce_gpu.py -v --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_tp.log 2>&1
rc=$?; echo "tp rc=$rc"; tail -8 gpurun_out/pytest_tp.log
# 1 = test failures (keep going); anything else (timeout, crash) ends the call here
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
if [ "$STEP" = "all" ] || [ "$STEP" = "suite" ]; then
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider --deselect tests/test_tp_gpu.py > gpurun_out/pytest_gpu.log 2>&1
echo "suite rc=$?"; tail -15 gpurun_out/pytest_gpu.log
fi
if [ "$STEP" = "all" ] || [ "$STEP" = "serve" ]; then
timeout -k 10 600 python -u tools/bench_serve.py --json-out gpurun_out/serve.json ${SERVE_ARGS:-} > gpurun_out/serve.log 2>&1
echo "serve rc=$?"; grep -E "^C=1|^Poisson" gpurun_out/serve.log
fi
if [ "$STEP" = "all" ] || [ "$STEP" = "bench" ]; then
timeout -k 10 600 python -u bench.py --steps ${BSTEPS:-3} --warmup 1 --json-out gpurun_out/bench.json > gpurun_out/bench.log 2>&1 &&
tail -2 gpurun_out/bench.log &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 1 --warmup 0 --c1 0 > gpurun_out/prof.log 2>&1
rc=$?; echo "bench rc=$rc"
rm -f gpurun_out/prof/*kernel_trace.csv  # keep the stats (the full trace exceeds the copy-back limit)
python tools/rocprof_summary.py gpurun_out/prof/run_kernel_stats.csv 40 > gpurun_out/rocprof_summary.txt 2>&1
fi
