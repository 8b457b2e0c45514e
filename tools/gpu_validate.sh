#!/bin/bash
# Round-4 validation on one MI355X: the whole GPU test suite, smoke(), a short headline bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu_r4.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -6 gpurun_out/pytest_gpu_r4.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r4.log 2>&1 || exit $?
tail -1 gpurun_out/smoke_r4.log
timeout -k 10 600 python -u bench.py --steps 5 --warmup 2 > gpurun_out/bench_r4.json 2> gpurun_out/bench_r4.err || exit $?
cat gpurun_out/bench_r4.json
