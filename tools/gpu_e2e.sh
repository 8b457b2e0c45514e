#!/bin/bash
# GPU validation + headline bench on one MI355X box (run via gpurun). Each GPU step has its own limit,
# steps are chained with && so nothing runs after a failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 &&
timeout -k 10 600 python -m pytest tests -m gpu -q -rf -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 900 python bench.py ${BENCH_ARGS:-} --json-out gpurun_out/bench.json > gpurun_out/bench.log 2>&1
rc=$?
echo "exit $rc"
tail -5 gpurun_out/pytest_gpu.log; tail -3 gpurun_out/smoke.log; tail -3 gpurun_out/bench.log
exit $rc
