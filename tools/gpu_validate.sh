#!/bin/bash
# Validation on one MI355X: the whole GPU test suite, smoke(), a short headline bench. TAG names the logs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r5}
timeout -k 10 1080 python -u -m pytest tests -m gpu -q -rf -x --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu_$T.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -6 gpurun_out/pytest_gpu_$T.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$T.log 2>&1 || exit $?
tail -1 gpurun_out/smoke_$T.log
[ "${BENCH:-1}" = "1" ] || exit 0
timeout -k 10 600 python -u bench.py --steps ${BSTEPS:-5} --warmup 2 > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err || exit $?
cat gpurun_out/bench_$T.json
