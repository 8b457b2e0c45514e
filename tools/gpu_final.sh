#!/bin/bash
# Closing validation on one MI355X: GPU suite, smoke(), a 10 + 3-step headline bench, and a rocprofv3
# kernel summary of a short bench run (gpu_profile_bench.sh). TAG names the logs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${TAG:-r5}
BENCH=0 TAG=$T bash tools/gpu_validate.sh || exit $?
timeout -k 10 600 python -u bench.py --steps ${BSTEPS:-10} --warmup 3 > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err || exit $?
cat gpurun_out/bench_$T.json
bash tools/gpu_profile_bench.sh
