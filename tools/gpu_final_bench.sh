#!/bin/bash
# Round-end evidence on one MI355X: the headline bench (10 timed + 3 warm-up steps), then the rocprofv3
# kernel summaries of the C=1 query path and of a short bench run. TAG names the outputs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-final}
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 600 python -u bench.py --steps ${BSTEPS:-10} --warmup 3 > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err || exit $?
  cat gpurun_out/bench_$T.json
fi
[ "${PROF:-1}" = "1" ] || exit 0
bash tools/gpu_c1_prof.sh || exit $?
bash tools/gpu_profile_bench.sh
