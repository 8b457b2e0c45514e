#!/bin/bash
# rocprofv3 kernel-trace summary of a short bench run (kernel stats only; no PMC here).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 &&
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 1 --warmup 0 ${BENCH_ARGS:-} > gpurun_out/prof.log 2>&1
rc=$?
find gpurun_out/prof -name "*stats*" | head
exit $rc
