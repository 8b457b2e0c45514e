#!/bin/bash
# Served path (Flask /generate -> MicroBatcher -> EngineLoop): C=1 + Poisson 8 req/s.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/bench_serve.py --c1 20 > gpurun_out/serve_r4_final.log 2>&1 || exit $?
grep -E "^C=1|^Poisson" gpurun_out/serve_r4_final.log
