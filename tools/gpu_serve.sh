#!/bin/bash
# Served path (Flask /generate -> MicroBatcher -> EngineLoop): C=1, then Poisson 8 req/s once per
# mixed:max prefill budget pair in CONFIGS (decode-aware cap : tokens per prefill step; same server).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r5}
timeout -k 10 900 python -u tools/bench_serve.py --c1 20 --poisson-configs ${CONFIGS:-0:8192,0:32768,2048:32768,8192:32768} \
  --json-out gpurun_out/serve_$T.json > gpurun_out/serve_$T.log 2>&1 || exit $?
grep -E "^C=1|^Poisson" gpurun_out/serve_$T.log
