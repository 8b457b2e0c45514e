#!/bin/bash
# Served path (Flask /generate -> MicroBatcher -> EngineLoop): C=1, then Poisson 8 req/s once per
# decode-aware prefill budget (MIXED, comma list; the first is the server's configured value).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r5}
timeout -k 10 800 python -u tools/bench_serve.py --c1 20 --mixed-prefill-tokens ${MIXED:-2048,1024,512} \
  --json-out gpurun_out/serve_$T.json > gpurun_out/serve_$T.log 2>&1 || exit $?
grep -E "^C=1|^Poisson" gpurun_out/serve_$T.log
