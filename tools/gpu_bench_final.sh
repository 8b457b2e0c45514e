#!/bin/bash
# Final headline run: bench.py 20 + 5 steps with the defaults, twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for r in 1 2; do
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_final_$r.json 2> gpurun_out/bench_final_$r.err || exit $?
  echo "run $r: $(grep -o '"value": [0-9.]*\|"p50_latency_c1_ms": [0-9.]*\|"ttft_p50_ms": [0-9.]*\|"p50_latency_ms": [0-9.]*' gpurun_out/bench_final_$r.json | tr '\n' ' ')"
done
