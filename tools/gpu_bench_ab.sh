#!/bin/bash
# Same-box A/B of the headline bench: OLD_ENV (default: the residual projections on hipBLASLt, RAGK_PREFILL_BLAS=resid) vs the
# current defaults, alternating runs. Each GPU step has its own limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for round in 1 2; do
  env ${OLD_ENV:-RAGK_PREFILL_BLAS=resid} timeout -k 10 500 python -u bench.py --steps ${BSTEPS:-3} --warmup 1 --c1 ${C1:-3} --json-out gpurun_out/bench_ab_old_$round.json > gpurun_out/bench_ab_old_$round.log 2>&1 || exit $?
  echo "old $round: $(grep -o '"value": [0-9.]*\|"p50_latency_c1_ms": [0-9.]*' gpurun_out/bench_ab_old_$round.log | tr '\n' ' ')"
  timeout -k 10 500 python -u bench.py --steps ${BSTEPS:-3} --warmup 1 --c1 ${C1:-3} --json-out gpurun_out/bench_ab_new_$round.json > gpurun_out/bench_ab_new_$round.log 2>&1 || exit $?
  echo "new $round: $(grep -o '"value": [0-9.]*\|"p50_latency_c1_ms": [0-9.]*' gpurun_out/bench_ab_new_$round.log | tr '\n' ' ')"
done
