#!/bin/bash
# Prefill chunk budget 32768 (default) vs 65536 tokens per step, bench 20+5 steps, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --c1 3 > gpurun_out/abch_$name.json 2> gpurun_out/abch_$name.err || return $?
  echo "$name: $(grep -o '"value": [0-9.]*\|"p50_latency_c1_ms": [0-9.]*\|"ttft_p50_ms": [0-9.]*\|"prefill_s": [0-9.]*' gpurun_out/abch_$name.json | tr '\n' ' ')"
}
for round in 1 2; do
  run c32k_$round X=1 || exit $?
  run c64k_$round MAX_PREFILL_TOKENS=65536 || exit $?
done
