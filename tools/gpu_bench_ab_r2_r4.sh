#!/bin/bash
# Round-4 evidence session on one MI355X:
#  1. the round-3 bench regression, settled on one box: round-2 HEAD (ab_r2/, a worktree of 28e502e with its
#     own built libraries) vs HEAD vs HEAD with the 4-wave prefill attention (RAGK_PREFILL_PP=0), 20+5 steps,
#     alternating;
#  2. the served path (Flask /generate, C=1 + Poisson).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # name, dir, env...
  local name=$1 dir=$2; shift 2
  (cd "$dir" && env "$@" timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --c1 3) \
    > gpurun_out/ab4_$name.json 2> gpurun_out/ab4_$name.err || return $?
  echo "$name: $(grep -o '"value": [0-9.]*\|"p50_latency_c1_ms": [0-9.]*' gpurun_out/ab4_$name.json | tr '\n' ' ')"
}
for round in 1 2; do
  run r2_$round ab_r2 X=1 || exit $?
  run head_$round . X=1 || exit $?
  run head_pp0_$round . RAGK_PREFILL_PP=0 || exit $?
done
timeout -k 10 500 python -u tools/bench_serve.py --c1 20 > gpurun_out/serve_r4.log 2>&1
