#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --c1 3 > gpurun_out/abnw_$name.json 2> gpurun_out/abnw_$name.err || return $?
  echo "$name: $(grep -o '"value": [0-9.]*\|"p50_latency_c1_ms": [0-9.]*\|"decode_s": [0-9.]*' gpurun_out/abnw_$name.json | tr '\n' ' ')"
}
for round in 1 2; do
  run nw8_$round X=1 || exit $?
  run nw4_$round RAGK_DECODE_NW8=0 || exit $?
done
