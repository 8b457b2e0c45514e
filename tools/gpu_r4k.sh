#!/bin/bash
# Non-temporal decode attention: batch threshold (1 / 4 / 16) and the bench A/B (nt from batch 8 vs never),
# then the idle-gap profile of a short bench run (tools/gpu_r4j.sh).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
DA_NT=1,0,1,0 DA_STEPS=48 timeout -k 10 400 python -u tools/decode_anatomy.py 1 4 16 > gpurun_out/r4k_nt.log 2>&1 || exit $?
grep -E "^--|ms/step" gpurun_out/r4k_nt.log | grep -v replay
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --c1 3 > gpurun_out/ab4k_$name.json 2> gpurun_out/ab4k_$name.err || return $?
  echo "$name: $(grep -o '"value": [0-9.]*\|"p50_latency_c1_ms": [0-9.]*\|"decode_s": [0-9.]*\|"prefill_s": [0-9.]*' gpurun_out/ab4k_$name.json | tr '\n' ' ')"
}
for round in 1 2; do
  run nt_$round X=1 || exit $?
  run nont_$round RAGK_DECODE_NT_MIN_B=100000 || exit $?
done
bash tools/gpu_r4j.sh
