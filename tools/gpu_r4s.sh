#!/bin/bash
# In-bench yardstick: prefill GEMMs on gemm_w4 (default) vs hipBLASLt for the plain qkv GEMM vs hipBLASLt
# for qkv + the residual-epilogue o_proj / down (in-place addmm). 20 + 5 steps, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --c1 3 > gpurun_out/ab4s_$name.json 2> gpurun_out/ab4s_$name.err || return $?
  echo "$name: $(grep -o '"value": [0-9.]*\|"p50_latency_c1_ms": [0-9.]*\|"decode_s": [0-9.]*\|"prefill_s": [0-9.]*' gpurun_out/ab4s_$name.json | tr '\n' ' ')"
}
for round in 1 2; do
  run w4_$round X=1 || exit $?
  run plain_$round RAGK_PREFILL_BLAS=plain || exit $?
  run all_$round RAGK_PREFILL_BLAS=all || exit $?
done
