#!/bin/bash
# The other BASELINE configs on one MI355X, each a JSON line plus a rocprofv3 kernel summary:
#   config 5: Llama-3.1-8B fp8 weights, bge-large embedder, 10k FlatL2, C=32
#   config 4 (one GPU): Llama-3.1-70B bf16, 1M-vector IVF-Flat, C=32
# TAG names the outputs (gpurun_out/bench_{fp8,70b_ivf}_$TAG.json, ..._kernels_$TAG.txt).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-r5}
run() {  # name, timeout, bench args...
  local name=$1 lim=$2
  shift 2
  timeout -k 10 "$lim" python -u bench.py "$@" > gpurun_out/bench_${name}_$T.json 2> gpurun_out/bench_${name}_$T.err || return $?
  cat gpurun_out/bench_${name}_$T.json
}
prof() {  # name, timeout, bench args...
  local name=$1 lim=$2
  shift 2
  rm -rf gpurun_out/prof_$name
  timeout -k 10 "$lim" rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$name -o run -- python3 bench.py "$@" \
    > gpurun_out/prof_${name}_$T.log 2>&1 || return $?
  local s
  s=$(find gpurun_out/prof_$name -name "*kernel_stats.csv" | head -1)
  python3 tools/rocprof_summary.py "$s" 40 > gpurun_out/bench_${name}_kernels_$T.txt && head -16 gpurun_out/bench_${name}_kernels_$T.txt
  find gpurun_out/prof_$name -name "*kernel_trace.csv" -delete
}
FP8="--dtype fp8 --embedder bge-large"
B70="--model 70b --index ivf --index-vectors 1000000"
case "${WHICH:-all}" in
  fp8) run fp8 600 $FP8 --steps 5 --warmup 2 && prof fp8 600 $FP8 --steps 2 --warmup 1 --c1 1 --c1-tp 0 ;;
  70b) run 70b_ivf 900 $B70 --steps 2 --warmup 1 --c1 1 && prof 70b_ivf 900 $B70 --steps 1 --warmup 1 --c1 0 --c1-tp 0 ;;
  70b_run) run 70b_ivf 1000 $B70 --steps 2 --warmup 1 --c1 1 ;;
  70b_prof) prof 70b_ivf 1000 $B70 --steps 1 --warmup 1 --c1 0 --c1-tp 0 ;;
  all) run fp8 600 $FP8 --steps 5 --warmup 2 && prof fp8 600 $FP8 --steps 2 --warmup 1 --c1 1 --c1-tp 0 &&
       run 70b_ivf 900 $B70 --steps 2 --warmup 1 --c1 1 && prof 70b_ivf 900 $B70 --steps 1 --warmup 1 --c1 0 --c1-tp 0 ;;
esac
