#!/bin/bash
# rocprofv3 kernel statistics of a short bench run (2 timed steps + 1 warmup, 2 C=1 queries).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_final
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_final -o run -- python3 bench.py --steps 2 --warmup 1 --c1 2 --c1-tp 0 > gpurun_out/prof_final.log 2>&1 || exit $?
s=$(find gpurun_out/prof_final -name "*kernel_stats.csv" | head -1)
python tools/rocprof_summary.py "$s" 40 > gpurun_out/prof_final_summary.txt && head -24 gpurun_out/prof_final_summary.txt
f=$(find gpurun_out/prof_final -name "*kernel_trace.csv" | head -1)
rm -f "$f"
