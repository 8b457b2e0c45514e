#!/bin/bash
# Where the bench step waits on the host: kernel trace of a 2-step bench run -> idle-gap report.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/prof_gap
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_gap -o run -- \
  python3 bench.py --steps 2 --warmup 1 --c1 0 --c1-tp 0 > gpurun_out/prof_gap.log 2>&1 || exit $?
f=$(find gpurun_out/prof_gap -name "*kernel_trace.csv" | head -1)
python tools/gap_report.py "$f" > gpurun_out/gap_report.txt && cat gpurun_out/gap_report.txt
s=$(find gpurun_out/prof_gap -name "*kernel_stats.csv" | head -1)
python tools/rocprof_summary.py "$s" 30 > gpurun_out/prof_gap_summary.txt
gzip -f "$f"
