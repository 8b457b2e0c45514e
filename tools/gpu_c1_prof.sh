#!/bin/bash
# rocprofv3 kernel summary of the C=1 RAG query path (tools/c1_probe.py) on one MI355X.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pc1
C1_N=4 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pc1 -o run -- python3 tools/c1_probe.py > gpurun_out/pc1.log 2>&1
rc=$?; rm -f gpurun_out/pc1/*kernel_trace.csv
python tools/rocprof_summary.py gpurun_out/pc1/run_kernel_stats.csv 40 > gpurun_out/pc1_summary.txt 2>&1
tail -1 gpurun_out/pc1.log; exit $rc
