#!/bin/bash
# 8 TP ranks as 8 processes on ONE GPU (tests/test_tp_gpu.py, opt-in case) under a rocprofv3 kernel trace:
# which collective kernel of which rank waited, and whether its peers' matching kernels were running.
# Analysis: python tools/tp_trace_report.py gpurun_out/tp8trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/tp8trace
RAGK_TEST_TP8=1 timeout -k 10 900 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tp8trace -o "%pid%_run" \
  -- python3 -m pytest tests/test_tp_gpu.py -k "widths_on_one_gpu and 8" -x -q -p no:cacheprovider --timeout 800 \
  --timeout-method thread > gpurun_out/tp8trace.log 2>&1
rc=$?
echo "pytest under rocprofv3 rc=$rc"
grep -E "passed|failed|CommError|timed out" gpurun_out/tp8trace.log | tail -12
python3 tools/tp_trace_report.py gpurun_out/tp8trace > gpurun_out/tp8trace_report.txt 2>&1
head -60 gpurun_out/tp8trace_report.txt
exit 0
