#!/bin/bash
# The 8-rank TP engine test (tests/test_tp_gpu.py, 8 processes on ONE GPU):
#  (b) as the suite runs it (2 hardware queues per rank: tests/test_tp_gpu.py _init sets them), no profiler;
#  (a) the same under a rocprofv3 kernel trace (_init overrides the GPU_MAX_HW_QUEUES below too): which
#      collective kernel of which rank waited, and whether its peers' matching kernels were running.
# Analysis of (a): python tools/tp_trace_report.py gpurun_out/tp8trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/tp8trace
rm -rf gpurun_out/tp8trace/*
T="tests/test_tp_gpu.py::test_tp_llama8b_widths_on_one_gpu[8]"
timeout -k 10 560 python3 -u -m pytest "$T" -x -q -p no:cacheprovider --timeout 540 \
  --timeout-method thread > gpurun_out/tp8_q1.log 2>&1
rc=$?
echo "(b) pytest, 2 queues per rank: rc=$rc"
tail -3 gpurun_out/tp8_q1.log
[ $rc -le 1 ] || exit $rc
[ "${TRACE:-1}" = "1" ] || exit $rc
GPU_MAX_HW_QUEUES=4 timeout -k 10 560 rocprofv3 --kernel-trace --output-format csv \
  -d gpurun_out/tp8trace -o "%pid%_run" -- python3 -m pytest "$T" -x -q -p no:cacheprovider --timeout 540 \
  --timeout-method thread > gpurun_out/tp8trace.log 2>&1
rc2=$?
echo "(a) pytest under rocprofv3, 2 queues per process: rc=$rc2"
grep -E "passed|failed|CommError|never arrived" gpurun_out/tp8trace.log | sort | uniq -c | head -12
python3 tools/tp_trace_report.py gpurun_out/tp8trace > gpurun_out/tp8trace_report.txt 2>&1
head -40 gpurun_out/tp8trace_report.txt
find gpurun_out/tp8trace -name "*kernel_trace.csv" -size +20M -delete
exit $rc
