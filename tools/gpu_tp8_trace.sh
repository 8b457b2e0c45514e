#!/bin/bash
# The 8-rank TP engine test (tests/test_tp_gpu.py, 8 processes on ONE GPU):
#  (a) with 4 hardware queues per process (the HIP default) under a rocprofv3 kernel trace: which
#      collective kernel of which rank waited, and whether its peers' matching kernels were running;
#  (b) without the profiler, with the test's own setting (one hardware queue per rank).
# Analysis of (a): python tools/tp_trace_report.py gpurun_out/tp8trace
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/tp8trace
rm -rf gpurun_out/tp8trace/*
GPU_MAX_HW_QUEUES=${TRACE_QUEUES:-4} RAGK_TEST_TP8=1 timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv \
  -d gpurun_out/tp8trace -o "%pid%_run" -- python3 -m pytest tests/test_tp_gpu.py -k "widths_on_one_gpu and 8" -x -q \
  -p no:cacheprovider --timeout 500 --timeout-method thread > gpurun_out/tp8trace.log 2>&1
rc=$?
echo "(a) pytest under rocprofv3, ${TRACE_QUEUES:-4} queues per process: rc=$rc"
grep -E "passed|failed|CommError|timed out|never arrived" gpurun_out/tp8trace.log | sort | uniq -c | head -12
python3 tools/tp_trace_report.py gpurun_out/tp8trace > gpurun_out/tp8trace_report.txt 2>&1
head -40 gpurun_out/tp8trace_report.txt
find gpurun_out/tp8trace -name "*kernel_trace.csv" -size +20M -delete
[ $rc -le 1 ] || exit $rc
RAGK_TEST_TP8=1 timeout -k 10 600 python3 -u -m pytest tests/test_tp_gpu.py -k "widths_on_one_gpu and 8" -x -q \
  -p no:cacheprovider --timeout 500 --timeout-method thread > gpurun_out/tp8_q1.log 2>&1
rc=$?
echo "(b) pytest, 1 queue per rank: rc=$rc"
tail -3 gpurun_out/tp8_q1.log
exit $rc
