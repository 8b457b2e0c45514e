#!/bin/bash
# GEMM routing tests + e2e / real-shape tests under the new default, then a profiled short bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_r4t
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_e2e_gpu.py tests/test_realshape_gpu.py -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "gemm or prefill or e2e or realshape or engine" > gpurun_out/pytest_r4t.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/pytest_r4t.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_r4t -o run -- python3 bench.py --steps 2 --warmup 1 --c1 2 --c1-tp 0 > gpurun_out/prof_r4t.log 2>&1 || exit $?
s=$(find gpurun_out/prof_r4t -name "*kernel_stats.csv" | head -1)
python tools/rocprof_summary.py "$s" 40 > gpurun_out/prof_r4t_summary.txt && head -30 gpurun_out/prof_r4t_summary.txt
f=$(find gpurun_out/prof_r4t -name "*kernel_trace.csv" | head -1)
rm -f "$f"
