#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_realshape_gpu.py tests/test_e2e_gpu.py -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "prefill or realshape or e2e" > gpurun_out/pytest_wide.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/pytest_wide.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 600 python -u bench.py --steps 5 --warmup 2 > gpurun_out/bench_wide.json 2> gpurun_out/bench_wide.err || exit $?
grep -o '"value": [0-9.]*\|"p50_latency_c1_ms": [0-9.]*\|"prefill_s": [0-9.]*\|"ttft_p50_ms": [0-9.]*' gpurun_out/bench_wide.json | tr '\n' ' '
