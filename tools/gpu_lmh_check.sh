#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_e2e_gpu.py -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider \
  -k "vocab_stream or stream or e2e or engine" > gpurun_out/pytest_lmh.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/pytest_lmh.log
