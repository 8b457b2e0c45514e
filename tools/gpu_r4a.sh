#!/bin/bash
# Round-4 first GPU session: TP engine at 2/4/8 ranks on one GPU, the full GPU suite, a short bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_tp_gpu.py tests/test_ipc_allreduce_gpu.py -x -v --timeout 600 \
  --timeout-method thread > gpurun_out/r4a_tp.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r4a_gpu.log 2>&1 &&
timeout -k 10 500 python bench.py --steps 10 --warmup 3 > gpurun_out/r4a_bench.json 2> gpurun_out/r4a_bench.err
