#!/bin/bash
# Phase C of the persistent decode MLP (next layer's input norm + qkv GEMM in-launch): engine + real-shape
# GPU tests, then the batch-1 decode step alternating phase C on / off in the engine.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_mlp_engine_gpu.py tests/test_realshape_gpu.py -x -q -p no:cacheprovider \
  --timeout 200 --timeout-method thread > gpurun_out/nq_tests.log 2>&1 || { tail -40 gpurun_out/nq_tests.log; exit 1; }
tail -2 gpurun_out/nq_tests.log
DA_NATIVE=MLP_ENGINE_NEXT_QKV:1,0,1,0 timeout -k 10 400 python -u tools/decode_anatomy.py 1 > gpurun_out/nq_c1.log 2>&1 || { tail -20 gpurun_out/nq_c1.log; exit 1; }
grep -E "^--|ms/step" gpurun_out/nq_c1.log
