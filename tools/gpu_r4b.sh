#!/bin/bash
# Round-4 GPU session: fused decode launches (attention + o_proj; qkv + attention + o_proj) vs the unfused
# kernels, C=1 A/B over the three decode paths, TP engine at 2/4/8 ranks, the full GPU suite, a short bench.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread \
  -k "attn_oproj or gemm_part_merge or attn_decode_rope" > gpurun_out/r4b_fused.log 2>&1 &&
C1_N=4 timeout -k 10 300 python tools/c1_probe.py > gpurun_out/r4b_c1_qao.log 2>&1 &&
C1_N=4 RAGK_DECODE_QAO=0 timeout -k 10 300 python tools/c1_probe.py > gpurun_out/r4b_c1_ao.log 2>&1 &&
C1_N=4 RAGK_DECODE_ATTN_OPROJ=0 timeout -k 10 300 python tools/c1_probe.py > gpurun_out/r4b_c1_unfused.log 2>&1 &&
timeout -k 10 900 python -u -m pytest tests/test_tp_gpu.py -x -v --timeout 600 --timeout-method thread \
  > gpurun_out/r4b_tp.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/r4b_gpu.log 2>&1 &&
timeout -k 10 500 python bench.py --steps 10 --warmup 3 > gpurun_out/r4b_bench.json 2> gpurun_out/r4b_bench.err
