#!/bin/bash
# A/B of the o_proj partition merge (RAGK_DECODE_OPROJ_MERGE) at decode batch 1 / 2 on one MI355X,
# plus its numerics tests and a C=1 anatomy.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "merge or decode or gemm_part or splitk" -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/t_merge.log 2>&1
rc=$?; tail -3 gpurun_out/t_merge.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 env RAGK_DECODE_OPROJ_MERGE=0 python -u tools/decode_anatomy.py 1 2 > gpurun_out/da_off.log 2>&1 && grep "graph replay" gpurun_out/da_off.log &&
timeout -k 10 300 env RAGK_DECODE_OPROJ_MERGE=1 python -u tools/decode_anatomy.py 1 2 > gpurun_out/da_on.log 2>&1 && grep "graph replay" gpurun_out/da_on.log &&
timeout -k 10 300 python -u tools/c1_probe.py > gpurun_out/c1_on.log 2>&1 && tail -1 gpurun_out/c1_on.log
