#!/bin/bash
# A/B of the round-2 C=1 levers on one MI355X: o_proj merging the decode attention's split-K
# partitions (RAGK_DECODE_OPROJ_MERGE), split-K prefill o_proj / down (RAGK_PREFILL_SPLITK), the
# decode attention's first-tile prefetch (always on; compare with the previous logs).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "merge or decode or gemm_part or splitk" -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/t_merge.log 2>&1
rc=$?; tail -4 gpurun_out/t_merge.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/decode_anatomy.py 1 4 32 > gpurun_out/da_on.log 2>&1 && tail -6 gpurun_out/da_on.log &&
timeout -k 10 300 python -u tools/c1_probe.py > gpurun_out/c1_on.log 2>&1 && tail -2 gpurun_out/c1_on.log
