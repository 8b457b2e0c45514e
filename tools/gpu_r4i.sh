#!/bin/bash
# Split-K decode GEMMs with the add_partials_rmsnorm consumer in their last blocks (gemm_part.hip TL):
# kernel tests, TP=1 decode-step A/B at batch 1 / 32 (same process, alternating), C=1 probe.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "part_tail or merge_tail or add_partials or test_gemm_part" > gpurun_out/r4i_tail.log 2>&1 || exit $?
tail -2 gpurun_out/r4i_tail.log
DA_TAIL=1,0,1,0 DA_STEPS=48 timeout -k 10 400 python -u tools/decode_anatomy.py 1 32 > gpurun_out/r4i_da.log 2>&1 || exit $?
grep -E "^--|ms/step" gpurun_out/r4i_da.log
for t in 1 0; do
  RAGK_DECODE_PART_TAIL=$t C1_N=4 timeout -k 10 300 python tools/c1_probe.py > gpurun_out/r4i_c1_$t.log 2>&1 || exit $?
  echo "tail=$t: $(tail -1 gpurun_out/r4i_c1_$t.log)"
done
DA_NT=1,0,1,0 DA_STEPS=48 timeout -k 10 400 python -u tools/decode_anatomy.py 32 > gpurun_out/r4i_nt.log 2>&1 || exit $?
grep -E "^--|ms/step" gpurun_out/r4i_nt.log
DA_FM=1,0,1,0 DA_STEPS=48 timeout -k 10 400 python -u tools/decode_anatomy.py 1 32 > gpurun_out/r4i_fm.log 2>&1 || exit $?
grep -E "^--|ms/step" gpurun_out/r4i_fm.log
