#!/bin/bash
# Fused decode v2 (full-K o_proj blocks, single-round-trip merge): tests, stamp timelines, C=1 A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "attn_oproj" > gpurun_out/r4f_fused.log 2>&1 || exit $?
FS_MODE=ao timeout -k 10 200 python -u tools/fused_stamps.py > gpurun_out/r4f_stamps_ao_b1.log 2>&1 || exit $?
FS_MODE=qao timeout -k 10 200 python -u tools/fused_stamps.py > gpurun_out/r4f_stamps_qao_b1.log 2>&1 || exit $?
FS_MODE=ao FS_B=4 timeout -k 10 200 python -u tools/fused_stamps.py > gpurun_out/r4f_stamps_ao_b4.log 2>&1 || exit $?
for mode in "qao:X=1" "ao:RAGK_DECODE_QAO=0" "unfused:RAGK_DECODE_ATTN_OPROJ=0"; do
  name=${mode%%:*}; envs=${mode#*:}
  env $envs C1_N=4 timeout -k 10 300 python tools/c1_probe.py > gpurun_out/r4f_c1_$name.log 2>&1 || exit $?
  echo "$name: $(tail -1 gpurun_out/r4f_c1_$name.log)"
done
