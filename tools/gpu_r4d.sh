#!/bin/bash
# Fused decode launches after the done-flag change: kernel tests, C=1 A/B over the decode paths, a kernel
# profile of the fused and the unfused C=1 path, the TP engine tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "attn_oproj or gemm_part_merge or attn_decode_rope" > gpurun_out/r4d_fused.log 2>&1 || exit $?
for mode in "qao:X=1" "qao0:RAGK_AO_MIA=0" "ao:RAGK_DECODE_QAO=0" "ao0:RAGK_DECODE_QAO=0 RAGK_AO_MIA=0" "unfused:RAGK_DECODE_ATTN_OPROJ=0"; do
  name=${mode%%:*}; envs=${mode#*:}
  env $envs C1_N=4 timeout -k 10 300 python tools/c1_probe.py > gpurun_out/r4d_c1_$name.log 2>&1 || exit $?
  echo "$name: $(tail -1 gpurun_out/r4d_c1_$name.log)"
done
for mode in "qao:X=1" "ao:RAGK_DECODE_QAO=0" "unfused:RAGK_DECODE_ATTN_OPROJ=0"; do
  name=${mode%%:*}; envs=${mode#*:}
  mkdir -p gpurun_out/pc1_$name
  env $envs C1_N=2 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pc1_$name -o run \
    -- python3 tools/c1_probe.py > gpurun_out/pc1_$name.log 2>&1 || exit $?
  rm -f gpurun_out/pc1_$name/*kernel_trace.csv
  python tools/rocprof_summary.py gpurun_out/pc1_$name/run_kernel_stats.csv 30 > gpurun_out/pc1_${name}_summary.txt 2>&1
done
timeout -k 10 900 python -u -m pytest tests/test_tp_gpu.py -x -v --timeout 600 --timeout-method thread \
  > gpurun_out/r4d_tp.log 2>&1
