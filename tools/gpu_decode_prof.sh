#!/bin/bash
# Decode anatomy at batch 1 and 32 (wall ms/step), then a rocprofv3 kernel-stats pass per batch size.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/decode_anatomy.py ${DA_BS:-1 32} > gpurun_out/decode_anatomy.log 2>&1 &&
cat gpurun_out/decode_anatomy.log | grep -v amdgpu.ids &&
for B in ${DA_PROF_BS:-1 32}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pdec$B -o run -- python3 tools/decode_anatomy.py $B > gpurun_out/pdec$B.log 2>&1 || exit $?
  rm -f gpurun_out/pdec$B/*kernel_trace.csv
  python3 tools/rocprof_summary.py gpurun_out/pdec$B/run_kernel_stats.csv 30 > gpurun_out/pdec${B}_summary.txt 2>&1
done
