#!/bin/bash
# Batch-32 decode anatomy (tools/decode_anatomy.py 32: engine ms/step, graph-replay ms/step) and its
# rocprofv3 kernel summary. TAG names the outputs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pdb32
T=${TAG:-r6}
DA_STEPS=${DA_STEPS:-64} timeout -k 10 300 python3 -u tools/decode_anatomy.py 32 > gpurun_out/decode_b32_$T.log 2>&1 || { tail -20 gpurun_out/decode_b32_$T.log; exit 1; }
grep "B=" gpurun_out/decode_b32_$T.log
[ "${PROF:-1}" = "1" ] || exit 0
rm -rf gpurun_out/pdb32/*
DA_STEPS=${DA_STEPS:-64} timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pdb32 -o run -- python3 tools/decode_anatomy.py 32 > gpurun_out/pdb32.log 2>&1 || exit $?
rm -f gpurun_out/pdb32/*kernel_trace.csv
python3 tools/rocprof_summary.py gpurun_out/pdb32/run_kernel_stats.csv 30 > gpurun_out/decode_b32_kernels_$T.txt && head -24 gpurun_out/decode_b32_kernels_$T.txt
