#!/bin/bash
# batch-32 decode: in-situ vs replay kernel durations (kernel trace split by phase) + replay variants
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pdb32t
rm -rf gpurun_out/pdb32t/*
DA_REPLAY_MODES=h2d,d2h,both DA_STEPS=64 timeout -k 10 300 python3 -u tools/decode_anatomy.py 32 > gpurun_out/da32_modes.log 2>&1 || { tail -20 gpurun_out/da32_modes.log; exit 1; }
grep "B=" gpurun_out/da32_modes.log
DA_STEPS=64 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pdb32t -o run -- python3 tools/decode_anatomy.py 32 > gpurun_out/pdb32t.log 2>&1 || { tail -5 gpurun_out/pdb32t.log; exit 1; }
f=$(find gpurun_out/pdb32t -name "*kernel_trace.csv" | head -1)
python3 tools/phase_kernel_stats.py "$f" attn_decode 672 64 > gpurun_out/phase_b32.txt && head -30 gpurun_out/phase_b32.txt
gzip -f "$f"
