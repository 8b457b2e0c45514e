#!/bin/bash
# A/B of the small-batch top-k chunking (RAGK_TOPK_SMALL_B=0: 7 chunks at every batch) at decode batch 1,
# engine GPU tests (sampling / async paths), and a kernel profile + C=1 anatomy with it on.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ptk
timeout -k 10 400 python -u -m pytest tests/test_e2e_gpu.py tests/test_kernels_gpu.py -k "sample or topk or engine or async or greedy" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/t_topk.log 2>&1
rc=$?; tail -3 gpurun_out/t_topk.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 env RAGK_TOPK_SMALL_B=0 python -u tools/decode_anatomy.py 1 2 > gpurun_out/tk_off.log 2>&1 && grep "decode steps" gpurun_out/tk_off.log &&
timeout -k 10 300 python -u tools/decode_anatomy.py 1 2 > gpurun_out/tk_on.log 2>&1 && grep "decode steps" gpurun_out/tk_on.log &&
DA_STEPS=32 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ptk -o run -- python3 tools/decode_anatomy.py 1 > gpurun_out/ptk.log 2>&1 &&
rm -f gpurun_out/ptk/*kernel_trace.csv && python tools/rocprof_summary.py gpurun_out/ptk/run_kernel_stats.csv 25 > gpurun_out/ptk_summary.txt 2>&1 && grep -E "topk|sample" gpurun_out/ptk_summary.txt | cut -c1-110 &&
timeout -k 10 300 python -u tools/c1_probe.py > gpurun_out/c1_tk.log 2>&1 && tail -1 gpurun_out/c1_tk.log
