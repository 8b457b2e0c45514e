cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pd1
DA_STEPS=32 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pd1 -o run -- python3 tools/decode_anatomy.py 1 > gpurun_out/pd1.log 2>&1
rc=$?; rm -f gpurun_out/pd1/*kernel_trace.csv; python tools/rocprof_summary.py gpurun_out/pd1/run_kernel_stats.csv 25 > gpurun_out/pd1_summary.txt 2>&1; cat gpurun_out/pd1_summary.txt | cut -c1-150; exit $rc
