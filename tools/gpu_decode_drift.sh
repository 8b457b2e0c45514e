#!/bin/bash
# Batch-32 decode step time in situ after the prefill, by window (RAGK_DECODE_TIMING=1), with and without an
# idle pause between prefill and decode, with GPU clocks / power sampled alongside (rocm-smi).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
( for i in $(seq 1 150); do date +%s.%N; /opt/rocm/bin/rocm-smi -c -P --csv 2>/dev/null | tail -n +2; sleep 0.3; done ) > gpurun_out/drift_smi.txt 2>&1 &
SMI=$!
for sl in 0 3; do
  RAGK_DECODE_TIMING=1 DA_SLEEP=$sl DA_STEPS=${DA_STEPS:-160} timeout -k 10 300 python3 -u tools/decode_anatomy.py 32 > gpurun_out/drift_$sl.log 2>&1 || { kill $SMI; tail -20 gpurun_out/drift_$sl.log; exit 1; }
  echo "sleep $sl:"; grep "B=" gpurun_out/drift_$sl.log
done
kill $SMI 2>/dev/null
exit 0
