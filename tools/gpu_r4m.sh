#!/bin/bash
# Split-K decode slabs from the LDS-DMA stream GEMM: kernel tests, decode A/B at batch 32 / 16, bench A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "stream_part or test_gemm_part" > gpurun_out/r4m_tests.log 2>&1 || exit $?
tail -1 gpurun_out/r4m_tests.log
DA_SP=1,0,1,0 DA_STEPS=48 timeout -k 10 400 python -u tools/decode_anatomy.py 32 16 > gpurun_out/r4m_sp.log 2>&1 || exit $?
grep -E "^--|ms/step" gpurun_out/r4m_sp.log | grep -v replay
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --c1 3 > gpurun_out/ab4m_$name.json 2> gpurun_out/ab4m_$name.err || return $?
  echo "$name: $(grep -o '"value": [0-9.]*\|"p50_latency_c1_ms": [0-9.]*\|"decode_s": [0-9.]*\|"prefill_s": [0-9.]*' gpurun_out/ab4m_$name.json | tr '\n' ' ')"
}
for round in 1 2; do
  run sp_$round RAGK_DECODE_STREAM_PART=1 || exit $?
  run base_$round X=1 || exit $?
done
