#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
AP_MODES=15,16,14,10 AP_ROUNDS=6 timeout -k 10 300 python -u tools/attn_pp_ab.py > gpurun_out/attn_prio_bench.log 2>&1 || exit $?
grep "pp=" gpurun_out/attn_prio_bench.log
AP_LENS=5200 AP_MODES=15,16 AP_ROUNDS=6 timeout -k 10 300 python -u tools/attn_pp_ab.py > gpurun_out/attn_prio_c1.log 2>&1 || exit $?
grep "pp=" gpurun_out/attn_prio_c1.log
