#!/bin/bash
# Prefill attention v3 with the LDS-staged whole-row epilogue (pp 15) vs the per-lane 8-B stores (pp 10):
# bench shape (6 x 5.4k causal), one 5.2k prompt (C=1), and a 2k chunk over 3k of context.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
AP_MODES=10,15 AP_ROUNDS=6 timeout -k 10 300 python -u tools/attn_pp_ab.py > gpurun_out/attn_wide_bench.log 2>&1 || exit $?
grep "pp=" gpurun_out/attn_wide_bench.log
AP_LENS=5200 AP_MODES=10,15 AP_ROUNDS=6 timeout -k 10 300 python -u tools/attn_pp_ab.py > gpurun_out/attn_wide_c1.log 2>&1 || exit $?
grep "pp=" gpurun_out/attn_wide_c1.log
AP_LENS=2048 AP_CTX=3072 AP_MODES=10,15 AP_ROUNDS=6 timeout -k 10 300 python -u tools/attn_pp_ab.py > gpurun_out/attn_wide_chunk.log 2>&1 || exit $?
grep "pp=" gpurun_out/attn_wide_chunk.log
