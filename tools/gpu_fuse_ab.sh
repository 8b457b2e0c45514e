#!/bin/bash
# Decode fusion A/B: GPU tests of the fused kernels, then decode anatomy (in-situ graph timing) for
# (rope fused, norm fused) = (0,0), (1,0), (1,1) at batch 32 and 1.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "attn_decode or rope or part_norm" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/t_fuse.log 2>&1 &&
timeout -k 10 300 python -u -m pytest tests/test_e2e_gpu.py tests/test_realshape_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/t_fuse_e2e.log 2>&1 || { tail -20 gpurun_out/t_fuse.log gpurun_out/t_fuse_e2e.log; exit 1; }
tail -n 1 gpurun_out/t_fuse.log gpurun_out/t_fuse_e2e.log
for cfg in ${FUSE_CFGS:-0,0 1,0 1,1}; do
  r=${cfg%,*}; n=${cfg#*,}
  echo "== rope_fused=$r norm_fused=$n"
  RAGK_DECODE_ROPE_FUSED=$r RAGK_DECODE_NORM_FUSED=$n RAGK_DECODE_TIMING=1 timeout -k 10 200 python3 -u tools/decode_anatomy.py ${DA_BS:-32 1} > gpurun_out/da_$r$n.log 2>&1 || exit $?
  grep "^B=" gpurun_out/da_$r$n.log
done
