cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
for mb in 256 512 1024; do
  RAGK_PART_MIN_BLOCKS=$mb timeout -k 10 400 python bench.py --steps 3 --warmup 1 > gpurun_out/ab_$mb.log 2>&1 || exit 1
  python -c "import json,sys; d=json.loads(open('gpurun_out/ab_$mb.log').read().strip().splitlines()[-1]); print('$mb', d['value'], d['engine']['decode_s'], d['engine']['prefill_s'])"
done
