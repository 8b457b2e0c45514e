cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests/test_kernels_gpu.py -q -rf -p no:cacheprovider > gpurun_out/kt1.log 2>&1
echo "pytest exit $?" >> gpurun_out/kt1.log
tail -40 gpurun_out/kt1.log
