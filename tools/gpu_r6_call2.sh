cd /root/repo
timeout -k 10 300 python -u -m pytest tests/test_mlp_engine_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pt_me.log 2>&1
rc=$?; tail -15 gpurun_out/pt_me.log; [ $rc = 0 ] || exit $rc
timeout -k 10 200 python -u tools/mlp_engine_bench.py 16 20 > gpurun_out/meb.log 2>&1 || { tail -8 gpurun_out/meb.log; exit 1; }
tail -8 gpurun_out/meb.log
bash tools/gpu_decode_drift.sh
