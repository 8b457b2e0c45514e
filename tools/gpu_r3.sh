#!/bin/bash
# Round-3 GPU steps on one MI355X (run via gpurun). STEP selects: search | kernels | suite | bench |
# prof. Every GPU step has its own time limit; a step that dies of anything but test failures ends the call.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
STEP=${STEP:-search}
ok() { rc=$1; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "step failed rc=$rc"; exit $rc; fi; }
case ",$STEP," in *,search,*)
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_ivf_gpu.py tests/test_canary_gpu.py -k "l2_search or ivf or kmeans or bounds or topk or sampl" -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_search.log 2>&1
rc=$?; echo "search tests rc=$rc"; tail -15 gpurun_out/pytest_search.log; ok $rc
timeout -k 10 300 python -u tools/search_bench.py > gpurun_out/search_bench.log 2>&1
rc=$?; echo "search bench rc=$rc"; cat gpurun_out/search_bench.log; ok $rc
timeout -k 10 200 python -u tools/sampler_bench.py > gpurun_out/sampler_bench.log 2>&1
rc=$?; echo "sampler bench rc=$rc"; grep '^{' gpurun_out/sampler_bench.log; ok $rc
;; esac
case ",$STEP," in *,part,*)
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_canary_gpu.py -k "gemm_part or silu" -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_part.log 2>&1
rc=$?; echo "part tests rc=$rc"; tail -8 gpurun_out/pytest_part.log; ok $rc
DG_TP=8 timeout -k 10 300 python -u tools/bench_decode_gemm.py 1 4 32 > gpurun_out/decode_gemm_tp8.log 2>&1
rc=$?; echo "tp8 gemm bench rc=$rc"; grep "^M=" gpurun_out/decode_gemm_tp8.log; ok $rc
;; esac
case ",$STEP," in *,siluab,*)
for v in tp 1; do
RAGK_DECODE_SILU_FUSED=$v RAGK_DECODE_TIMING=1 DA_STEPS=48 timeout -k 10 400 python -u tools/decode_anatomy.py 1 4 > gpurun_out/siluab_$v.log 2>&1
rc=$?; echo "silu fused=$v rc=$rc"; grep "^B=" gpurun_out/siluab_$v.log; ok $rc
done
;; esac
case ",$STEP," in *,tp,*)
timeout -k 10 900 python -u -m pytest tests/test_ipc_allreduce_gpu.py tests/test_tp_gpu.py -v --timeout 400 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_tp.log 2>&1
rc=$?; echo "tp tests rc=$rc"; tail -15 gpurun_out/pytest_tp.log; ok $rc
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "attn_decode or gemm_part_merge" -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_attn_tp.log 2>&1
rc=$?; echo "attn tp-layout tests rc=$rc"; tail -6 gpurun_out/pytest_attn_tp.log; ok $rc
;; esac
case ",$STEP," in *,probe,*)
timeout -k 10 400 python -u tools/tp_decode_probe.py 1 32 > gpurun_out/tp_probe.log 2>&1
rc=$?; echo "probe rc=$rc"; cat gpurun_out/tp_probe.log | grep -v amdgpu.ids; ok $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_tp -o tp -- python3 tools/tp_decode_probe.py 1 > gpurun_out/tp_probe_prof.log 2>&1
rc=$?; echo "probe prof rc=$rc"; rm -f gpurun_out/prof_tp/*kernel_trace.csv
python tools/rocprof_summary.py gpurun_out/prof_tp/tp_kernel_stats.csv 40 > gpurun_out/tp_probe_summary.txt 2>&1; head -45 gpurun_out/tp_probe_summary.txt; ok $rc
;; esac
case ",$STEP," in *,probeab,*)
for mt in ${PAB_TILES:-4 2 1}; do
RAGK_DECODE_MIN_TILES=$mt timeout -k 10 300 python -u tools/tp_decode_probe.py ${PAB_B:-1 32} > gpurun_out/tp_probe_mt$mt.log 2>&1
rc=$?; echo "probe min_tiles=$mt rc=$rc"; grep "^B=" gpurun_out/tp_probe_mt$mt.log; ok $rc
done
;; esac
case ",$STEP," in *,normt,*)
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_canary_gpu.py -k "partials or norm" -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_normt.log 2>&1
rc=$?; echo "norm tests rc=$rc"; tail -4 gpurun_out/pytest_normt.log; ok $rc
;; esac
case ",$STEP," in *,order,*)
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_canary_gpu.py -k "prefill" -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_order.log 2>&1
rc=$?; echo "prefill tests rc=$rc"; tail -4 gpurun_out/pytest_order.log; ok $rc
for cfg in "5215:0" "5400,5400,5400,5400,5400,5400:0,0,0,0,0,0" "2048:3072"; do
AP_LENS=${cfg%%:*} AP_CTX=${cfg##*:} AP_MODES=10 AP_ORDERS=1,0 AP_STAMP=0 AP_ROUNDS=7 timeout -k 10 200 python -u tools/attn_pp_ab.py > gpurun_out/order_ab.log 2>&1
rc=$?; echo "order A/B $cfg rc=$rc"; grep "^lens" gpurun_out/order_ab.log; ok $rc
done
;; esac
case ",$STEP," in *,searchprof,*)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_search -o s -- python3 tools/search_bench.py > gpurun_out/search_prof.log 2>&1
rc=$?; echo "search prof rc=$rc"; rm -f gpurun_out/prof_search/*kernel_trace.csv
python tools/rocprof_summary.py gpurun_out/prof_search/s_kernel_stats.csv 20 > gpurun_out/search_prof_summary.txt 2>&1; head -20 gpurun_out/search_prof_summary.txt; grep '^{' gpurun_out/search_prof.log; ok $rc
;; esac
case ",$STEP," in *,suite,*)
timeout -k 10 1100 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -15 gpurun_out/pytest_gpu.log; ok $rc
;; esac
case ",$STEP," in *,bench,*)
timeout -k 10 600 python -u bench.py --steps ${BSTEPS:-3} --warmup 1 --json-out gpurun_out/bench.json > gpurun_out/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -2 gpurun_out/bench.log; ok $rc
;; esac
case ",$STEP," in *,prof,*)
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 1 --warmup 0 --c1 ${PROF_C1:-0} > gpurun_out/prof.log 2>&1
rc=$?; echo "prof rc=$rc"
rm -f gpurun_out/prof/*kernel_trace.csv
python tools/rocprof_summary.py gpurun_out/prof/run_kernel_stats.csv 40 > gpurun_out/rocprof_summary.txt 2>&1
head -30 gpurun_out/rocprof_summary.txt; ok $rc
;; esac
exit 0
