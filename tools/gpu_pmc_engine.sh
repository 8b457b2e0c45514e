#!/bin/bash
# PMC passes (one rocprofv3 run per counter set, kernel-trace only) over the persistent decode tail
# (tools/mlp_engine_bench.py, 4 layers) and the separate kernels it replaces. Summary: gpurun_out/pmc_engine.txt
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmce
P1="FETCH_SIZE GRBM_GUI_ACTIVE"
P2="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_LDS TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
timeout -s KILL 150 rocprofv3 --pmc $P1 --kernel-trace --output-format csv -d gpurun_out/pmce/p1 -o run -- python3 tools/mlp_engine_bench.py 4 5 > gpurun_out/pmce/p1.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --pmc $P2 --kernel-trace --output-format csv -d gpurun_out/pmce/p2 -o run -- python3 tools/mlp_engine_bench.py 4 5 > gpurun_out/pmce/p2.log 2>&1
rc=$?
python3 - <<'PY' > gpurun_out/pmc_engine.txt 2>&1
import csv, glob, collections
for p in ("p1", "p2"):
    for f in glob.glob("gpurun_out/pmce/%s/**/*counter_collection.csv" % p, recursive=True):
        acc = collections.defaultdict(lambda: collections.defaultdict(list))
        for r in csv.DictReader(open(f)):
            k = r.get("Kernel_Name", "")
            name = "mlp_engine" if "mlp_engine" in k else ("gemm_stream" if "gemm_stream" in k else
                   ("gemm_skinny" if "gemm_skinny" in k else ("add_partials" if "add_partials" in k else None)))
            if name:
                acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
        for name, cs in acc.items():
            print(p, name, " ".join("%s=%.4g" % (c, sum(v) / len(v)) for c, v in sorted(cs.items())))
PY
cat gpurun_out/pmc_engine.txt
exit $rc
