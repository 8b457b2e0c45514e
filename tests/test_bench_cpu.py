"""bench.py contract on the CPU (gloo) rehearsal: one JSON line from rank 0 with the driver's keys, and
for N > 1 data-parallel runs the TP=N C=1 latency appended after the headline (tiny model)."""
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _bench(n, *extra, env_extra=None, rc=0):
    args = ["--gpus", str(n), "--model", "tiny", "--embedder", "tiny", "--chunks", "48", "--chunk-words", "60",
            "--concurrency", "2", "--max-new-tokens", "3", "--steps", "1", "--warmup", "0", "--c1", "1"] + list(extra)
    if n == 1:
        cmd = [sys.executable, "bench.py"] + args
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n),
               "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py"] + args
    env = dict(os.environ, OMP_NUM_THREADS="2", CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="", **(env_extra or {}))
    # stdout and stderr apart: a rank's stderr message written while rank 0 prints its JSON line could
    # otherwise land inside that line (seen with the injected TP-phase hang)
    r = subprocess.run(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=600)
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert r.returncode == rc and len(lines) == 1, (r.returncode, r.stdout[-2000:], r.stderr[-2000:])
    return json.loads(lines[0])


def test_bench_two_ranks_appends_tp_c1():
    res = _bench(2, "--c1-tp", "1")
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in res
    assert res["n_gpus"] == 2 and res["config"]["parallelism"] == "dp2" and res["value"] > 0
    assert res["c1_tp_degree"] == 2 and res["p50_latency_c1_tp_ms"] > 0, res
    assert "c1_tp_error" not in res


def test_bench_one_rank_tp_line_is_the_headline_c1():
    res = _bench(1)
    assert res["c1_tp_degree"] == 1 and res["p50_latency_c1_tp_ms"] == res["p50_latency_c1_ms"]


def test_bench_tp_phase_hang_exits_nonzero():
    """A hung cross-device phase (injected stall > the watchdog bound) still prints the headline line, but
    the run's exit status says it failed (bench.py EXIT_TP_HANG = 3; torchrun reports a failed child as 1)."""
    res = _bench(2, "--c1-tp", "1", "--c1-tp-timeout", "5", env_extra={"RAGK_FAULTS": "bench_tp_hang_s=60"}, rc=1)
    assert res["value"] > 0 and res["p50_latency_c1_tp_ms"] is None
    assert res["c1_tp_error"].startswith("timeout after 5")
