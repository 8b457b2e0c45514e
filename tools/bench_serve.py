#!/usr/bin/env python
"""Served-path benchmark: what a user of the reference's `POST /generate` sees.

Every request goes through the real HTTP stack -- a threaded Werkzeug server running
`create_app(service)` -> /generate -> MicroBatcher (embed + HBM L2 top-k) -> prompt build ->
EngineLoop (continuous batching, mixed prefill+decode steps, hipGraph decode) -> answer --
exactly the reference's call path (/root/reference/llm/rag.py:146-181, web/app.py:12-13), on the
BASELINE config-2 workload (Llama-3.1-8B random init, bf16, MiniLM-shaped embedder, 10k-chunk
FlatL2, top-4 context, 150 new tokens, EOS ignored so every answer has 150 tokens).

Modes (both by default):
  * C=1: one request at a time (closed loop) -> single-query latency p50/p99, TTFT, TPOT;
  * Poisson: open-loop arrivals at `--rate` requests/s for `--duration` seconds -> latency,
    TTFT and TPOT percentiles and the achieved generated tokens/s.
TTFT / TPOT come from the server's per-request spans ("queue+prefill", "decode"; debug=true).
Writes one JSON object (stdout and --json-out).
"""
import argparse
import http.client
import json
import os
import random
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def pct(xs, p):
    xs = sorted(xs)
    if not xs:
        return None
    k = (len(xs) - 1) * p / 100.0
    f = int(k)
    c = min(f + 1, len(xs) - 1)
    return round(xs[f] + (xs[c] - xs[f]) * (k - f), 2)


def post(port, prompt, timeout=600):
    c = http.client.HTTPConnection("127.0.0.1", port, timeout=timeout)
    body = json.dumps({"prompt": prompt, "debug": True})
    t0 = time.perf_counter()
    c.request("POST", "/generate", body=body, headers={"Content-Type": "application/json"})
    r = c.getresponse()
    data = r.read()
    dt = time.perf_counter() - t0
    c.close()
    if r.status != 200:
        raise RuntimeError("HTTP %d: %s" % (r.status, data[:200]))
    j = json.loads(data)
    tm = j.get("timings_ms", {})
    gen = j.get("generated_tokens", 0)
    dec = tm.get("decode", 0.0)
    return dict(latency_ms=dt * 1e3, ttft_ms=tm.get("queue+prefill"), tpot_ms=dec / max(1, gen - 1),
                gen=gen, prompt_tokens=j.get("prompt_tokens"), retrieve_ms=tm.get("embed", 0) + tm.get("search", 0))


def summarize(rs, wall=None):
    out = {"requests": len(rs)}
    for k in ("latency_ms", "ttft_ms", "tpot_ms"):
        v = [r[k] for r in rs if r.get(k) is not None]
        out[k] = {"p50": pct(v, 50), "p90": pct(v, 90), "p99": pct(v, 99), "mean": round(sum(v) / len(v), 2) if v else None}
    out["prompt_tokens_mean"] = round(sum(r["prompt_tokens"] for r in rs) / len(rs), 1) if rs else None
    if wall:
        out["gen_tokens_per_s"] = round(sum(r["gen"] for r in rs) / wall, 1)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="8b", choices=["8b", "tiny"])
    ap.add_argument("--embedder", default="minilm")
    ap.add_argument("--chunks", type=int, default=10000)
    ap.add_argument("--max-new-tokens", type=int, default=150)
    ap.add_argument("--max-batch", type=int, default=64)
    ap.add_argument("--max-prefill-tokens", type=int, default=32768,
                    help="prefill budget per (mixed) engine step: bounds how long a step can stall decoding requests")
    ap.add_argument("--mixed-prefill-tokens", type=int, default=0,
                    help="prompt tokens a step carrying decode rows may take (engine mixed_prefill_tokens; 0 = off)")
    ap.add_argument("--poisson-configs", default=None,
                    help="comma list of mixed:max prefill budgets (e.g. 0:8192,2048:32768): the Poisson phase once "
                         "per pair on the same server (default: the two flags above)")
    ap.add_argument("--c1", type=int, default=20, help="sequential single requests (0 = skip)")
    ap.add_argument("--rate", type=float, default=8.0, help="Poisson arrival rate, requests/s (0 = skip)")
    ap.add_argument("--duration", type=float, default=30.0, help="seconds of Poisson arrivals")
    ap.add_argument("--json-out", default=None)
    a = ap.parse_args()

    import logging

    import torch
    from werkzeug.serving import make_server

    logging.getLogger("werkzeug").setLevel(logging.WARNING)  # no per-request access log lines

    from rag_llm_k8s_amd import _build
    from rag_llm_k8s_amd.server.app import create_app
    from rag_llm_k8s_amd.utils.workload import build_workload, make_queries

    _build.build_all()
    configs = ([tuple(int(v) for v in c.split(":")) for c in a.poisson_configs.split(",")] if a.poisson_configs
               else [(a.mixed_prefill_tokens, a.max_prefill_tokens)])
    dev = "cuda:0" if torch.cuda.is_available() else "cpu"
    t0 = time.time()
    wl = build_workload(model=a.model, embedder=a.embedder, n_chunks=a.chunks, retrieve_k=4, context_k=4,
                        max_new_tokens=a.max_new_tokens, max_batch=a.max_batch,
                        max_prefill_tokens=max(c[1] for c in configs),
                        device=dev, seed=0, use_graphs=dev.startswith("cuda"), start_threads=True, ignore_eos=True,
                        mixed_prefill_tokens=configs[0][0],
                        **({"word_vocab": 20000, "chunk_words": 120} if a.model == "tiny" else {}))
    svc = wl.svc
    svc.engine.warmup_graphs() if dev.startswith("cuda") else None
    srv = make_server("127.0.0.1", 0, create_app(svc), threaded=True)
    port = srv.server_port
    th = threading.Thread(target=srv.serve_forever, daemon=True)
    th.start()
    setup_s = time.time() - t0
    qs = make_queries(wl.wm, 4096, seed=7)
    qi = iter(qs)
    for _ in range(3):  # warm the HTTP path, the batcher and every kernel once
        post(port, next(qi))
    res = {"bench": "served /generate path (Flask -> MicroBatcher -> EngineLoop)", "device": dev,
           "config": {"model": "Llama-3.1-8B-Instruct" if a.model == "8b" else "llama-tiny",
                      "embedder": "all-MiniLM-L6-v2", "index": "FlatL2 %d vectors" % a.chunks, "retrieve_k": 4,
                      "context_k": 4, "max_new_tokens": a.max_new_tokens, "max_prefill_tokens": a.max_prefill_tokens,
                      "poisson_configs": ["%d:%d" % c for c in configs], "max_batch": a.max_batch, "dtype": "bf16"},
           "data": "synthetic (random-init weights; Zipfian pseudo-English corpus)", "setup_s": round(setup_s, 1)}
    if a.c1:
        rs = [post(port, next(qi)) for _ in range(a.c1)]
        res["c1"] = summarize(rs)
        print("C=1: %s" % json.dumps(res["c1"]), flush=True)
    for bi, (budget, maxp) in enumerate(configs if a.rate > 0 else []):
        # between runs the engine is idle; both are read per step (LLMEngine._admit)
        svc.engine.mixed_prefill_tokens, svc.engine.max_prefill_tokens = budget, maxp
        rng = random.Random(11)
        out, lock, threads = [], threading.Lock(), []

        def fire(q):
            try:
                r = post(port, q)
            except Exception as e:  # counted, not fatal
                r = {"error": str(e)}
            with lock:
                out.append(r)

        tstart = time.perf_counter()
        t = 0.0
        while t < a.duration:
            now = time.perf_counter() - tstart
            if t > now:
                time.sleep(t - now)
            th_ = threading.Thread(target=fire, args=(next(qi),), daemon=True)
            th_.start()
            threads.append(th_)
            t += rng.expovariate(a.rate)
        for th_ in threads:
            th_.join()
        wall = time.perf_counter() - tstart
        ok = [r for r in out if "error" not in r]
        s = summarize(ok, wall)
        s.update(rate_rps=a.rate, duration_s=a.duration, errors=len(out) - len(ok),
                 offered_tokens_per_s=round(a.rate * a.max_new_tokens, 1), mixed_prefill_tokens=budget,
                 max_prefill_tokens=maxp)
        res["poisson" if bi == 0 else "poisson_%d_%d" % (budget, maxp)] = s
        print("Poisson %.1f/s, mixed %d max %d: %s" % (a.rate, budget, maxp, json.dumps(s)), flush=True)
    res["engine"] = {k: (round(v, 3) if isinstance(v, float) else v) for k, v in svc.engine.stats.items()}
    line = json.dumps(res)
    print(line, flush=True)
    if a.json_out:
        with open(a.json_out, "w") as f:
            f.write(line + "\n")
    srv.shutdown()
    svc.shutdown()


if __name__ == "__main__":
    main()
