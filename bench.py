#!/usr/bin/env python
"""Headline benchmark (BASELINE.json): end-to-end RAG query p50 latency + generation tokens/s,
Llama-3.1-8B (random init, bf16), all-MiniLM-L6-v2-shaped embedder, 10k-chunk FlatL2 index
resident in HBM, retrieve top-k = 4 (all 4 go into the prompt), 150 new tokens per query.

One "step" = one wave of `--concurrency` concurrent /query requests per engine (TP group)
served end to end: batched query embedding -> HBM L2 top-k -> prompt build (reference template) ->
tokenize -> continuous-batching prefill + hipGraph decode (temperature 0.7, top-p 0.9, top-k 50,
150 tokens, EOS ignored so every request produces exactly 150 tokens) -> detokenize ->
"Chatbot:" post-processing.

Multi-GPU: one process per GPU (torchrun), weak scaling (32 concurrent queries per GPU per step).
The default layout is N data-parallel replicas (TP=1 engines, the k8s replicas behind the Service):
an 8B model plus its KV cache fits one 288 GB GPU many times over, and on this workload tensor
parallelism only adds xGMI traffic -- a TP=8 step all-reduces ~11 GB per layer-half of prefill
activations (docs/PERF_NOTES.md, "TP=8 budget"), so a TP=8 engine is comm-bound in prefill while
its per-rank decode gains do not make up for it. `--tp T` runs T-way tensor-parallel engines
(Megatron TP over xGMI: the fused peer-mapped reduction in decode, RCCL / peer-mapped all-reduces
overlapped with the next micro-batch in prefill; BASELINE config 3 is `--tp 8`), tp x dp layouts
for T < N.

value = total generated tokens of all ranks / max-over-ranks wall time of the K timed steps.
p50_latency_ms is the wave latency of a step; p50_latency_c1_ms the single-query latency (C=1,
measured after the timed steps: the reference serves one query per /generate call).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "end-to-end RAG query p50 latency + gen tokens/sec, Llama-3.1-8B top-k=4"
# exit status of a run whose headline line went out but whose TP=N C=1 phase hung / raised
EXIT_TP_HANG = 3
EXIT_TP_ERROR = 4


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--concurrency", type=int, default=None,
                    help="concurrent queries per engine (TP group) per step; default 32 x TP degree")
    ap.add_argument("--tp", type=int, default=None, help="TP degree per engine (default 1: N data-parallel replicas)")
    ap.add_argument("--dp", action="store_true", help="N data-parallel replicas (the default; kept for compatibility)")
    ap.add_argument("--model", default="8b", choices=["8b", "70b", "tiny"])
    ap.add_argument("--embedder", default="minilm", choices=["minilm", "bge-large", "bge-m3", "tiny"])
    ap.add_argument("--chunks", type=int, default=10000)
    ap.add_argument("--chunk-words", type=int, default=1000, help="words per corpus chunk (reference chunker: 1000)")
    ap.add_argument("--retrieve-k", type=int, default=4)
    ap.add_argument("--context-k", type=int, default=4)
    ap.add_argument("--max-new-tokens", type=int, default=150)
    ap.add_argument("--index", default="flat", choices=["flat", "ivf"])
    ap.add_argument("--index-vectors", type=int, default=0,
                    help="pad the index to this many vectors (config 4: 1000000) after the embedded corpus")
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp8"],
                    help="linear-layer weights: bf16 (headline) or fp8 e4m3 (BASELINE config 5)")
    ap.add_argument("--seq-parallel", action="store_true",
                    help="TP prefill with Megatron sequence parallelism (reduce-scatter/all-gather)")
    ap.add_argument("--c1", type=int, default=5,
                    help="after the timed steps: this many single queries one at a time (C=1 latency; untimed)")
    ap.add_argument("--c1-tp", type=int, default=3,
                    help="N > 1 data-parallel runs: after the headline, this many C=1 queries on ONE TP=N engine "
                         "spanning every GPU (untimed; p50_latency_c1_tp_ms, the xGMI latency path); 0 = skip")
    ap.add_argument("--c1-tp-timeout", type=float, default=float(os.environ.get("RAGK_BENCH_TP_TIMEOUT", "420")),
                    help="seconds the TP=N C=1 phase may take before the headline line is printed without it")
    ap.add_argument("--json-out", default=None)
    return ap.parse_args()


def pct(xs, p):
    xs = sorted(xs)
    if not xs:
        return None
    k = (len(xs) - 1) * p / 100.0
    f = int(k)
    c = min(f + 1, len(xs) - 1)
    return xs[f] + (xs[c] - xs[f]) * (k - f)


def tp_c1_phase(a, ctx, params):
    """C=1 latency of one TP=N engine over all N GPUs of the job (BASELINE config 3's layout), run after
    the data-parallel headline in the same process group: a TP group of every rank, the peer-mapped
    collectives over xGMI (fences on across devices), the same synthetic workload shape. Untimed for
    `value`; returns (p50 ms, ttft p50 ms, samples)."""
    import dataclasses

    import torch
    import torch.distributed as dist

    from rag_llm_k8s_amd.parallel.comm import TPComm
    from rag_llm_k8s_amd.utils.workload import build_workload, make_queries

    ranks = list(range(ctx.world))
    grp = dist.new_group(ranks)
    cgrp = dist.new_group(ranks, backend="gloo")
    tctx = dataclasses.replace(ctx, tp=ctx.world, tp_rank=ctx.rank, dp=1, dp_rank=0, tp_group=grp,
                               tp_cpu_group=cgrp, dp_group=None)
    comm = TPComm(grp, tctx.tp, tctx.tp_rank, ctx.device, cgrp)
    wl = build_workload(model=a.model, embedder=a.embedder, n_chunks=a.chunks, chunk_words=a.chunk_words,
                        retrieve_k=a.retrieve_k, context_k=a.context_k, max_new_tokens=a.max_new_tokens, max_batch=4,
                        device=ctx.device,
                        ctx=tctx, tp_comm=comm, seed=0, use_graphs=not a.no_graphs, index_type=a.index,
                        dtype=a.dtype)
    wl.svc.engine.warmup_graphs()
    lat, ttft = [], []
    for i in range(a.c1_tp + 1):  # the first query warms the TP path
        q = make_queries(wl.wm, 1, seed=888000 + i)
        o = wl.svc.generate_batch(q, params=params, seeds=[5151 + i])[0]
        if i and "_latency_s" in o:
            lat.append(o["_latency_s"] * 1e3)
            ttft.append(o["_ttft_s"] * 1e3)
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    return (round(pct(lat, 50), 1) if lat else None, round(pct(ttft, 50), 1) if ttft else None, len(lat),
            bool(comm.ipc is not None), bool(comm.ipc is not None and comm.ipc.fences))


def main():
    a = parse()
    import torch

    from rag_llm_k8s_amd import _build
    from rag_llm_k8s_amd.engine.llm_engine import SamplingParams
    from rag_llm_k8s_amd.parallel import dist as D
    from rag_llm_k8s_amd.parallel.comm import TPComm
    from rag_llm_k8s_amd.utils import faults
    from rag_llm_k8s_amd.utils.workload import build_workload, make_queries

    if a.seq_parallel:
        os.environ["RAGK_SEQ_PARALLEL"] = "1"
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != a.gpus:
        print("warning: --gpus %d but WORLD_SIZE=%d; using WORLD_SIZE" % (a.gpus, world), file=sys.stderr)
    if a.dp and a.tp not in (None, 1):
        raise SystemExit("bench.py: --dp (N data-parallel TP=1 replicas) conflicts with --tp %d" % a.tp)
    if a.tp is None:
        a.tp = 1
    if a.concurrency is None:
        a.concurrency = 32 * a.tp
    if int(os.environ.get("LOCAL_RANK", "0")) == 0:
        _build.build_all()
    ctx = D.init_distributed(tp=a.tp)
    D.barrier(ctx)
    dev = ctx.device
    comm = TPComm(ctx.tp_group, ctx.tp, ctx.tp_rank, dev, ctx.tp_cpu_group) if ctx.tp > 1 else None
    t_setup = time.time()

    def progress(msg):  # rank 0, stderr (the JSON line is the only stdout)
        if ctx.rank == 0:
            print("bench: " + msg, file=sys.stderr, flush=True)

    wl = build_workload(model=a.model, embedder=a.embedder, n_chunks=a.chunks, chunk_words=a.chunk_words,
                        retrieve_k=a.retrieve_k, context_k=a.context_k, max_new_tokens=a.max_new_tokens,
                        max_batch=a.concurrency,
                        device=dev, ctx=ctx, tp_comm=comm, seed=0, use_graphs=not a.no_graphs, index_type=a.index,
                        dtype=a.dtype, index_vectors=a.index_vectors, progress=progress)
    svc = wl.svc
    svc.engine.warmup_graphs()
    progress("graphs captured, setup %.1f s" % (time.time() - t_setup))
    params = SamplingParams(max_new_tokens=a.max_new_tokens, temperature=0.7, top_p=0.9, top_k=50, do_sample=True,
                            ignore_eos=True)
    setup_s = time.time() - t_setup

    def run_step(step_id):
        # identical queries/seeds inside a TP group, different across DP replicas and steps
        qs = make_queries(wl.wm, a.concurrency, seed=100000 * ctx.dp_rank + 1000 + step_id)
        seeds = [1000 * (step_id + 1000) + i for i in range(len(qs))]
        return svc.generate_batch(qs, params=params, seeds=seeds)

    def sync():  # the CPU plumbing rehearsal (gloo) has no device to synchronise
        if torch.cuda.is_available():
            torch.cuda.synchronize()

    for w in range(a.warmup):
        run_step(-1 - w)
        progress("warmup step %d done" % w)
    D.barrier(ctx)
    sync()
    t0 = time.perf_counter()
    lat, ttft, ptoks, gtoks, step_ms = [], [], [], [], []
    for s in range(a.steps):
        ts = time.perf_counter()
        outs = run_step(s)
        step_ms.append((time.perf_counter() - ts) * 1e3)
        for o in outs:
            if "_latency_s" in o:
                lat.append(o["_latency_s"] * 1e3)
                ttft.append(o["_ttft_s"] * 1e3)
                ptoks.append(o["_prompt_tokens"])
                gtoks.append(o["_gen_tokens"])
    sync()
    D.barrier(ctx)
    elapsed = time.perf_counter() - t0
    # single-request latency (the reference serves one query per /generate call): outside the timed
    # region, same service path, one query at a time
    c1_lat, c1_ttft = [], []
    for i in range(a.c1):
        q = make_queries(wl.wm, 1, seed=777000 + 1000 * ctx.dp_rank + i)
        o = svc.generate_batch(q, params=params, seeds=[4242 + i])[0]
        if "_latency_s" in o:
            c1_lat.append(o["_latency_s"] * 1e3)
            c1_ttft.append(o["_ttft_s"] * 1e3)
    elapsed_max = D.all_reduce_max(ctx, elapsed)
    my_tokens = sum(gtoks) if ctx.tp_rank == 0 else 0
    total_tokens = D.all_reduce_sum(ctx, float(my_tokens))
    allstats = D.all_gather_object(ctx, dict(lat=lat, ttft=ttft, ptoks=ptoks, eng=svc.engine.stats,
                                             setup=wl.timings, step_ms=step_ms, c1=c1_lat, c1_ttft=c1_ttft))
    if ctx.rank == 0:
        L = [x for s in allstats for x in s["lat"]]
        T = [x for s in allstats for x in s["ttft"]]
        P = [x for s in allstats for x in s["ptoks"]]
        value = total_tokens / elapsed_max
        par = "dp%d" % ctx.dp if ctx.tp == 1 else ("tp%d" % ctx.tp if ctx.dp == 1 else "tp%d_dp%d" % (ctx.tp, ctx.dp))
        if ctx.tp > 1 and a.seq_parallel:
            par += "_sp"
        eng = allstats[0]["eng"]
        res = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "generated tokens/s (aggregate over all GPUs)",
            "n_gpus": ctx.world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(elapsed_max / a.steps * 1e3, 2),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16" if a.dtype == "bf16" else "fp8-weights (bf16 activations/KV)",
            "data": "synthetic (random-init weights of the named architectures; Zipfian pseudo-English corpus "
                    "of %d x %d-word chunks%s; trained 128k BPE + %s tokenizers)" % (
                        a.chunks, a.chunk_words, (" + %d embedded 1000-word topical chunks" % (a.index_vectors - a.chunks)
                                   if a.index_vectors > a.chunks else ""),
                        "XLM-R SentencePiece Unigram" if a.embedder == "bge-m3" else "WordPiece"),
            "config": {
                "model": {"8b": "Llama-3.1-8B-Instruct", "70b": "Llama-3.1-70B-Instruct", "tiny": "llama-tiny"}[a.model],
                "embedder": {"minilm": "all-MiniLM-L6-v2", "bge-large": "bge-large-en-v1.5", "bge-m3": "bge-m3",
                             "tiny": "tiny"}[a.embedder],
                "index": "%s %d vectors (HBM-resident; %d embedded chunks)" % (
                    "FlatL2" if a.index == "flat" else "IVF-Flat", max(a.chunks, a.index_vectors), a.chunks),
                "retrieve_k": a.retrieve_k, "context_k": a.context_k,
                "global_batch": a.concurrency * ctx.dp,
                "seq_len": int(round(sum(P) / max(1, len(P)))),
                "max_new_tokens": a.max_new_tokens,
                "parallelism": par,
            },
            "p50_latency_ms": round(pct(L, 50), 1) if L else None,
            "p90_latency_ms": round(pct(L, 90), 1) if L else None,
            "ttft_p50_ms": round(pct(T, 50), 1) if T else None,
            "p50_latency_c1_ms": round(pct(allstats[0]["c1"], 50), 1) if allstats[0]["c1"] else None,
            "ttft_c1_p50_ms": round(pct(allstats[0]["c1_ttft"], 50), 1) if allstats[0]["c1_ttft"] else None,
            "per_gpu_tokens_per_s": round(value / ctx.world, 2),
            "engine": {k: (round(v, 3) if isinstance(v, float) else v) for k, v in eng.items()},
            "setup_s": round(setup_s, 1),
            # ingest throughput of the corpus build (tokenize + batched varlen encoder, one GPU)
            "ingest_embed_chunks_per_s": round(a.chunks / max(1e-9, allstats[0]["setup"].get("embed_s", 0.0)), 1),
        }
    else:
        res = None

    def emit(r):
        line = json.dumps(r)
        print(line, flush=True)
        if a.json_out:
            with open(a.json_out, "w") as f:
                f.write(line + "\n")

    # TP=N C=1 latency over every GPU of the job (after the headline; never changes `value`). At N = 1
    # (or when the headline engine already spans the job) the headline's own C=1 is that number.
    if ctx.tp == ctx.world or a.c1_tp <= 0:
        if res is not None:
            res["p50_latency_c1_tp_ms"] = res["p50_latency_c1_ms"] if ctx.tp == ctx.world else None
            res["c1_tp_degree"] = ctx.tp
            emit(res)
        D.shutdown(ctx)
        return
    import threading

    done = threading.Event()

    def watchdog():  # a hung cross-device phase must not cost the headline line -- nor look like success
        if not done.wait(a.c1_tp_timeout):
            if res is not None:
                res.update(p50_latency_c1_tp_ms=None, c1_tp_degree=ctx.world,
                           c1_tp_error="timeout after %.0f s" % a.c1_tp_timeout)
                emit(res)
            sys.stdout.flush()
            sys.stderr.write("bench.py: TP=%d C=1 phase hung (> %.0f s); exiting %d\n"
                             % (ctx.world, a.c1_tp_timeout, EXIT_TP_HANG))
            sys.stderr.flush()
            os._exit(EXIT_TP_HANG)  # every rank: a stuck peer never reaches the shutdown barrier

    threading.Thread(target=watchdog, daemon=True).start()
    rc = 0
    try:
        hang = faults.value("bench_tp_hang_s")  # fault injection: the TP phase stalls (tests)
        if hang:
            time.sleep(float(hang))
        p50, tt, n, ipc, fences = tp_c1_phase(a, ctx, params)
        tp_res = dict(p50_latency_c1_tp_ms=p50, ttft_c1_tp_p50_ms=tt, c1_tp_degree=ctx.world, c1_tp_queries=n,
                      c1_tp_peer_mapped=ipc, c1_tp_fences=fences)
    except Exception as e:  # the headline line still goes out, but the run's exit status reports the failure
        tp_res = dict(p50_latency_c1_tp_ms=None, c1_tp_degree=ctx.world, c1_tp_error="%s: %s" % (type(e).__name__, e))
        rc = EXIT_TP_ERROR
    done.set()
    if res is not None:
        res.update(tp_res)
        emit(res)
    if rc:
        sys.stdout.flush()
        os._exit(rc)  # peers may be stuck in the failed collective: no shutdown barrier
    D.shutdown(ctx)


if __name__ == "__main__":
    main()
