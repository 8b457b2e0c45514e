"""Why is an engine decode step slower than a bare replay of its graph? Replays the captured
B-bucket decode graph of a Llama-3.1-8B engine (5.2k-token contexts) under different host patterns:
  E0 back-to-back replays; E1 replay + full sync each step; E2 + the per-step H2D input copy and D2H
  token copy; E3 the engine's pipeline (sync on the previous step's event) with those copies."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from rag_llm_k8s_amd import _build
    from rag_llm_k8s_amd.engine.llm_engine import LLMEngine, SamplingParams
    from rag_llm_k8s_amd.models import llama as L

    _build.build_all()
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    cfg = L.llama31_8b()
    w = L.LlamaWeights.random(cfg, "cuda:0", seed=0)
    m = L.LlamaModel(cfg, w, "cuda:0", max_positions=8192)
    eng = LLMEngine(m, num_blocks=B * 128 + 16, max_batch=B, max_prefill_tokens=32768, max_model_len=8192,
                    eos_ids=cfg.eos_token_id, graph_buckets=[B])
    eng.warmup_graphs([B])
    g = torch.Generator().manual_seed(B)
    p = SamplingParams(max_new_tokens=int(os.environ.get("DPP_TOKENS", "8")), temperature=0.7, top_p=0.9, top_k=50, ignore_eos=True)
    for i in range(B):
        eng.add_request(torch.randint(3, cfg.vocab_size, (5200,), generator=g).tolist(), p, seed=i)
    while any(s.computed < len(s.prompt) for s in eng.running) or eng.waiting:
        eng.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    n0 = eng.stats["decode_steps"]
    eng.run_until_done()
    torch.cuda.synchronize()
    n = eng.stats["decode_steps"] - n0
    print("engine decode: %d steps, %.3f ms/step" % (n, (time.perf_counter() - t0) / max(1, n) * 1e3), flush=True)
    if eng._timing:
        tl = eng._timing
        inside = [a.elapsed_time(b) for a, b in tl]
        gaps = [tl[i][1].elapsed_time(tl[i + 1][0]) for i in range(len(tl) - 1)]
        print("  in-situ graph time: median %.3f ms (min %.3f, max %.3f); end->next start gap: median %.3f ms, max %.3f"
              % (np.median(inside), min(inside), max(inside), np.median(gaps), max(gaps)), flush=True)
        print("  per-step graph ms:", " ".join("%.2f" % x for x in inside[:60]), flush=True)
    e = eng.graphs[B]
    packed, out = e["packed"], e["out"]
    host_in = torch.from_numpy(packed.cpu().numpy().copy()).pin_memory()
    host_out = torch.empty(B, dtype=torch.int32).pin_memory()
    st = torch.cuda.current_stream()
    N = 20

    def bench(name, body):
        body(2)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        body(N)
        torch.cuda.synchronize()
        print("%-44s %.3f ms/step" % (name, (time.perf_counter() - t0) / N * 1e3), flush=True)

    def e0(n):
        for _ in range(n):
            e["graph"].replay()

    def e1(n):
        for _ in range(n):
            e["graph"].replay()
            torch.cuda.synchronize()

    def e2(n):
        for _ in range(n):
            packed.copy_(host_in, non_blocking=True)
            e["graph"].replay()
            host_out.copy_(out, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(st)

    def e3(n):
        prev = None
        for _ in range(n):
            packed.copy_(host_in, non_blocking=True)
            e["graph"].replay()
            host_out.copy_(out, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(st)
            if prev is not None:
                prev.synchronize()
            prev = ev

    def e4(n):  # E3 with the H2D staged through a fresh device tensor, as _h2d_i32 does
        prev = None
        for _ in range(n):
            packed.copy_(host_in.to(packed.device, non_blocking=True), non_blocking=True)
            e["graph"].replay()
            host_out.copy_(out, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(st)
            if prev is not None:
                prev.synchronize()
            prev = ev

    bench("E0 back-to-back replay", e0)
    for rep in range(4):  # sustained: is a long run slower (power / clock management)?
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e0(100)
        torch.cuda.synchronize()
        print("E0 sustained block %d (100 steps)              %.3f ms/step" % (rep, (time.perf_counter() - t0) / 100 * 1e3),
              flush=True)
    bench("E1 replay + sync", e1)
    bench("E2 + H2D in / D2H out copies", e2)
    bench("E3 engine pipeline (prev-event sync)", e3)
    bench("E4 E3 + staged H2D (fresh device tensor)", e4)


if __name__ == "__main__":
    main()
