"""Decode-step anatomy of the Llama-3.1-8B engine (random init, bf16) at batch B with ~5.2k-token
contexts (the bench's RAG prompts): wall ms per decode step from the engine (hipGraph + async
decode) and, under `rocprofv3 --kernel-trace --stats`, the per-kernel split.

  python tools/decode_anatomy.py 1 32          # batch sizes
  DA_PROMPT=5200 DA_STEPS=64 ...

"graph replay only" replays the step's graph back to back from the engine's metadata at mid-run (DA_MID,
default DA_STEPS / 2), so every row is live.
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def replay_probe(eng, B, mid):
    """Back-to-back replays of the B-bucket graph from the engine's current (mid-run) metadata: the GPU time
    of one decode step with no host work in between; DA_REPLAY_MODES=h2d,d2h,both,adv,sync,pipe,pipe_copy add
    the engine's per-step copies / waits around the replays."""
    e = eng.graphs.get(B)
    if e is None or e["graph"] is None:
        return
    pk = e["packed"]
    live = int((pk[3 * B:4 * B] > 1).sum())
    e["graph"].replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(20):
        e["graph"].replay()
    torch.cuda.synchronize()
    print("B=%d graph replay only (after %d steps, %d live rows): %.3f ms/step" % (
        B, mid, live, (time.perf_counter() - t0) / 20 * 1e3), flush=True)
    pin = torch.empty(pk.numel(), dtype=torch.int32, pin_memory=True)
    pin.copy_(pk.cpu())
    tok_host = torch.empty(e["out"].numel(), dtype=torch.int32, pin_memory=True)
    # adv: every replay advances each row by one token (positions, KV-append slots, kv_lens), as the
    # engine's steps do; sync: the host waits for every replay before launching the next
    base = pin.clone()
    prev_ev = None
    for mode in [m for m in os.environ.get("DA_REPLAY_MODES", "").split(",") if m]:
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for it in range(20):
            if mode in ("h2d", "both", "pipe_copy"):
                pk.copy_(pin.to(pk.device, non_blocking=True), non_blocking=True)
            if mode == "adv":
                stg = torch.empty_like(pin).pin_memory()
                stg.copy_(base)
                stg[B:4 * B] += it + 1  # pos, slots, kv_lens (the rows stay inside their last block)
                pk.copy_(stg.to(pk.device, non_blocking=True), non_blocking=True)
            e["graph"].replay()
            if mode in ("d2h", "both"):
                tok_host.copy_(e["out"], non_blocking=True)
                torch.cuda.Event().record()
            if mode == "sync":
                torch.cuda.current_stream().synchronize()
            if mode in ("pipe", "pipe_copy"):  # the engine's pipeline: wait for the PREVIOUS replay
                if mode == "pipe_copy":
                    tok_host.copy_(e["out"], non_blocking=True)
                ev = torch.cuda.Event()
                ev.record()
                if it:
                    prev_ev.synchronize()
                prev_ev = ev
        torch.cuda.synchronize()
        print("B=%d graph replay + %s: %.3f ms/step" % (B, mode, (time.perf_counter() - t0) / 20 * 1e3), flush=True)
    pk.copy_(base.to(pk.device))  # the engine continues from its own metadata
    torch.cuda.synchronize()


def main():
    from rag_llm_k8s_amd import _build
    from rag_llm_k8s_amd.engine.llm_engine import LLMEngine, SamplingParams
    from rag_llm_k8s_amd.models import llama as L

    _build.build_all()
    Bs = [int(a) for a in sys.argv[1:]] or [1, 32]
    plen = int(os.environ.get("DA_PROMPT", "5200"))
    steps = int(os.environ.get("DA_STEPS", "64"))
    cfg = L.llama31_8b()
    dev = "cuda:0"
    w = L.LlamaWeights.random(cfg, dev, seed=0)
    m = L.LlamaModel(cfg, w, dev, max_positions=8192)
    # DA_NT="0,1,0,1": alternate non-temporal K/V loads in the decode attention (native.DECODE_NT_MIN_BH)
    nts = [t for t in os.environ.get("DA_NT", "").split(",") if t] or [None]
    # DA_PAIR="128,64,...": tile rows of the SiLU*up stream GEMM (ragk_gemm_stream_set_pair_rows)
    pairs = [int(t) for t in os.environ.get("DA_PAIR", "").split(",") if t] or [None]
    # DA_NATIVE="NAME:v1,v2,...": alternate an integer policy global of ops/native.py (e.g.
    # STREAM_PART_MIN_M:1,17,1,17 or STREAM_MAX_ROWS:200000,32768)
    nat_name, nat_vals = None, [None]
    if os.environ.get("DA_NATIVE"):
        nat_name, vals = os.environ["DA_NATIVE"].split(":")
        nat_vals = [int(v) for v in vals.split(",")]
    # DA_LLAMA="NAME:v1,v2,...": alternate an integer policy global of models/llama.py
    ll_name, ll_vals = None, [None]
    if os.environ.get("DA_LLAMA"):
        ll_name, vals = os.environ["DA_LLAMA"].split(":")
        ll_vals = [int(v) for v in vals.split(",")]
    runs = [(B, nt, nv, pr, lv) for lv in ll_vals for pr in pairs for nv in nat_vals for nt in nts for B in Bs]
    from rag_llm_k8s_amd.ops import _lib, native
    for B, nt, nv, pr, lv in runs:
        if lv is not None:
            setattr(L, ll_name, lv)
            print("-- llama.%s = %d" % (ll_name, lv), flush=True)
        if pr is not None:
            _lib.lib().ragk_gemm_stream_set_pair_rows(pr)
            print("-- stream pair rows %d" % pr, flush=True)
        if nv is not None:
            setattr(native, nat_name, nv)
            print("-- native.%s = %d" % (nat_name, nv), flush=True)
        if nt is not None:
            native.DECODE_NT_MIN_BH = 1 if nt == "1" else 1 << 30
            print("-- decode attention nt %s" % nt, flush=True)
        eng = LLMEngine(m, num_blocks=B * 128 + 16, max_batch=B, max_prefill_tokens=32768, max_model_len=8192,
                        eos_ids=cfg.eos_token_id, graph_buckets=[B])
        eng.warmup_graphs([B])
        g = torch.Generator().manual_seed(B)
        p = SamplingParams(max_new_tokens=steps + 1, temperature=0.7, top_p=0.9, top_k=50, ignore_eos=True)
        for i in range(B):
            eng.add_request(torch.randint(3, cfg.vocab_size, (plen,), generator=g).tolist(), p, seed=i)
        while any(s.computed < len(s.prompt) for s in eng.running) or eng.waiting:
            eng.step()
        torch.cuda.synchronize()
        # DA_SLEEP=s: idle this long between the prefill and the decode steps (does the decode rate depend on
        # how recently the GPU ran the MFMA-bound prefill? power / clock state)
        if float(os.environ.get("DA_SLEEP", "0")) > 0:
            time.sleep(float(os.environ["DA_SLEEP"]))
        d0, n0 = eng.stats["decode_s"], eng.stats["decode_steps"]
        # the graph is replayed from a MID-RUN state: at the end of a run the packed metadata is the last step's,
        # whose batch has shrunk (sequences prefilled in earlier chunks rode along in the mixed prefill steps
        # and finish first), so an end-of-run replay streams only those rows' KV (a round-6 finding: the
        # "graph replay only" number of earlier rounds was a 7-row step at B = 32)
        mid = int(os.environ.get("DA_MID", str(max(1, steps // 2))))
        for _ in range(mid):
            eng.step()
        torch.cuda.synchronize()
        replay_probe(eng, B, mid)
        t0 = time.perf_counter()
        eng.run_until_done()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        n = eng.stats["decode_steps"] - n0
        print("B=%d ctx=%d: %d decode steps, %.3f ms/step (engine decode_s %.3f ms/step), %.0f tok/s" % (
            B, plen, n, dt / n * 1e3, (eng.stats["decode_s"] - d0) / n * 1e3, B * n / dt), flush=True)
        if eng._timing:  # RAGK_DECODE_TIMING=1: GPU time of each captured step, in situ
            seq = [a.elapsed_time(b) for a, b in eng._timing[-n:]]
            ts = sorted(seq)
            print("B=%d in-situ graph time: median %.3f ms, min %.3f, max %.3f" % (
                B, ts[len(ts) // 2], ts[0], ts[-1]), flush=True)
            w = max(1, len(seq) // 8)  # in order: does the step time drift after the prefill?
            print("B=%d in-situ graph time by window of %d steps: %s" % (B, w, " ".join(
                "%.3f" % (sum(seq[i:i + w]) / len(seq[i:i + w])) for i in range(0, len(seq), w))), flush=True)
            eng._timing.clear()
        del eng
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
