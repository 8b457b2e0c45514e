"""Decode-step anatomy of the Llama-3.1-8B engine (random init, bf16) at batch B with ~5.2k-token
contexts (the bench's RAG prompts): wall ms per decode step from the engine (hipGraph + async
decode) and, under `rocprofv3 --kernel-trace --stats`, the per-kernel split.

  python tools/decode_anatomy.py 1 32          # batch sizes
  DA_PROMPT=5200 DA_STEPS=64 ...
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


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
        # pure GPU time of the captured decode step: back-to-back replays of the B-bucket graph
        # (stale inputs are fine: same shapes and context lengths), no host work in between
        e = eng.graphs.get(B)
        if e is not None and e["graph"] is not None:
            e["graph"].replay()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(20):
                e["graph"].replay()
            torch.cuda.synchronize()
            print("B=%d graph replay only: %.3f ms/step" % (B, (time.perf_counter() - t0) / 20 * 1e3), flush=True)
        del eng
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
