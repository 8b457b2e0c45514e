"""Host-side profile (cProfile) of the engine's decode loop at batch B (Llama-3.1-8B random init,
5.2k-token contexts): where the time between graph replays goes when the engine step is slower than
a bare replay of its decode graph (tools/decode_anatomy.py prints both)."""
import cProfile
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from rag_llm_k8s_amd import _build
    from rag_llm_k8s_amd.engine.llm_engine import LLMEngine, SamplingParams
    from rag_llm_k8s_amd.models import llama as L

    _build.build_all()
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    plen, steps = int(os.environ.get("DA_PROMPT", "5200")), int(os.environ.get("DA_STEPS", "48"))
    cfg = L.llama31_8b()
    w = L.LlamaWeights.random(cfg, "cuda:0", seed=0)
    m = L.LlamaModel(cfg, w, "cuda:0", max_positions=8192)
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
    pr = cProfile.Profile()
    t0 = time.perf_counter()
    pr.enable()
    eng.run_until_done()
    pr.disable()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print("B=%d: %.3f ms/step over %d steps" % (B, dt / steps * 1e3, steps), flush=True)
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(25)
    st.sort_stats("cumulative").print_stats(25)


if __name__ == "__main__":
    main()
