"""Decode sampler micro-bench on one GPU: top-k candidate selection + sampling over a Llama-3 vocab
(128256 fp32 logits per row), at the chunkings the engine picks (llm_engine.SMALL_BATCH_TOPK_*) and
the 7-chunk radix path for comparison. Prints one JSON line per case: us per call of back-to-back
launches from Python (median of 5 x 200; host-bound for one-block kernels) and both_dev_us, the device
time of one (top-k, sample) pair from a captured hipGraph."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rag_llm_k8s_amd.ops import native as N  # noqa: E402


def timed(fn, iters=200, reps=5):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    out = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(iters):
            fn()
        b.record()
        b.synchronize()
        out.append(a.elapsed_time(b) * 1e3 / iters)
    return sorted(out)[len(out) // 2]


def main():
    V, K = 128256, 64
    for B in (1, 4, 32):
        logits = torch.randn(B, V, device="cuda") * 3
        temps = torch.full((B,), 0.7, device="cuda")
        ks = torch.full((B,), 50, dtype=torch.int32, device="cuda")
        ps = torch.full((B,), 0.9, device="cuda")
        seeds = torch.arange(B, dtype=torch.int64, device="cuda")
        steps = torch.zeros(B, dtype=torch.int32, device="cuda")
        for chunks in sorted({N.topk_chunks(V, K, 512), min(V // 4096, 2048 // K, 64)}):
            cv, ci = N.topk_candidates(logits, K, chunks=chunks)
            tok = torch.empty(B, dtype=torch.int32, device="cuda")
            t_topk = timed(lambda: N.topk_candidates(logits, K, chunks=chunks, cand_v=cv, cand_i=ci))
            t_samp = timed(lambda: N.sample_candidates(cv, ci, temps, ks, ps, seeds, steps, out_tok=tok, list_len=K))
            t_both = timed(lambda: (N.topk_candidates(logits, K, chunks=chunks, cand_v=cv, cand_i=ci),
                                    N.sample_candidates(cv, ci, temps, ks, ps, seeds, steps, out_tok=tok,
                                                        list_len=K)))
            # device time: 20 (top-k, sample) pairs captured in one hipGraph, replayed back to back
            g = torch.cuda.CUDAGraph()
            st = torch.cuda.Stream()
            st.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(st), torch.cuda.graph(g, stream=st):
                for _ in range(20):
                    N.topk_candidates(logits, K, chunks=chunks, cand_v=cv, cand_i=ci)
                    N.sample_candidates(cv, ci, temps, ks, ps, seeds, steps, out_tok=tok, list_len=K)
            torch.cuda.current_stream().wait_stream(st)
            t_dev = timed(g.replay, iters=5, reps=5) / 20
            print(json.dumps({"B": B, "chunks": chunks, "topk_us": round(t_topk, 2), "sample_us": round(t_samp, 2),
                              "both_us": round(t_both, 2), "both_dev_us": round(t_dev, 2)}), flush=True)


if __name__ == "__main__":
    main()
