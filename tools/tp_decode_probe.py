"""One-GPU probe of a tensor-parallel decode step: rank 0's TP shard of Llama-3.1-8B (default TP=8:
4 query heads, 1 KV head, 1792 FFN rows, a 16k-row vocab shard), batch B with ~5.2k-token contexts,
hipGraph-captured + asynchronous decode through the engine -- with every collective replaced by a
same-sized call of the peer-mapped kernels on a one-rank communicator (parallel/comm.py
SingleRankTPComm): the fused reduction + residual + RMSNorm (2 per layer), the sampler's candidate
all-gather. Reports ms per step (graph replay and in-situ) and, under rocprofv3 --kernel-trace
--stats, launches per step.

  python tools/tp_decode_probe.py 1 32        # batch sizes;  TPP_TP=8 TPP_PROMPT=5200 TPP_STEPS=48
  TPP_MODEL=70b TPP_PREFILL=32768 python tools/tp_decode_probe.py 1 32   # + one 32k-token prefill step

TPP_PREFILL=T: after the decode probes, one prefill step of T tokens (prompts of TPP_PROMPT tokens) is
timed on the shard. Its bulk row-parallel all-reduces exceed the peer-mapped size limit and go to RCCL
in a real TP group; here they are skipped (one GPU cannot host an RCCL peer), so the number is the
shard's compute, and the xGMI time of the step is the bytes printed divided by the link rate.
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
    from rag_llm_k8s_amd.parallel.comm import SingleRankTPComm

    _build.build_all()
    Bs = [int(a) for a in sys.argv[1:]] or [1, 32]
    tp = int(os.environ.get("TPP_TP", "8"))
    plen = int(os.environ.get("TPP_PROMPT", "5200"))
    steps = int(os.environ.get("TPP_STEPS", "48"))
    model = os.environ.get("TPP_MODEL", "8b")
    cfg = L.llama31_8b() if model == "8b" else L.llama31_70b()
    dev = "cuda:0"
    comm = SingleRankTPComm(tp, 0, dev)
    w = L.LlamaWeights.random(cfg, dev, tp_rank=0, tp_size=tp, seed=0)
    m = L.LlamaModel(cfg, w, dev, comm=comm, max_positions=8192)
    g = w.geom()
    print("TP=%d rank-0 shard of %s: Hq=%d Hkv=%d I=%d vocab shard %d, %.2f GB of weights" % (
        tp, model, g["Hq"], g["Hkv"], g["I"], g["V"], w.nbytes() / 1e9), flush=True)
    for B in Bs:
        eng = LLMEngine(m, num_blocks=B * 128 + 16, max_batch=B, max_prefill_tokens=32768, max_model_len=8192,
                        eos_ids=cfg.eos_token_id, graph_buckets=[B])
        assert eng.tp_size == tp
        eng.warmup_graphs([B])
        gen = torch.Generator().manual_seed(B)
        p = SamplingParams(max_new_tokens=steps + 1, temperature=0.7, top_p=0.9, top_k=50, ignore_eos=True)
        for i in range(B):
            eng.add_request(torch.randint(3, cfg.vocab_size, (plen,), generator=gen).tolist(), p, seed=i)
        while any(s.computed < len(s.prompt) for s in eng.running) or eng.waiting:
            eng.step()
        torch.cuda.synchronize()
        d0, n0 = eng.stats["decode_s"], eng.stats["decode_steps"]
        t0 = time.perf_counter()
        eng.run_until_done()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        n = eng.stats["decode_steps"] - n0
        print("B=%d ctx=%d: %d decode steps, %.3f ms/step wall" % (B, plen, n, dt / n * 1e3), flush=True)
        del eng
        torch.cuda.empty_cache()
        # graph replay from a MID-RUN state (every row live; an end-of-run replay would stream only the rows
        # of the shrunken last batch): a fresh engine, half the decode steps, then back-to-back replays
        eng = LLMEngine(m, num_blocks=B * 128 + 16, max_batch=B, max_prefill_tokens=32768, max_model_len=8192,
                        eos_ids=cfg.eos_token_id, graph_buckets=[B])
        eng.warmup_graphs([B])
        gen = torch.Generator().manual_seed(B)
        for i in range(B):
            eng.add_request(torch.randint(3, cfg.vocab_size, (plen,), generator=gen).tolist(), p, seed=i)
        while any(s.computed < len(s.prompt) for s in eng.running) or eng.waiting:
            eng.step()
        for _ in range(max(1, steps // 2)):
            eng.step()
        torch.cuda.synchronize()
        e = eng.graphs.get(B)
        live = int((e["packed"][3 * B:4 * B] > 1).sum())
        e["graph"].replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            e["graph"].replay()
        torch.cuda.synchronize()
        print("B=%d graph replay only (mid-run, %d live rows): %.3f ms/step" % (
            B, live, (time.perf_counter() - t0) / 20 * 1e3), flush=True)
        eng.run_until_done()
        del eng
        torch.cuda.empty_cache()
    T = int(os.environ.get("TPP_PREFILL", "0"))
    if T:
        n = -(-T // plen)
        eng = LLMEngine(m, num_blocks=n * (-(-plen // 64)) + 16, max_batch=max(n, 1), max_prefill_tokens=T,
                        max_model_len=8192, eos_ids=cfg.eos_token_id, use_graphs=False)
        gen = torch.Generator().manual_seed(99)
        p = SamplingParams(max_new_tokens=2, temperature=0.7, top_p=0.9, top_k=50, ignore_eos=True)
        for rep in range(2):  # the first step warms the kernels
            for i in range(n):
                eng.add_request(torch.randint(3, cfg.vocab_size, (min(plen, T - i * plen),), generator=gen).tolist(),
                                p, seed=i)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            eng.step()
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            eng.run_until_done()
        H = cfg.hidden_size
        ar_bytes = 2 * cfg.num_hidden_layers * T * H * 2
        print("prefill step of %d tokens (%d prompts): %.1f ms compute on the shard (%.1f TFLOP/s); a real TP=%d "
              "step all-reduces %.1f GB of bf16 rows (2 per layer)" % (
                  T, n, dt * 1e3, 2 * T * w.nbytes() / 2 / dt / 1e12, tp, ar_bytes / 1e9), flush=True)


if __name__ == "__main__":
    main()
