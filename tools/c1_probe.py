"""Single-query (C=1) latency anatomy of the served RAG path on one GPU (bench.py's config-2 workload):
query embed, index search, prompt build + tokenize, the prefill step (first token) and the decode
steps, each bracketed by torch.cuda.synchronize(). Prints ms per phase (median of N queries)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from rag_llm_k8s_amd import _build
    from rag_llm_k8s_amd.engine.llm_engine import SamplingParams
    from rag_llm_k8s_amd.ingest.text import build_context, build_prompt
    from rag_llm_k8s_amd.parallel import dist as D
    from rag_llm_k8s_amd.utils.workload import build_workload, make_queries

    _build.build_all()
    ctx = D.init_distributed(tp=1)
    wl = build_workload(model="8b", embedder="minilm", n_chunks=10000, retrieve_k=4,
                        context_k=4, max_new_tokens=150, max_batch=32, device=ctx.device, ctx=ctx, tp_comm=None,
                        seed=0, use_graphs=True, index_type="flat", dtype="bf16", index_vectors=0)
    svc = wl.svc
    eng = svc.engine
    eng.warmup_graphs()
    params = SamplingParams(max_new_tokens=150, temperature=0.7, top_p=0.9, top_k=50, do_sample=True,
                            ignore_eos=True)
    n = int(os.environ.get("C1_N", "8"))
    rows = []
    for i in range(n + 1):
        q = make_queries(wl.wm, 1, seed=777000 + i)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e = svc.embedder.embed(q)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        res = svc.store.search(e, svc.cfg.retrieve_k)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        full = build_prompt(build_context(res[0], svc.cfg.context_k), q[0])
        ids = svc.tok.encode_batch([full], add_special_tokens=True)[0]
        t3 = time.perf_counter()
        s = eng.add_request(svc._prompt_ids(None, ids=ids), params, seed=4242 + i)
        while not s.out:
            eng.step()
        torch.cuda.synchronize()
        t4 = time.perf_counter()
        while eng.has_work():
            eng.step()
        torch.cuda.synchronize()
        t5 = time.perf_counter()
        if i:  # first query warms up
            rows.append([(t1 - t0) * 1e3, (t2 - t1) * 1e3, (t3 - t2) * 1e3, (t4 - t3) * 1e3, (t5 - t4) * 1e3,
                         (t5 - t0) * 1e3, len(ids), len(s.out)])
    med = [sorted(r[k] for r in rows)[len(rows) // 2] for k in range(8)]
    print("C=1 anatomy (median of %d): embed %.2f ms, search %.2f ms, prompt+tokenize %.2f ms, prefill->first "
          "token %.2f ms, decode %.2f ms (%d tokens, %.3f ms/token), total %.1f ms, prompt %d tokens" % (
              len(rows), med[0], med[1], med[2], med[3], med[4], med[7] - 1, med[4] / max(1, med[7] - 1), med[5],
              med[6]), flush=True)


if __name__ == "__main__":
    main()
