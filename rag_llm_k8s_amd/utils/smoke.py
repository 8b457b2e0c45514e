"""smoke(): one tiny end-to-end RAG query on the GPU through the native kernels."""
from __future__ import annotations

import time

import torch


def run_smoke(device="cuda:0"):
    from .. import _build
    from ..engine.llm_engine import SamplingParams
    from ..ops import _lib
    from .workload import build_workload, make_queries

    _build.build_all()
    torch.cuda.set_device(torch.device(device))
    t0 = time.time()
    wl = build_workload(model="tiny", embedder="tiny", n_chunks=64, chunk_words=120, retrieve_k=4, context_k=4,
                        max_new_tokens=8, max_batch=4, max_model_len=2048, max_prefill_tokens=4096, device=device,
                        word_vocab=20000)
    assert _lib._lib is not None, "native gfx950 kernel library was not loaded"
    qs = make_queries(wl.wm, 3, seed=1)
    outs = wl.svc.generate_batch(qs, params=SamplingParams(max_new_tokens=8, temperature=0.7, top_p=0.9, top_k=50,
                                                           ignore_eos=True), seeds=[1, 2, 3])
    torch.cuda.synchronize()
    for o in outs:
        assert isinstance(o["generated_text"], str)
        assert o["context"].startswith("Document 'synthetic_")
        assert o["_gen_tokens"] == 8
    print("smoke ok: %d queries, prompt tokens %s, %.1fs, lib=%s" % (
        len(outs), [o["_prompt_tokens"] for o in outs], time.time() - t0, _lib.LIB_PATH))
