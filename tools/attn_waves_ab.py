"""Prefill attention A/B: 4 vs 8 waves per block (GQA 4:1), interleaved rounds, bench shape."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rag_llm_k8s_amd.ops import native as N  # noqa: E402

Hq, Hkv, D = 32, 8, 128
dev = "cuda"
for B, S in [(6, 5184), (2, 2048)]:
    nb = B * S // 64 + 8
    kc = torch.randn(nb, Hkv, 64, D, device=dev).bfloat16()
    vc = torch.randn_like(kc)
    bt = torch.arange(nb, dtype=torch.int32, device=dev)[: B * S // 64].reshape(B, S // 64).contiguous()
    q = torch.randn(B * S, Hq * D, device=dev).bfloat16()
    cu = torch.arange(0, B + 1, dtype=torch.int32, device=dev) * S
    kvl = torch.full((B,), S, dtype=torch.int32, device=dev)
    out = torch.empty_like(q)
    res, ts = {}, {4: [], 8: []}
    for r in range(4):
        for w in (4, 8):
            N.set_prefill_waves(w)
            tiles = N.build_prefill_tiles([S] * B, Hq, Hkv).to(dev)
            fn = lambda: N.attn_prefill(q, kc, vc, cu, kvl, tiles, out, Hq, Hkv, D, causal=True, paged=True,  # noqa
                                        block_tables=bt)
            fn()
            torch.cuda.synchronize()
            res[w] = out.clone()
            s, e = torch.cuda.Event(True), torch.cuda.Event(True)
            s.record()
            for _ in range(5):
                fn()
            e.record()
            torch.cuda.synchronize()
            ts[w].append(s.elapsed_time(e) / 5 * 1e-3)
    N.set_prefill_waves(4)
    assert torch.equal(res[4], res[8]), (res[4].float() - res[8].float()).abs().max()
    flops = 4 * B * S * S * Hq * D / 2
    for w in (4, 8):
        t = sorted(ts[w])[1]
        print("B=%d S=%d waves=%d  %.1f us  %.0f TF" % (B, S, w, t * 1e6, flops / t / 1e12), flush=True)
