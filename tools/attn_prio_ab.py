"""Prefill attention A/B: wave priority around the MFMA clusters (attention.hip PRIO 0 / 1 / 2),
Llama-8B GQA 4:1 causal paged config, bench-like shapes, interleaved rounds in one process."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rag_llm_k8s_amd.ops import _lib  # noqa: E402
from rag_llm_k8s_amd.ops import native as N  # noqa: E402

L = _lib.lib()
Hq, Hkv, D = 32, 8, 128
dev = "cuda"
VARIANTS = (0, 1, 3)  # 3 = prio 1 + buffer-descriptor K/V staging
for B, S in [(6, 5184), (2, 2048)]:
    nb = B * S // 64 + 8
    kc = torch.randn(nb, Hkv, 64, D, device=dev).bfloat16()
    vc = torch.randn_like(kc)
    bt = torch.arange(nb, dtype=torch.int32, device=dev)[: B * S // 64].reshape(B, S // 64).contiguous()
    q = torch.randn(B * S, Hq * D, device=dev).bfloat16()
    cu = torch.arange(0, B + 1, dtype=torch.int32, device=dev) * S
    kvl = torch.full((B,), S, dtype=torch.int32, device=dev)
    out = torch.empty_like(q)
    tiles = N.build_prefill_tiles([S] * B, Hq, Hkv).to(dev)
    res, ts = {}, {v: [] for v in VARIANTS}

    def fn():
        N.attn_prefill(q, kc, vc, cu, kvl, tiles, out, Hq, Hkv, D, causal=True, paged=True, block_tables=bt)

    for r in range(5):
        for v in VARIANTS:
            L.ragk_attn_prefill_set_prio(min(v, 1) if v != 2 else 2)
            L.ragk_attn_prefill_set_buf(1 if v == 3 else 0)
            fn()
            torch.cuda.synchronize()
            res[v] = out.clone()
            s, e = torch.cuda.Event(True), torch.cuda.Event(True)
            s.record()
            for _ in range(5):
                fn()
            e.record()
            torch.cuda.synchronize()
            ts[v].append(s.elapsed_time(e) / 5 * 1e-3)
    L.ragk_attn_prefill_set_prio(1)
    L.ragk_attn_prefill_set_buf(1)
    for v in VARIANTS:
        assert torch.equal(res[v], res[0]), v
    flops = 4 * B * S * S * Hq * D / 2
    for v in VARIANTS:
        t = sorted(ts[v])[2]
        print("B=%d S=%d prio=%d  %.1f us  %.0f TF" % (B, S, v, t * 1e6, flops / t / 1e12), flush=True)
