"""Decode attention A/B in one process, interleaved rounds: default vs non-temporal K/V loads."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rag_llm_k8s_amd.ops import _lib  # noqa: E402
from rag_llm_k8s_amd.ops import native as N  # noqa: E402

Hq, Hkv, D = 32, 8, 128
L = _lib.lib()
for B, Lk in [(32, 5300), (1, 5300), (64, 2048)]:
    nbs = (Lk + 63) // 64
    kc = torch.randn(B * nbs + 4, Hkv, 64, D, device="cuda").bfloat16()
    vc = torch.randn_like(kc)
    bt = torch.randperm(B * nbs, device="cuda").int().reshape(B, nbs).contiguous()
    q = torch.randn(B, Hq * D, device="cuda").bfloat16()
    kvl = torch.full((B,), Lk, dtype=torch.int32, device="cuda")
    pt, mp = N.decode_partitions(Lk, B, Hkv)
    out = torch.empty_like(q)
    wo = torch.empty(B, Hq, mp, D, device="cuda")
    wml = torch.empty(B, Hq, mp, 2, device="cuda")
    ts = {0: [], 1: []}
    ref = None
    for r in range(5):
        for nt in (0, 1):
            L.ragk_attn_decode_set_nt(nt)
            N.attn_decode(q, kc, vc, bt, kvl, out, Hq, Hkv, D, pt, mp, wo, wml)
            torch.cuda.synchronize()
            if ref is None:
                ref = out.clone()
            assert torch.equal(out, ref)
            s, e = torch.cuda.Event(True), torch.cuda.Event(True)
            s.record()
            for _ in range(20):
                N.attn_decode(q, kc, vc, bt, kvl, out, Hq, Hkv, D, pt, mp, wo, wml)
            e.record()
            torch.cuda.synchronize()
            ts[nt].append(s.elapsed_time(e) / 20 * 1e-3)
    L.ragk_attn_decode_set_nt(0)
    byts = B * Lk * Hkv * D * 2 * 2
    for nt in (0, 1):
        t = sorted(ts[nt])[2]
        print("B=%d L=%d parts=%d x %d tiles nt=%d  %.1f us  %.2f TB/s" % (B, Lk, mp, pt, nt, t * 1e6, byts / t / 1e12))
