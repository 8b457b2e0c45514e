"""Decode attention A/B in one process, interleaved rounds.

Arms: the engine's former fixed split (partitions of 32 tiles, sized for max_model_len 8192) vs the
length-balanced split (attention.hip:decode_part_tiles) at grid targets of 512 / 1024 / 2048 blocks.
Different splits change the fp32 summation order, so each arm is checked against the first one
with a tolerance."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rag_llm_k8s_amd.ops import native as N  # noqa: E402

Hq, Hkv, D = 32, 8, 128
MAX_LEN = 8192
for B, Lk in [(32, 5300), (32, 2000), (16, 5300), (64, 2048)]:
    nbs = (Lk + 63) // 64
    kc = torch.randn(B * nbs + 4, Hkv, 64, D, device="cuda").bfloat16()
    vc = torch.randn_like(kc)
    bt = torch.randperm(B * nbs, device="cuda").int().reshape(B, nbs).contiguous()
    q = torch.randn(B, Hq * D, device="cuda").bfloat16()
    kvl = torch.full((B,), Lk, dtype=torch.int32, device="cuda")
    arms = {"fixed32": (32, -(-((MAX_LEN + 63) // 64) // 32))}
    for tb in (256, 512, 1024):
        arms["bal%d" % tb] = N.decode_partitions(MAX_LEN, B, Hkv, target_blocks=tb)
    ts = {k: [] for k in arms}
    ref = None
    for r in range(5):
        for name, (pt, mp) in arms.items():
            out = torch.empty_like(q)
            wo = torch.empty(B, Hq, mp, D, device="cuda")
            wml = torch.empty(B, Hq, mp, 2, device="cuda")
            N.attn_decode(q, kc, vc, bt, kvl, out, Hq, Hkv, D, pt, mp, wo, wml)
            torch.cuda.synchronize()
            if ref is None:
                ref = out.float().clone()
            err = ((out.float() - ref).norm() / ref.norm()).item()
            assert err < 1e-2, (name, err)
            s, e = torch.cuda.Event(True), torch.cuda.Event(True)
            s.record()
            for _ in range(20):
                N.attn_decode(q, kc, vc, bt, kvl, out, Hq, Hkv, D, pt, mp, wo, wml)
            e.record()
            torch.cuda.synchronize()
            ts[name].append(s.elapsed_time(e) / 20 * 1e-3)
    byts = B * Lk * Hkv * D * 2 * 2
    for name, (pt, mp) in arms.items():
        t = sorted(ts[name])[2]
        print("B=%d L=%d %-8s min_tiles=%d max_parts=%d  %.1f us  %.2f TB/s" % (B, Lk, name, pt, mp, t * 1e6,
                                                                           byts / t / 1e12), flush=True)
