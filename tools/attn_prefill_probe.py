"""Prefill attention probe at the bench shape (one 32k-token prefill step: 6 prompts of 5.4k tokens,
causal, paged KV, Llama-8B heads) for rocprofv3 PMC passes and TF/s:

  python tools/attn_prefill_probe.py        # prints us per call and TF/s (causal FLOPs)
"""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rag_llm_k8s_amd.ops import native as N  # noqa: E402


def main():
    Hq, Hkv, D = 32, 8, 128
    lens = [int(x) for x in os.environ.get("AP_LENS", "5400,5400,5400,5400,5400,5400").split(",")]
    iters = int(os.environ.get("AP_ITERS", "5"))
    dev = "cuda:0"
    torch.manual_seed(0)
    nb = [(L + 63) // 64 for L in lens]
    total = sum(nb) + 1
    kc = (torch.randn(total, Hkv, 64, D, device=dev) * 0.5).bfloat16()
    vc = torch.randn(total, Hkv, 64, D, device=dev).bfloat16()
    perm = torch.randperm(total - 1, device=dev).int() + 1
    maxb = max(nb)
    bt = torch.zeros(len(lens), maxb, dtype=torch.int32, device=dev)
    i = 0
    for s, n in enumerate(nb):
        bt[s, :n] = perm[i:i + n]
        i += n
    T = sum(lens)
    q = (torch.randn(T, Hq * D, device=dev) * 0.5).bfloat16()
    cu = torch.tensor([0] + list(torch.cumsum(torch.tensor(lens), 0)), dtype=torch.int32, device=dev)
    kvl = torch.tensor(lens, dtype=torch.int32, device=dev)
    tiles = N.build_prefill_tiles(lens, Hq, Hkv).to(dev)
    out = torch.empty(T, Hq * D, device=dev).bfloat16()

    def run():
        N.attn_prefill(q, kc, vc, cu, kvl, tiles, out, Hq, Hkv, D, causal=True, paged=True, block_tables=bt)

    run()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(True), torch.cuda.Event(True)
    a.record()
    for _ in range(iters):
        run()
    b.record()
    b.synchronize()
    us = a.elapsed_time(b) / iters * 1e3
    flops = sum(4.0 * Hq * D * L * (L + 1) / 2 for L in lens)
    print("attn_prefill lens=%s: %.1f us, %.0f TF/s (causal FLOPs)" % (lens, us, flops / us / 1e6), flush=True)

if __name__ == "__main__":
    main()
