"""The prefill qkv projection (Llama-3.1-8B: 32 q / 8 KV heads, K 4096) over one 32k-token chunk: gemm_w4
followed by rope_kv vs the GEMM with rope_kv's work in its epilogue (gemm_rope_kv), alternating, us per
chunk (median of 5 rounds of 5 launches each).

  python tools/rope_gemm_probe.py
"""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from rag_llm_k8s_amd import _build
    from rag_llm_k8s_amd.ops import native
    from rag_llm_k8s_amd.ops import reference as R

    _build.build_hip()
    M = int(os.environ.get("RP_M", "32768"))
    Hq, Hkv, D, K, BS = 32, 8, 128, 4096, 64
    N = (Hq + 2 * Hkv) * D
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    x = (torch.randn(M, K, device=dev, generator=g) * 0.5).bfloat16()
    w = (torch.randn(N, K, device=dev, generator=g) / math.sqrt(K)).bfloat16()
    cos, sin = R.rope_tables(D, 131072, theta=500000.0)
    cos, sin = cos.to(dev), sin.to(dev)
    pos = (torch.arange(M, device=dev) % 5400).int()
    nb = M // BS + 8
    slots = (torch.arange(M, device=dev) + BS).int()
    kc = torch.zeros(nb, Hkv, BS, D, device=dev).bfloat16()
    vc = torch.zeros_like(kc)
    out = torch.empty(M, N, device=dev).bfloat16()

    def separate():
        native.gemm(x, w, out=out)
        native.rope_kv(out, pos, cos, sin, slots, kc, vc, Hq, Hkv, D)

    def fused():
        native.gemm_rope_kv(x, w, pos, cos, sin, slots, kc, vc, Hq, Hkv, D, out=out)

    def timed(fn):
        ts = []
        for r in range(6):
            a, b = torch.cuda.Event(True), torch.cuda.Event(True)
            a.record()
            for _ in range(5):
                fn()
            b.record()
            b.synchronize()
            if r:
                ts.append(a.elapsed_time(b) / 5 * 1e3)
        return sorted(ts)[len(ts) // 2]

    for rnd in range(3):
        ts, tf = timed(separate), timed(fused)
        print("round %d: gemm + rope_kv %.1f us, fused %.1f us (M %d)" % (rnd, ts, tf, M), flush=True)


if __name__ == "__main__":
    main()
