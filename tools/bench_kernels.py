"""Kernel microbenchmarks on one MI355X: our HIP kernels vs torch (hipBLASLt / aten).

python tools/bench_kernels.py [--quick]   -> prints a table and writes profiles/kernels_*.json
"""
import argparse
import json
import math
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rag_llm_k8s_amd.ops import native as N  # noqa: E402
from rag_llm_k8s_amd.ops import fp8 as F8  # noqa: E402
from rag_llm_k8s_amd.ops import reference as R  # noqa: E402


def timeit(fn, iters=20, warmup=5):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e-3  # seconds


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--out", default="gpurun_out/kernels.json")
    args = ap.parse_args()
    dev = "cuda"
    rows = []
    torch.manual_seed(0)

    # ---------------- prefill GEMMs (Llama-3.1-8B shapes, M = tokens)
    for M in ([4096] if args.quick else [512, 4096, 16384]):
        for (N_, K, epi, name) in [(6144, 4096, "none", "qkv"), (4096, 4096, "resid", "o_proj"),
                                   (14336, 4096, "silu_mul", "gate_up+silu"), (4096, 14336, "resid", "down")]:
            x = torch.randn(M, K, device=dev).bfloat16()
            wn = 2 * N_ if epi == "silu_mul" else N_
            w = (torch.randn(wn, K, device=dev) / math.sqrt(K)).bfloat16()
            r = torch.randn(M, N_, device=dev).bfloat16() if epi == "resid" else None
            out = torch.empty(M, N_, device=dev).bfloat16()
            t = timeit(lambda: N.gemm(x, w, resid=r, epi=epi, out=out, path=6))
            t0 = timeit(lambda: N.gemm(x, w, resid=r, epi=epi, out=out, path=0))
            w8 = F8.quantize_weight(w)
            t8 = timeit(lambda: N.gemm_fp8(x, w8, resid=r, epi=epi, out=out))
            flops = 2 * M * wn * K
            tt = timeit(lambda: torch.matmul(x, w.t()))
            rows.append(dict(kind="gemm_prefill", name=name, M=M, N=wn, K=K, pp_us=t * 1e6, pp_tflops=flops / t / 1e12,
                             tile128_tflops=flops / t0 / 1e12, fp8_w8a8_tflops=flops / t8 / 1e12,
                             torch_us=tt * 1e6, torch_tflops=flops / tt / 1e12))
            print(rows[-1], flush=True)

    # ---------------- decode GEMMs (weight streaming)
    for M in ([1, 32] if args.quick else [1, 8, 32, 64]):
        for (N_, K, epi, name) in [(6144, 4096, "none", "qkv"), (4096, 4096, "resid", "o_proj"),
                                   (14336, 4096, "silu_mul", "gate_up+silu"), (4096, 14336, "resid", "down"),
                                   (128256, 4096, "none", "lm_head")]:
            x = torch.randn(M, K, device=dev).bfloat16()
            wn = 2 * N_ if epi == "silu_mul" else N_
            # rotate through >= 1.5 GB of weight copies so nothing is served from the 256 MB
            # Infinity Cache (a real decode step streams ~15 GB of distinct weights)
            ncopy = max(2, -(-(1536 << 20) // (wn * K * 2)))
            ws_ = [(torch.randn(wn, K, device=dev) / math.sqrt(K)).bfloat16() for _ in range(ncopy)]
            r = torch.randn(M, N_, device=dev).bfloat16() if epi == "resid" else None
            out = torch.empty(M, N_, device=dev).bfloat16()
            it = [0]

            def nxt():
                it[0] = (it[0] + 1) % ncopy
                return ws_[it[0]]

            w8s = [F8.quantize_weight(wc) for wc in ws_]
            it8 = [0]

            def nxt8():
                it8[0] = (it8[0] + 1) % ncopy
                return w8s[it8[0]]

            t8 = timeit(lambda: N.gemm_fp8(x, nxt8(), resid=r, epi=epi, out=out), iters=ncopy * 4)
            del w8s
            t5 = timeit(lambda: N.gemm(x, nxt(), resid=r, epi=epi, out=out, path=5), iters=ncopy * 4)
            t3 = timeit(lambda: N.gemm(x, nxt(), resid=r, epi=epi, out=out, path=4), iters=ncopy * 4)
            t1 = timeit(lambda: N.gemm(x, nxt(), resid=r, epi=epi, out=out, path=1), iters=ncopy * 4)
            tt = timeit(lambda: torch.matmul(x, nxt().t()), iters=ncopy * 4)
            del ws_
            byts = wn * K * 2
            rows.append(dict(kind="gemm_decode", name=name, M=M, N=wn, K=K, fp8_us=t8 * 1e6,
                             fp8_TBps=byts / 2 / t8 / 1e12, v4_us=t5 * 1e6, v4_TBps=byts / t5 / 1e12, v3_us=t3 * 1e6, v3_TBps=byts / t3 / 1e12,
                             v1_TBps=byts / t1 / 1e12, torch_us=tt * 1e6, torch_TBps=byts / tt / 1e12))
            print(rows[-1], flush=True)

    # ---------------- prefill attention (causal, GQA 32/8, D=128)
    Hq, Hkv, D = 32, 8, 128
    for S, B in ([(4096, 1)] if args.quick else [(1024, 8), (4096, 2), (8192, 1)]):
        nb = B * S // 64 + 8
        kc = torch.randn(nb, Hkv, 64, D, device=dev).bfloat16()
        vc = torch.randn_like(kc)
        bt = torch.arange(nb, dtype=torch.int32, device=dev)[: B * S // 64].reshape(B, S // 64).contiguous()
        q = torch.randn(B * S, Hq * D, device=dev).bfloat16()
        cu = torch.arange(0, B + 1, dtype=torch.int32, device=dev) * S
        kvl = torch.full((B,), S, dtype=torch.int32, device=dev)
        tiles = N.build_prefill_tiles([S] * B, Hq, Hkv).to(dev)
        out = torch.empty_like(q)
        t = timeit(lambda: N.attn_prefill(q, kc, vc, cu, kvl, tiles, out, Hq, Hkv, D, causal=True, paged=True,
                                          block_tables=bt))
        flops = 4 * B * S * S * Hq * D / 2
        qq = q.reshape(B, S, Hq, D).transpose(1, 2)
        kk = torch.randn(B, Hkv, S, D, device=dev).bfloat16().repeat_interleave(4, 1)
        vv = torch.randn_like(kk)
        tt = timeit(lambda: torch.nn.functional.scaled_dot_product_attention(qq, kk, vv, is_causal=True))
        rows.append(dict(kind="attn_prefill", S=S, B=B, ours_us=t * 1e6, ours_tflops=flops / t / 1e12,
                         torch_sdpa_us=tt * 1e6, torch_tflops=flops / tt / 1e12))
        print(rows[-1], flush=True)

    # ---------------- decode attention
    for B, L in ([(32, 5600)] if args.quick else [(1, 5600), (32, 5600), (64, 2048)]):
        nbs = (L + 63) // 64
        kc = torch.randn(B * nbs + 4, Hkv, 64, D, device=dev).bfloat16()
        vc = torch.randn_like(kc)
        bt = torch.arange(B * nbs, dtype=torch.int32, device=dev).reshape(B, nbs).contiguous()
        q = torch.randn(B, Hq * D, device=dev).bfloat16()
        kvl = torch.full((B,), L, dtype=torch.int32, device=dev)
        pt, mp = N.decode_partitions(L, B, Hkv)
        out = torch.empty_like(q)
        wo = torch.empty(B, Hq, mp, D, device=dev)
        wml = torch.empty(B, Hq, mp, 2, device=dev)
        t = timeit(lambda: N.attn_decode(q, kc, vc, bt, kvl, out, Hq, Hkv, D, pt, mp, wo, wml), iters=50)
        byts = B * L * Hkv * D * 2 * 2
        rows.append(dict(kind="attn_decode", B=B, L=L, part_tiles=pt, parts=mp, ours_us=t * 1e6,
                         ours_TBps=byts / t / 1e12))
        print(rows[-1], flush=True)

    # ---------------- norms / sampling / search
    x = torch.randn(4096, 4096, device=dev).bfloat16()
    w = torch.randn(4096, device=dev).bfloat16()
    t = timeit(lambda: N.rmsnorm(x, w, 1e-5))
    rows.append(dict(kind="rmsnorm", T=4096, H=4096, ours_us=t * 1e6, TBps=2 * x.numel() * 2 / t / 1e12))
    print(rows[-1], flush=True)
    lg = torch.randn(32, 128256, device=dev)
    t = timeit(lambda: N.topk_candidates(lg, 50))
    rows.append(dict(kind="topk50", B=32, V=128256, ours_us=t * 1e6))
    print(rows[-1], flush=True)
    for n, d in [(10000, 384), (1000000, 1024)] if not args.quick else [(10000, 384)]:
        xt = torch.randn(d, n, device=dev)
        qv = torch.randn(32, d, device=dev)
        t = timeit(lambda: N.l2_search(xt, n, n, qv, 4), iters=5, warmup=1)
        rows.append(dict(kind="l2_search", N=n, d=d, nq=32, ours_us=t * 1e6, TBps=n * d * 4 / t / 1e12))
        print(rows[-1], flush=True)

    os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
    with open(args.out, "w") as f:
        json.dump({"device": torch.cuda.get_device_name(), "time": time.time(), "rows": rows}, f, indent=1)


if __name__ == "__main__":
    main()
