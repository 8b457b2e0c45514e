"""Batch-32 decode attention in isolation, as the engine runs it (fused RoPE + KV append from the qkv
split-K slabs, paged cache with each sequence's blocks contiguous, 8-wave single-partition blocks,
non-temporal K / V), over NL distinct layer caches replayed in a hipGraph (nothing served from the
Infinity Cache). Prints us per launch and TB/s of KV for each variant:

  python tools/attn_decode_probe.py                 # AP_B=32 AP_CTX=5264 AP_NL=6 AP_JITTER=0
  AP_VARIANTS=base,diag,base python tools/attn_decode_probe.py

variants: base | diag (loads + waits only, no QK^T / softmax / PV: attention.hip DG = 1) | diag_dma (as diag,
K by 1 KiB LDS-DMA pieces too: DG = 2) | kl (4-wave blocks, K tiles by LDS-DMA: attention.hip KL) | nt0
(default cache policy). AP_CHECK=1: every variant's output vs the base kernel's. AP_JITTER=n: context lengths uniform in [ctx - n, ctx + n] (the bench's RAG prompts vary).
"""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from rag_llm_k8s_amd import _build
    from rag_llm_k8s_amd.ops import _lib, native
    from rag_llm_k8s_amd.ops.reference import rope_tables

    _build.build_all()
    B = int(os.environ.get("AP_B", "32"))
    ctx = int(os.environ.get("AP_CTX", "5264"))
    NL = int(os.environ.get("AP_NL", "6"))
    jit = int(os.environ.get("AP_JITTER", "0"))
    reps = int(os.environ.get("AP_REPS", "20"))
    # AP_HKV=1 with AP_B=256: the same 256 (sequence, KV head) streams and bytes, each stream's tiles in
    # consecutive cache blocks -- the access pattern of a head-major cache layout ([Hkv][blocks][64][D])
    Hkv = int(os.environ.get("AP_HKV", "8"))
    Hq, D = 4 * Hkv, 128
    dev = "cuda"
    g = torch.Generator().manual_seed(1)
    lens = [ctx + (int(torch.randint(-jit, jit + 1, (1,), generator=g)) if jit else 0) for _ in range(B)]
    nbs = [(n + 63) // 64 + 1 for n in lens]
    nblocks = 1 + sum(nbs)
    mb = max(nbs)
    bt = torch.zeros(B, mb, dtype=torch.int32)
    nxt = 1
    for i, n in enumerate(nbs):  # each sequence's blocks contiguous, as the engine's block manager hands them out
        bt[i, :n] = torch.arange(nxt, nxt + n, dtype=torch.int32)
        nxt += n
    pos = torch.tensor([n - 1 for n in lens], dtype=torch.int32)
    slots = torch.tensor([int(bt[i, p // 64]) * 64 + p % 64 for i, p in enumerate(pos.tolist())], dtype=torch.int32)
    kvl = torch.tensor(lens, dtype=torch.int32)
    bt, pos, slots, kvl = bt.to(dev), pos.to(dev), slots.to(dev), kvl.to(dev)
    # AP_VOFF=bytes: K and V of a layer in ONE allocation, V starting that many bytes past the end of K (a
    # tile's K and V pieces then sit at different offsets modulo the memory interleave); default: two
    # separate allocations
    voff = int(os.environ.get("AP_VOFF", "-1"))

    def kv_pair():
        n = nblocks * Hkv * 64 * D
        if voff < 0:
            return (torch.randn(nblocks, Hkv, 64, D, device=dev).bfloat16(),
                    torch.randn(nblocks, Hkv, 64, D, device=dev).bfloat16())
        buf = torch.randn(2 * n + voff // 2, device=dev).bfloat16()
        return buf[:n].view(nblocks, Hkv, 64, D), buf[n + voff // 2:2 * n + voff // 2].view(nblocks, Hkv, 64, D)

    caches = [kv_pair() for _ in range(NL)]
    cos, sin = rope_tables(D, 8192, 500000.0, None)
    cos, sin = cos.to(dev), sin.to(dev)
    P = torch.randn(4, B, (Hq + 2 * Hkv) * D, device=dev) * 0.1
    out = torch.empty(B, Hq * D, device=dev).bfloat16()
    pt, mp = native.decode_partitions(8192, B, Hkv)
    kv_bytes = sum(lens) * Hkv * D * 2 * 2
    print("B=%d ctx %d..%d (mean %.0f) NL=%d: %.1f MB of KV per launch, part_tiles %d max_parts %d" % (
        B, min(lens), max(lens), sum(lens) / B, NL, kv_bytes / 1e6, pt, mp), flush=True)
    L = _lib.lib()

    def run():
        for kc, vc in caches:
            native.attn_decode_rope(P, pos, cos, sin, slots, kc, vc, bt, kvl, out, Hq, Hkv, D, pt, mp)

    variants = [v for v in os.environ.get("AP_VARIANTS", "base,diag,base,diag").split(",") if v]
    if os.environ.get("AP_CHECK") == "1":
        outs = {}
        kl_default = native.DECODE_KL
        for v in ("base", "kl"):
            native.DECODE_KL = v == "kl"
            kc, vc = caches[0]
            native.attn_decode_rope(P, pos, cos, sin, slots, kc, vc, bt, kvl, out, Hq, Hkv, D, pt, mp)
            torch.cuda.synchronize()
            outs[v] = out.clone()
        native.DECODE_KL = kl_default
        print("kl vs base: bit-identical %s, max abs diff %.3g" % (
            torch.equal(outs["kl"], outs["base"]), (outs["kl"].float() - outs["base"].float()).abs().max().item()),
            flush=True)
    graphs = {}
    for v in variants:
        key = v
        if key not in graphs:
            L.ragk_attn_decode_set_diag({"diag": 1, "diag_dma": 2}.get(v, 0))
            kl_default = native.DECODE_KL
            native.DECODE_KL = v == "kl"  # base: the 8-wave kernel with K in registers
            nt_min = native.DECODE_NT_MIN_BH
            native.DECODE_NT_MIN_BH = 1 << 30 if v == "nt0" else nt_min
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                run()
            torch.cuda.current_stream().wait_stream(s)
            torch.cuda.synchronize()
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr, stream=s):
                run()
            graphs[key] = gr
            native.DECODE_NT_MIN_BH = nt_min
            L.ragk_attn_decode_set_diag(0)
            native.DECODE_KL = kl_default
        gr = graphs[key]
        gr.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            gr.replay()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / reps / NL
        print("%-6s %8.1f us per launch  %.2f TB/s of KV" % (v, us, kv_bytes / us / 1e6), flush=True)


if __name__ == "__main__":
    main()
