"""Decode gate/up GEMM (gemm_stream, SiLU*up epilogue, M=32) A/B: default vs non-temporal weight
LDS-DMA, interleaved rounds in one process. The weights rotate over 8 layers' matrices (1.9 GB) so
every call streams from HBM, as in a decode step (the whole model is 16 GB, the Infinity Cache 256 MB)."""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rag_llm_k8s_amd.ops import _lib  # noqa: E402
from rag_llm_k8s_amd.ops import native as N  # noqa: E402

L = _lib.lib()
K, F, LAYERS = 4096, 14336, 8
for M in (32, 1):
    x = torch.randn(M, K, device="cuda").bfloat16()
    ws = [(torch.randn(2 * F, K, device="cuda") / math.sqrt(K)).bfloat16() for _ in range(LAYERS)]
    out = torch.empty(M, F, device="cuda").bfloat16()
    ts = {0: [], 1: []}
    ref = None
    for r in range(5):
        for nt in (0, 1):
            L.ragk_gemm_stream_set_nt(nt)
            N.gemm(x, ws[0], epi="silu_mul", out=out, path=5)
            torch.cuda.synchronize()
            if ref is None:
                ref = out.clone()
            assert torch.equal(out, ref), "policy must not change results"
            s, e = torch.cuda.Event(True), torch.cuda.Event(True)
            s.record()
            for i in range(4 * LAYERS):
                N.gemm(x, ws[i % LAYERS], epi="silu_mul", out=out, path=5)
            e.record()
            torch.cuda.synchronize()
            ts[nt].append(s.elapsed_time(e) / (4 * LAYERS) * 1e-3)
    L.ragk_gemm_stream_set_nt(1)
    byts = 2 * F * K * 2
    for nt in (0, 1):
        t = sorted(ts[nt])[2]
        print("gate/up M=%d nt=%d  %.1f us  %.2f TB/s" % (M, nt, t * 1e6, byts / t / 1e12), flush=True)
