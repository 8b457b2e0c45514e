"""Prefill attention cycle anatomy (stamp build) on the bench shape: causal GQA 32/8, D=128,
paged cache, 6 x 5200-token prompts."""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rag_llm_k8s_amd.ops import _lib  # noqa: E402
from rag_llm_k8s_amd.ops import native as N  # noqa: E402
from rag_llm_k8s_amd.ops._lib import check, stream_ptr  # noqa: E402

Hq, Hkv, D = 32, 8, 128
B, S = 6, 5184
dev = "cuda"
nb = B * S // 64 + 8
kc = torch.randn(nb, Hkv, 64, D, device=dev).bfloat16()
vc = torch.randn_like(kc)
bt = torch.arange(nb, dtype=torch.int32, device=dev)[: B * S // 64].reshape(B, S // 64).contiguous()
q = torch.randn(B * S, Hq * D, device=dev).bfloat16()
cu = torch.arange(0, B + 1, dtype=torch.int32, device=dev) * S
kvl = torch.full((B,), S, dtype=torch.int32, device=dev)
tiles = N.build_prefill_tiles([S] * B, Hq, Hkv).to(dev)
out = torch.empty_like(q)
fn = lambda: N.attn_prefill(q, kc, vc, cu, kvl, tiles, out, Hq, Hkv, D, causal=True, paged=True, block_tables=bt)  # noqa
for _ in range(3):
    fn()
torch.cuda.synchronize()
s, e = torch.cuda.Event(True), torch.cuda.Event(True)
s.record()
for _ in range(5):
    fn()
e.record()
torch.cuda.synchronize()
t = s.elapsed_time(e) / 5 * 1e-3
flops = 4 * B * S * S * Hq * D / 2
print("B=%d S=%d  %.1f us  %.0f TF (causal flops)" % (B, S, t * 1e6, flops / t / 1e12))
nt = tiles.shape[0]
grid = nt * Hkv * (Hq // Hkv // 4)
dbg = torch.zeros(grid * 4 * 6, dtype=torch.int64, device=dev)
L = _lib.lib()
check(L.ragk_attn_prefill_stamp(q.data_ptr(), q.stride(0), kc.data_ptr(), vc.data_ptr(), bt.data_ptr(), bt.stride(0),
                                cu.data_ptr(), kvl.data_ptr(), tiles.data_ptr(), nt, out.data_ptr(), out.stride(0),
                                Hq, Hkv, 1.0 / math.sqrt(D), dbg.data_ptr(), stream_ptr()), "stamp")
torch.cuda.synchronize()
d = dbg.view(grid, 4, 6).double().cpu()
n = d[:, :, 5].sum()
tot = d[:, :, :5].sum((0, 1)) / n
print("per 64-key tile per wave (mean cycles): DMA issue %.0f | QK^T %.0f | softmax %.0f | PV %.0f | wait+barrier %.0f"
      " = %.0f  (64 MFMA x 16 = 1024 ideal per wave; 2 waves/SIMD)" % (*tot.tolist(), tot.sum().item()))
