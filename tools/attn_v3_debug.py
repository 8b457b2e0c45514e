"""Debug: which rows / heads of the 8-wave v3 prefill kernel differ from the 4-wave kernel."""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rag_llm_k8s_amd.ops import native as N  # noqa: E402


def run(q_lens, kv_lens, Hq, Hkv, mode):
    D = 128
    torch.manual_seed(19)
    dev = "cuda"
    nb = [(L + 63) // 64 for L in kv_lens]
    total = sum(nb) + 3
    kc = torch.zeros(total, Hkv, 64, D, device=dev).bfloat16()
    vc = torch.zeros_like(kc)
    kc[1:] = torch.randn(total - 1, Hkv, 64, D, device=dev).bfloat16()
    vc[1:] = torch.randn(total - 1, Hkv, 64, D, device=dev).bfloat16()
    bt = torch.zeros(len(kv_lens), max(nb), dtype=torch.int32, device=dev)
    i = 1
    for s_, n in enumerate(nb):
        bt[s_, :n] = torch.arange(i, i + n, dtype=torch.int32)
        i += n
    T = sum(q_lens)
    q = torch.randn(T, Hq * D, device=dev).bfloat16()
    cu = torch.tensor([0] + list(torch.cumsum(torch.tensor(q_lens), 0)), dtype=torch.int32, device=dev)
    kvl = torch.tensor(kv_lens, dtype=torch.int32, device=dev)
    outs = []
    for m in (0, mode):
        N.set_prefill_waves(4, pp=m)
        tiles = N.build_prefill_tiles(q_lens, Hq, Hkv).to(dev)
        out = torch.full((T, Hq * D), float("nan"), device=dev).bfloat16()
        N.attn_prefill(q, kc, vc, cu, kvl, tiles, out, Hq, Hkv, D, causal=True, paged=True, block_tables=bt)
        torch.cuda.synchronize()
        outs.append(out.float().view(T, Hq, D))
    N.set_prefill_waves(4, pp=0)
    err = (outs[1] - outs[0]).abs().amax(-1)  # [T, Hq]
    bad = (err > 0.05) | ~torch.isfinite(err)
    print("q_lens", q_lens, "kv", kv_lens, "Hq/Hkv", Hq, Hkv, "mode", mode, "bad rows:",
          sorted(set(bad.nonzero()[:, 0].tolist()))[:40], "bad heads:", sorted(set(bad.nonzero()[:, 1].tolist())))


for mode in (10, 6):
    run([37], [37], 8, 2, mode)
    run([64], [64], 4, 1, mode)
    run([100], [100], 4, 1, mode)
    run([200], [200], 4, 1, mode)
    run([1], [1], 4, 1, mode)
