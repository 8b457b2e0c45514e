"""Prefill attention timing at the bench shapes (Llama-8B heads, causal, paged KV): by default one
32k-token prefill step of 6 prompts of ~5.4k tokens; AP_LENS / AP_CTX set other workloads (a single
5.2k prompt: AP_LENS=5200; a 2k chunk over 3k of context: AP_LENS=2048 AP_CTX=3072). Prints the
median time of AP_ROUNDS rounds of 5 launches, the attention TFLOP/s and the error against the fp32
oracle on the first prompt.

  python tools/attn_pp_ab.py
"""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rag_llm_k8s_amd.ops import native as N  # noqa: E402
from rag_llm_k8s_amd.ops import reference as R  # noqa: E402


def main():
    Hq, Hkv, D = 32, 8, 128
    lens = [int(x) for x in os.environ.get("AP_LENS", "5400,5400,5400,5400,5400,5400").split(",")]
    ctx = [int(x) for x in os.environ.get("AP_CTX", ",".join("0" for _ in lens)).split(",")]
    rounds = int(os.environ.get("AP_ROUNDS", "5"))
    dev = "cuda:0"
    torch.manual_seed(0)
    kvl_l = [q + c for q, c in zip(lens, ctx)]
    nb = [(L + 63) // 64 for L in kvl_l]
    total = sum(nb) + 1
    kc = (torch.randn(total, Hkv, 64, D, device=dev) * 0.5).bfloat16()
    vc = torch.randn(total, Hkv, 64, D, device=dev).bfloat16()
    perm = torch.randperm(total - 1, device=dev).int() + 1
    bt = torch.zeros(len(lens), max(nb), dtype=torch.int32, device=dev)
    i = 0
    for s, n in enumerate(nb):
        bt[s, :n] = perm[i:i + n]
        i += n
    T = sum(lens)
    q = (torch.randn(T, Hq * D, device=dev) * 0.5).bfloat16()
    cu = torch.tensor([0] + list(torch.cumsum(torch.tensor(lens), 0)), dtype=torch.int32, device=dev)
    kvl = torch.tensor(kvl_l, dtype=torch.int32, device=dev)
    flops = sum(4 * Hq * D * (q_ * c_ + q_ * q_ / 2) for q_, c_ in zip(lens, ctx))
    tiles = N.build_prefill_tiles(lens, Hq, Hkv).to(dev)
    out = torch.empty(T, Hq * D, device=dev).bfloat16()
    times = []
    for r in range(rounds + 1):
        a, b = torch.cuda.Event(True), torch.cuda.Event(True)
        a.record()
        for _ in range(5):
            N.attn_prefill(q, kc, vc, cu, kvl, tiles, out, Hq, Hkv, D, causal=True, paged=True, block_tables=bt)
        b.record()
        b.synchronize()
        if r:
            times.append(a.elapsed_time(b) / 5 * 1e3)
    t = sorted(times)[len(times) // 2]
    # fp32 oracle on the first prompt
    L0, c0 = lens[0], kvl_l[0]
    kf = R.paged_kv_view(kc.cpu(), bt[0].cpu(), c0, 64)
    vf = R.paged_kv_view(vc.cpu(), bt[0].cpu(), c0, 64)
    ref = R.attention_varlen(q[:L0].cpu().reshape(L0, Hq, D), None, None, torch.tensor([0, L0], dtype=torch.int32),
                             [c0], True, 1 / math.sqrt(D), k_full=lambda s: kf, v_full=lambda s: vf)
    got = out[:L0].float().cpu().reshape(L0, Hq, D)
    rel = ((got - ref).norm() / ref.norm()).item()
    print("lens=%s x%d ctx=%s  %.1f us  %.0f TF  rel_err(prompt 0 vs fp32)=%.2e" % (
        lens[0], len(lens), ctx[0], t, flops / t / 1e6, rel))


if __name__ == "__main__":
    main()
