"""A/B of the prefill attention kernels at the bench shape (one 32k-token prefill step: 6 prompts of
~5.4k tokens, causal, paged KV, Llama-8B heads): 4-wave kernel vs the 8-wave ping-pong kernel
(attention.hip attn_prefill_pp_kernel, mode 1 / 2 = + static priority for waves 4-7). Interleaved
rounds in one process; outputs must be bit-identical.

  python tools/attn_pp_ab.py            # AP_LENS=5400,... AP_ROUNDS=5
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
    ctx = [int(x) for x in os.environ.get("AP_CTX", ",".join("0" for _ in lens)).split(",")]
    rounds = int(os.environ.get("AP_ROUNDS", "5"))
    modes = [int(x) for x in os.environ.get("AP_MODES", "0,10,14").split(",")]
    # block orders (attention.hip prefill_block): 1 = head group fastest (default), 0 = (tile, head) grid
    orders = [int(x) for x in os.environ.get("AP_ORDERS", "1").split(",")]
    from rag_llm_k8s_amd.ops import _lib

    def set_order(o):
        _lib.check(_lib.lib().ragk_attn_prefill_set_order(o), "order")
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
    tiles = {}
    for m in modes:
        N.set_prefill_waves(4, pp=m)
        tiles[m] = N.build_prefill_tiles(lens, Hq, Hkv).to(dev)
    keys = [(m, o) for m in modes for o in orders]
    outs = {(m, o): torch.empty(T, Hq * D, device=dev).bfloat16() for m, o in keys}
    times = {k: [] for k in keys}
    for r in range(rounds + 1):
        for m, o in keys:
            N.set_prefill_waves(4, pp=m)
            set_order(o)
            a, b = torch.cuda.Event(True), torch.cuda.Event(True)
            a.record()
            for _ in range(5):
                N.attn_prefill(q, kc, vc, cu, kvl, tiles[m], outs[(m, o)], Hq, Hkv, D, causal=True, paged=True,
                               block_tables=bt)
            b.record()
            b.synchronize()
            if r:
                times[(m, o)].append(a.elapsed_time(b) / 5 * 1e3)
    set_order(1)
    if os.environ.get("AP_STAMP", "1") == "1":
        # stamp build of the software-pipelined kernel (pp mode 7): per wave [fast slots, fast wait +
        # barrier, prologue + warm-up, epilogue] cycles, fast iterations
        for smode, sname, nw in ((7, "4w full", 4), (11, "8w full", 8), (12, "8w no softmax", 8),
                                 (13, "8w no LDS reads", 8)):
            N.set_prefill_waves(4, pp=smode)
            t7 = N.build_prefill_tiles(lens, Hq, Hkv).to(dev)
            grid = t7.shape[0] * Hkv
            dbg = torch.zeros(grid * nw * 6, dtype=torch.int64, device=dev)
            _lib.check(_lib.lib().ragk_attn_set_dbg(dbg.data_ptr()), "dbg")
            o7 = torch.empty(T, Hq * D, device=dev).bfloat16()
            N.attn_prefill(q, kc, vc, cu, kvl, t7, o7, Hq, Hkv, D, causal=True, paged=True, block_tables=bt)
            torch.cuda.synchronize()
            _lib.check(_lib.lib().ragk_attn_set_dbg(None), "dbg")
            d = dbg.view(grid, nw, 6).double().cpu()
            nf = d[:, :, 5].sum()
            print(sname, "v3 stamps per fast iteration: slots %.0f | wait+barrier %.0f cycles (32 MFMA x 32 = 1024);"
                  " per block: prologue+warm-up %.0f, epilogue %.0f cycles; %.1f fast of %.1f tiles per block"
                  % (d[:, :, 0].sum() / nf, d[:, :, 1].sum() / nf, d[:, :, 2].mean(), d[:, :, 3].mean(),
                     d[:, 0, 5].mean(), d[:, 0, 4].mean()))
    if os.environ.get("AP_STAMP_PP", "0") == "1":
        # stamp build (pp mode 5 = variant 4 + s_memtime per phase): mean cycles per segment pair
        N.set_prefill_waves(4, pp=5)
        t5 = N.build_prefill_tiles(lens, Hq, Hkv).to(dev)
        grid = t5.shape[0] * Hkv
        dbg = torch.zeros(grid * 8 * 6, dtype=torch.int64, device=dev)
        _lib.check(_lib.lib().ragk_attn_set_dbg(dbg.data_ptr()), "dbg")
        o5 = torch.empty(T, Hq * D, device=dev).bfloat16()
        N.attn_prefill(q, kc, vc, cu, kvl, t5, o5, Hq, Hkv, D, causal=True, paged=True, block_tables=bt)
        torch.cuda.synchronize()
        _lib.check(_lib.lib().ragk_attn_set_dbg(None), "dbg")
        d = dbg.view(grid, 8, 6).double().cpu()
        for g, name in ((0, "A (waves 0-3)"), (1, "B (waves 4-7)")):
            dd = d[:, 4 * g:4 * g + 4]
            n = dd[:, :, 4].sum()
            m = dd[:, :, :4].sum((0, 1)) / n
            print("stamps %s per tile: MFMA phase %.0f | barrier %.0f | VALU phase %.0f | barrier %.0f = %.0f cycles"
                  " (64 MFMA x 16 = 1024 per wave)" % (name, *m.tolist(), m.sum().item()))
        print("stamp build bit-identical:", torch.equal(o5, outs[keys[0]]))
    def rel(a_, b_):
        return ((a_.float() - b_.float()).norm() / b_.float().norm()).item()
    N.set_prefill_waves(4, pp=0)
    for m, o in keys:
        t = sorted(times[(m, o)])[len(times[(m, o)]) // 2]
        ref = outs[keys[0]]
        same = torch.equal(outs[(m, o)], ref)
        print("lens=%s ctx=%s pp=%d order=%d  %.1f us  %.0f TF  bit-identical=%s rel=%.2e" % (
            lens[0], ctx[0], m, o, t, flops / t / 1e6, same, rel(outs[(m, o)], ref)))


if __name__ == "__main__":
    main()
