"""gemm_w4 K-loop schedule A/B (interleaved rounds, one process, random operands) on the
Llama-3.1-8B prefill shapes at M = 32768, against hipBLASLt (torch.matmul) as the yardstick.

Variants (ragk_gemm_w4_diag): 0 = production w4_iter (S1=32, S3=16); 9..13 = w4_iter2 (spread
reads, barrier A at BA, one DMA per DS MFMAs): 9 (32,4) 10 (32,5) 11 (32,6) 12 (48,4) 13 (16,6).
Prints us / TF per variant and the stamped cycles per K-tile of w4_iter2 (read phase, barrier A,
DMA phase, barrier B, rest)."""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rag_llm_k8s_amd.ops import _lib  # noqa: E402
from rag_llm_k8s_amd.ops._lib import check, stream_ptr  # noqa: E402

VARIANTS = [int(v) for v in os.environ.get("AB_VARIANTS", "0,14,15,16,17").split(",")]
M = int(os.environ.get("AB_M", "32768"))
ROUNDS = int(os.environ.get("AB_ROUNDS", "5"))
SHAPES = [(6144, 4096), (4096, 4096), (4096, 14336), (28672, 4096)]
L = _lib.lib()


def run(v, stamp, x, w, out, N, K, dbg):
    check(L.ragk_gemm_w4_diag(v, stamp, x.data_ptr(), K, w.data_ptr(), K, out.data_ptr(), N, M, N, K,
                              dbg.data_ptr() if dbg is not None else None, stream_ptr()), "w4_diag")


def timed(fn, iters=3):
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e-3


torch.manual_seed(0)
for (N, K) in SHAPES:
    x = torch.rand(M, K, device="cuda").sub_(0.5).bfloat16()
    w = (torch.rand(N, K, device="cuda").sub_(0.5) / math.sqrt(K)).bfloat16()
    out = torch.empty(M, N, device="cuda").bfloat16()
    ref = torch.matmul(x, w.t())
    for v in VARIANTS:
        run(v, 0, x, w, out, N, K, None)
        err = ((out.float() - ref.float()).norm() / ref.float().norm()).item()
        assert err < 1e-2, (v, N, K, err)
    ts = {v: [] for v in VARIANTS + ["blaslt"]}
    for _ in range(ROUNDS):
        for v in VARIANTS:
            ts[v].append(timed(lambda: run(v, 0, x, w, out, N, K, None)))
        ts["blaslt"].append(timed(lambda: torch.matmul(x, w.t(), out=out)))
    fl = 2.0 * M * N * K
    line = "M=%d N=%d K=%d" % (M, N, K)
    for v in VARIANTS + ["blaslt"]:
        t = sorted(ts[v])[len(ts[v]) // 2]
        line += " | %s %.0fus %.0fTF" % (v, t * 1e6, fl / t / 1e12)
    print(line, flush=True)
    nwg = (M // 256) * (N // 256)
    dbg = torch.zeros(nwg * 4 * 8, dtype=torch.int64, device="cuda")
    for v in VARIANTS:
        dbg.zero_()
        run(v, 1, x, w, out, N, K, dbg)
        torch.cuda.synchronize()
        d = dbg.view(nwg, 4, 8).double().cpu()
        d = d[d[:, 0, 5] > 0]
        it = d[:, :, 5]
        per = (d[:, :, :5] / it.unsqueeze(-1)).reshape(-1, 5).median(0).values.tolist()
        tiles = it / max(1, K // 64 - 2)
        lp = (d[:, :, 6] / tiles).median().item()
        ep = (d[:, :, 7] / tiles).median().item()
        print("   v%d stamped cycles/K-tile: %.0f %.0f %.0f %.0f rest %.0f = %.0f (ideal 2048) | per tile: loop %.0f "
              "(%.0f/K-tile) epilogue %.0f (%.1f%%)" % (v, per[0], per[1], per[2], per[3], per[4] - sum(per[:4]),
                                                        per[4], lp, lp / (K // 64), ep, 100 * ep / (lp + ep)),
              flush=True)
