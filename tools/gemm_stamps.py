"""gemm_w4 K-loop tuning: segment-split variants A/B'd in interleaved rounds (clean builds), plus the
wave-cycle anatomy of each from the s_memtime stamp build (ragk_gemm_w4_diag)."""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rag_llm_k8s_amd.ops import _lib  # noqa: E402
from rag_llm_k8s_amd.ops._lib import check, stream_ptr  # noqa: E402

VARIANTS = {0: (32, 16), 1: (24, 24), 3: (32, 32), 6: (32, 0), 7: (24, 0), 8: (40, 0)}
L = _lib.lib()


def run(v, stamp, x, w, out, M, N, K, dbg):
    check(L.ragk_gemm_w4_diag(v, stamp, x.data_ptr(), K, w.data_ptr(), K, out.data_ptr(), N, M, N, K,
                              dbg.data_ptr() if dbg is not None else None, stream_ptr()), "w4_diag")


def timed(fn, iters=5):
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e-3


for (M, N, K) in [(16384, 4096, 4096), (16384, 6144, 4096), (16384, 4096, 14336)]:
    x = torch.randn(M, K, device="cuda").bfloat16()
    w = (torch.randn(N, K, device="cuda") / math.sqrt(K)).bfloat16()
    out = torch.empty(M, N, device="cuda").bfloat16()
    ref = x.float() @ w.float().t()
    nwg = (M // 256) * (N // 256)
    dbg = torch.zeros(nwg * 4 * 8, dtype=torch.int64, device="cuda")
    ts = {v: [] for v in VARIANTS}
    for v in VARIANTS:
        run(v, 0, x, w, out, M, N, K, None)
        err = ((out.float() - ref).norm() / ref.norm()).item()
        assert err < 5e-3, (v, err)
    for _ in range(4):
        for v in VARIANTS:
            ts[v].append(timed(lambda: run(v, 0, x, w, out, M, N, K, None)))
    tt = timed(lambda: torch.matmul(x, w.t()))
    print("M=%d N=%d K=%d  hipBLASLt %.1f us %.0f TF" % (M, N, K, tt * 1e6, 2 * M * N * K / tt / 1e12))
    for v, (s1, s3) in VARIANTS.items():
        t = sorted(ts[v])[len(ts[v]) // 2]
        run(v, 1, x, w, out, M, N, K, dbg)
        torch.cuda.synchronize()
        d = dbg.view(nwg, 4, 8).double().cpu()
        d = d[d[:, 0, 5] > 0]  # persistent grid: only blocks that ran
        it = d[:, :, 5]
        per = (d[:, :, :5] / it.unsqueeze(-1)).reshape(-1, 5).median(0).values.tolist()
        print("  v%d S1=%d S3=%d  %.1f us %.0f TF | stamped cycles/K-tile: seg1 %.0f b1 %.0f seg2 %.0f b2 %.0f "
              "seg3 %.0f = %.0f" % (v, s1, s3, t * 1e6, 2 * M * N * K / t / 1e12, per[0], per[1], per[2], per[3],
                                    per[4] - sum(per[:4]), per[4]), flush=True)
