"""Is gemm_w4's per-tile epilogue bandwidth-bound? Stamped build (ragk_gemm_w4_diag variant 0), the
persistent grid capped at G blocks: if the epilogue's cycles per tile shrink as G falls, the cost is the
lock-step store burst of all CUs (G x 128 KiB at once), not the store issue of one block.

  python tools/gemm_epi_probe.py      # one line per (shape, G)
"""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rag_llm_k8s_amd.ops import _lib  # noqa: E402
from rag_llm_k8s_amd.ops._lib import check, stream_ptr  # noqa: E402

L = _lib.lib()
GRIDS = [int(g) for g in os.environ.get("EP_GRIDS", "256,128,64,32").split(",")]
# M x N x K; a small N packs a tile's 256 output rows into a contiguous 128 KiB (TLB / page footprint test)
SHAPES = [tuple(int(v) for v in sh.split("x"))
          for sh in os.environ.get("EP_SHAPES", "32768x4096x4096,32768x28672x4096").split(",")]
VARIANT = int(os.environ.get("EP_VARIANT", "0"))

torch.manual_seed(0)
for (M, N, K) in SHAPES:
    x = torch.rand(M, K, device="cuda").sub_(0.5).bfloat16()
    w = (torch.rand(N, K, device="cuda").sub_(0.5) / math.sqrt(K)).bfloat16()
    out = torch.empty(M, N, device="cuda").bfloat16()
    nwg = (M // 256) * (N // 256)
    dbg = torch.zeros(nwg * 4 * 8, dtype=torch.int64, device="cuda")
    for G in GRIDS:
        check(L.ragk_gemm_w4_set_grid(G), "grid")
        for stamp in (0, 1):
            for _ in range(2):
                dbg.zero_()
                s, e = torch.cuda.Event(True), torch.cuda.Event(True)
                s.record()
                check(L.ragk_gemm_w4_diag(VARIANT, stamp, x.data_ptr(), K, w.data_ptr(), K, out.data_ptr(), N, M, N, K,
                                          dbg.data_ptr(), stream_ptr()), "w4_diag")
                e.record()
                torch.cuda.synchronize()
            if stamp == 0:
                us = s.elapsed_time(e) * 1e3
                continue
            d = dbg.view(nwg, 4, 8).double().cpu()
            d = d[d[:, 0, 5] > 0]
            tiles = d[:, :, 5] / max(1, K // 64 - (3 if VARIANT == 22 else 2))
            lp = (d[:, :, 6] / tiles).median().item()
            ep = (d[:, :, 7] / tiles).median().item()
            print("M=%d N=%d K=%d G=%d  %.0f us (%.0f TF/s at this grid)  per tile: loop %.0f cycles, epilogue %.0f "
                  "(%.1f%%)" % (M, N, K, G, us, 2.0 * M * N * K / us / 1e6, lp, ep, 100 * ep / (lp + ep)), flush=True)
    check(L.ragk_gemm_w4_set_grid(-1), "grid")
    del x, w, out
    torch.cuda.empty_cache()
