"""Decode-GEMM microbench (cache-cold: rotates through >= 1.5 GB of weight copies): the routed
decode kernels (native.gemm) vs the split-K partial GEMM (native.gemm_part).

python tools/bench_decode_gemm.py [M ...]
"""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rag_llm_k8s_amd.ops import native as N  # noqa: E402

SHAPES = [(6144, 4096, "none", "qkv"), (4096, 4096, "resid", "o_proj"), (4096, 14336, "resid", "down"),
          (14336, 4096, "silu_mul", "gate_up")]


def timeit(fn, iters=40):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e-3


def main():
    Ms = [int(a) for a in sys.argv[1:]] or [32]
    torch.manual_seed(0)
    for M in Ms:
        for (n, k, epi, name) in SHAPES:
            wn = 2 * n if epi == "silu_mul" else n
            x = torch.randn(M, k, device="cuda").bfloat16()
            ncopy = max(2, -(-(1536 << 20) // (wn * k * 2)))
            ws = [(torch.randn(wn, k, device="cuda") / math.sqrt(k)).bfloat16() for _ in range(ncopy)]
            r = torch.randn(M, n, device="cuda").bfloat16() if epi == "resid" else None
            out = torch.empty(M, n, device="cuda").bfloat16()
            it = [0]

            def nxt():
                it[0] = (it[0] + 1) % ncopy
                return ws[it[0]]

            t0 = timeit(lambda: N.gemm(x, nxt(), resid=r, epi=epi, out=out))
            row = "M=%d %-8s N=%-6d K=%-6d routed %6.1f us %5.2f TB/s" % (M, name, wn, k, t0 * 1e6,
                                                                         wn * k * 2 / t0 / 1e12)
            if epi != "silu_mul":
                ks, S = N.gemm_part_slabs(M, wn, k)
                P = torch.empty(S, M, wn, dtype=torch.float32, device="cuda")
                t1 = timeit(lambda: N.gemm_part(x, nxt(), out=P))
                row += " | part(ks=%d,S=%d) %6.1f us %5.2f TB/s" % (ks, S, t1 * 1e6, wn * k * 2 / t1 / 1e12)
                for ks2 in (8, 16, 32):
                    k2, S2 = N.gemm_part_slabs(M, wn, k, ks2)
                    if S2 and ks2 != ks and 16 * ((M + 15) // 16) * ks2 * 128 <= 128 * 1024:
                        P2 = torch.empty(S2, M, wn, dtype=torch.float32, device="cuda")
                        t2 = timeit(lambda: N.gemm_part(x, nxt(), out=P2, ks=ks2))
                        row += " | ks=%d %6.1f us" % (ks2, t2 * 1e6)
            print(row, flush=True)
            del ws


if __name__ == "__main__":
    main()
