"""Decode-GEMM microbench (cache-cold: rotates through >= 1.5 GB of weight copies; graph-captured device time): the routed
decode kernels (native.gemm) vs the split-K partial GEMM (native.gemm_part).

python tools/bench_decode_gemm.py [M ...]      DG_TP=8: the shapes of one tensor-parallel rank's shard
(qkv / gate_up split by columns, o_proj / down by K); the gate/up row also times the glds-ring stream
kernel and the plain split-K partials of the packed weight.
"""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rag_llm_k8s_amd.ops import native as N  # noqa: E402

SHAPES = [(6144, 4096, "none", "qkv"), (4096, 4096, "resid", "o_proj"), (4096, 14336, "resid", "down"),
          (14336, 4096, "silu_mul", "gate_up")]


def timeit(fn, ws, reps=5):
    """Device time of fn(w) per call: one call per weight copy (cache-cold), all captured in one hipGraph
    and replayed back to back (launch gaps of a captured decode step included, no host overhead)."""
    for w in ws[:3]:
        fn(w)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(st), torch.cuda.graph(g, stream=st):
        for w in ws:
            fn(w)
    torch.cuda.current_stream().wait_stream(st)
    g.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        s, e = torch.cuda.Event(True), torch.cuda.Event(True)
        s.record()
        g.replay()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e) / len(ws) * 1e-3)
    return sorted(ts)[len(ts) // 2]


def main():
    Ms = [int(a) for a in sys.argv[1:]] or [32]
    tp = int(os.environ.get("DG_TP", "1"))
    shapes = [(n // tp if name in ("qkv", "gate_up") else n, k // tp if name in ("o_proj", "down") else k, epi, name)
              for (n, k, epi, name) in SHAPES]
    torch.manual_seed(0)
    for M in Ms:
        for (n, k, epi, name) in shapes:
            wn = 2 * n if epi == "silu_mul" else n
            x = torch.randn(M, k, device="cuda").bfloat16()
            ncopy = max(2, -(-(1536 << 20) // (wn * k * 2)))
            ws = [(torch.randn(wn, k, device="cuda") / math.sqrt(k)).bfloat16() for _ in range(ncopy)]
            r = torch.randn(M, n, device="cuda").bfloat16() if epi == "resid" else None
            out = torch.empty(M, n, device="cuda").bfloat16()
            t0 = timeit(lambda w: N.gemm(x, w, resid=r, epi=epi, out=out), ws)
            row = "M=%d %-8s N=%-6d K=%-6d routed %6.1f us %5.2f TB/s" % (M, name, wn, k, t0 * 1e6,
                                                                         wn * k * 2 / t0 / 1e12)
            if epi == "silu_mul":
                t5 = timeit(lambda w: N.gemm(x, w, epi=epi, out=out, path=5), ws)
                row += " | stream %6.1f us" % (t5 * 1e6)
            ks, S = N.gemm_part_slabs(M, wn, k)
            if S:
                P = torch.empty(S, M, wn, dtype=torch.float32, device="cuda")
                t1 = timeit(lambda w: N.gemm_part(x, w, out=P), ws)
                row += " | part(ks=%d,S=%d) %6.1f us %5.2f TB/s" % (ks, S, t1 * 1e6, wn * k * 2 / t1 / 1e12)
                for ks2 in (4, 8, 16, 32):
                    k2, S2 = N.gemm_part_slabs(M, wn, k, ks2)
                    if S2 and ks2 != ks and 16 * ((M + 15) // 16) * ks2 * 128 <= 128 * 1024:
                        P2 = torch.empty(S2, M, wn, dtype=torch.float32, device="cuda")
                        t2 = timeit(lambda w: N.gemm_part(x, w, out=P2, ks=ks2), ws)
                        row += " | ks=%d %6.1f us" % (ks2, t2 * 1e6)
            print(row, flush=True)
            del ws


if __name__ == "__main__":
    main()
