"""Per-tile fixed cost of a prefill GEMM kernel: time vs K at fixed M, N (T = a + b*K)."""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rag_llm_k8s_amd.ops import native as N  # noqa: E402


def timeit(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(True), torch.cuda.Event(True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e-3


M, Nn = 16384, 4096
for path in (6, "torch"):
    pts = []
    for K in (1024, 2048, 4096, 8192):
        x = torch.randn(M, K, device="cuda").bfloat16()
        w = (torch.randn(Nn, K, device="cuda") / math.sqrt(K)).bfloat16()
        out = torch.empty(M, Nn, device="cuda").bfloat16()
        fn = (lambda: torch.matmul(x, w.t())) if path == "torch" else (lambda: N.gemm(x, w, out=out, path=path))
        t = min(timeit(fn) for _ in range(3))
        pts.append((K, t))
        print("path=%s K=%d %.1f us %.1f TF" % (path, K, t * 1e6, 2 * M * Nn * K / t / 1e12), flush=True)
    (k0, t0), (k1, t1) = pts[0], pts[-1]
    b = (t1 - t0) / (k1 - k0)
    print("path=%s fixed per launch %.1f us (%.1f us per tile round), slope %.1f us per 1k K" % (
        path, (t0 - b * k0) * 1e6, (t0 - b * k0) * 1e6 / 4, b * 1e9), flush=True)
