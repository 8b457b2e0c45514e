"""Prefill GEMM routing probe: the measured gemm_w4-vs-hipBLASLt choice (ops/native.py
_prefer_blaslt) on the Llama-3.1-8B prefill shapes at M = 32768, plus an end-to-end timing of the
chosen route against gemm_w4 (in place on the residual, as the model calls it)."""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rag_llm_k8s_amd.ops import native as N  # noqa: E402
from rag_llm_k8s_amd.ops import reference as R  # noqa: E402

M = int(os.environ.get("PROBE_M", "32768"))
torch.manual_seed(0)
for n, k, epi in [(6144, 4096, "none"), (4096, 4096, "resid"), (14336, 4096, "silu_mul"), (4096, 14336, "resid")]:
    x = torch.randn(M, k, device="cuda").bfloat16()
    w = (torch.randn(2 * n if epi == "silu_mul" else n, k, device="cuda") / math.sqrt(k)).bfloat16()
    h = torch.randn(M, n, device="cuda").bfloat16()
    kw = dict(resid=h, epi="resid", out=h) if epi == "resid" else dict(epi=epi)
    N.gemm(x, w, **kw)
    t = N._blaslt_times.get((w.shape[0], k, epi, max(0, M.bit_length() - 1)))
    route = {}
    for name, path in (("auto", None), ("w4", 6)):
        ev = [torch.cuda.Event(True) for _ in range(2)]
        ev[0].record()
        for _ in range(5):
            N.gemm(x, w, path=path, **kw)
        ev[1].record()
        torch.cuda.synchronize()
        route[name] = ev[0].elapsed_time(ev[1]) / 5 * 1e3
    print("N=%d K=%d epi=%s: probe %s | routed %.1f us, w4 %.1f us" % (
        n, k, epi, "w4 %.1f us vs hipBLASLt %.1f us" % (t[1] * 1e3, t[2] * 1e3) if t else "n/a", route["auto"],
        route["w4"]), flush=True)
