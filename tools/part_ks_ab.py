"""Split-K partial decode GEMM (gemm_part.hip) slice-size A/B at M=32, cache-cold (weights rotate over
>= 1.5 GB of copies), interleaved rounds in one process. Prints us and TB/s per (shape, ks_steps); the
grid is N/64 x K/(64*ks) blocks of 512 threads, one per CU when the activation slice exceeds 80 KB."""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rag_llm_k8s_amd.ops import native as N  # noqa: E402

M = int(os.environ.get("PART_M", "32"))
SHAPES = [("qkv", 6144, 4096, (8, 16, 32)), ("o_proj", 4096, 4096, (8, 16, 32)),
          ("down", 4096, 14336, (14, 16, 28, 32)), ("gate_up", 28672, 4096, (8, 16, 32))]
if os.environ.get("PART_SHAPES"):
    SHAPES = [sh for sh in SHAPES if sh[0] in os.environ["PART_SHAPES"].split(",")]
FP8 = os.environ.get("PART_FP8", "0") == "1"
torch.manual_seed(0)
for name, n, k, kss in SHAPES:
    x = torch.randn(M, k, device="cuda").bfloat16()
    ncopy = max(2, -(-(1536 << 20) // (n * k * 2)))
    ws = [(torch.randn(n, k, device="cuda") / math.sqrt(k)).bfloat16() for _ in range(ncopy)]
    if FP8:
        from rag_llm_k8s_amd.ops.fp8 import quantize_weight

        ws = [quantize_weight(w) for w in ws]
    ref = x.float() @ (ws[0].dequant() if FP8 else ws[0].float()).t()
    ts = {ks: [] for ks in kss}
    outs = {ks: torch.empty((k // (64 * ks), M, n), dtype=torch.float32, device="cuda") for ks in kss}
    for ks in kss:
        P = N.gemm_part(x, ws[0], out=outs[ks], ks=ks)
        err = ((P.sum(0) - ref).norm() / ref.norm()).item()
        assert err < 1e-2, (name, ks, err)
    for _ in range(5):
        for ks in kss:
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(True), torch.cuda.Event(True)
            s.record()
            for i in range(2 * ncopy):
                N.gemm_part(x, ws[i % ncopy], out=outs[ks], ks=ks)
            e.record()
            torch.cuda.synchronize()
            ts[ks].append(s.elapsed_time(e) / (2 * ncopy) * 1e-3)
    for ks in kss:
        t = sorted(ts[ks])[2]
        blocks = (n // 64) * (k // (64 * ks))
        print("M=%d %-7s N=%d K=%d ks=%2d blocks=%4d %s %.1f us  %.2f TB/s" % (
            M, name, n, k, ks, blocks, "fp8" if FP8 else "bf16", t * 1e6, n * k * (1 if FP8 else 2) / t / 1e12),
            flush=True)
