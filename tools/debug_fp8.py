"""Diagnose the fp8 GEMM kernels with unit-vector activations (GPU)."""
import torch

from rag_llm_k8s_amd.ops import fp8 as F8
from rag_llm_k8s_amd.ops import native as N

torch.manual_seed(0)
K, Nn = 128, 16
w = torch.randn(Nn, K, device="cuda").bfloat16()
wq = F8.quantize_weight(w)
wd = wq.dequant()
for M in (1, 64, 128):
    x = torch.zeros(M, K, device="cuda").bfloat16()
    for m in range(M):
        x[m, m % K] = 1.0
    y = N.gemm_fp8(x, wq, out_f32=True)
    ref = x.float() @ wd.t()
    print("M", M, "max err", (y - ref).abs().max().item())
    # which column of wd does y[m] match?
    for m in list(range(min(M, 8))) + [33, 64, 100]:
        if m >= M:
            continue
        d = (wd.t()[:, :] - y[m][None, :]).abs().sum(1)  # [K]
        print("  row", m, "expects k", m % K, "best k", int(d.argmin()), "dist", float(d.min()),
              "y0..3", [round(v, 3) for v in y[m, :4].tolist()], "ref0..3", [round(v, 3) for v in ref[m, :4].tolist()])
# conversion check: weight row of known values
vals = torch.tensor([0.0, 1.0, -1.0, 0.5, 2.0, 448.0, -448.0, 0.015625] * 16, device="cuda")
w2 = vals.repeat(16, 1).bfloat16()
wq2 = F8.quantize_weight(w2)
print("w8 bytes", wq2.w8.view(torch.uint8)[0, :8].tolist(), "scale", wq2.scale[0].item())
x = torch.zeros(1, 128, device="cuda").bfloat16()
for k in range(8):
    x.zero_()
    x[0, k] = 1.0
    print("k", k, "val", vals[k].item(), "got", N.gemm_fp8(x, wq2, out_f32=True)[0, 0].item())
