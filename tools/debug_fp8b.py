import math
import torch
from rag_llm_k8s_amd.ops import fp8 as F8
from rag_llm_k8s_amd.ops import native as N

M, Nn, K = 65, 768, 1024
torch.manual_seed(M + Nn)
x = torch.randn(M, K, device="cuda").bfloat16()
w = (torch.randn(Nn, K, device="cuda") / math.sqrt(K)).bfloat16()
wq = F8.quantize_weight(w)
q, s = N.quant_fp8_rows(x)
rq, rs = F8.quantize_rows(x)
print("scale diff rows", (s - rs).abs().max().item(), "bytes diff per row", (q.view(torch.uint8) != rq.view(torch.uint8)).sum(1).tolist()[-5:])
y = N.gemm_fp8(x, wq, out_f32=True)
ref = F8.reference_linear(x, wq, out_f32=True)
err = ((y - ref).norm(dim=1) / ref.norm(dim=1))
print("per-row rel err (last 6)", [round(v, 4) for v in err[-6:].tolist()], "max row", int(err.argmax()))
for M2 in (64, 65, 66, 100, 127, 128, 129, 200):
    xx = torch.randn(M2, K, device="cuda").bfloat16()
    y = N.gemm_fp8(xx, wq, out_f32=True)
    ref = F8.reference_linear(xx, wq, out_f32=True)
    err = ((y - ref).norm(dim=1) / ref.norm(dim=1))
    bad = (err > 1e-3).nonzero().flatten().tolist()
    print("M", M2, "max err", round(err.max().item(), 5), "bad rows", bad[:10], len(bad))
