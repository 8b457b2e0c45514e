"""Sweep the split-K factor of the stream decode GEMM (gemm_stream.hip) on Llama-8B decode shapes."""
import json
import math
import sys

import torch

sys.path.insert(0, ".")
from rag_llm_k8s_amd.ops import fp8 as F8  # noqa: E402
from rag_llm_k8s_amd.ops import native as N  # noqa: E402


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e-3


rows = []
for M in (1, 32, 64):
    for (Nn, K, epi, name) in [(6144, 4096, "none", "qkv"), (4096, 4096, "resid", "o_proj"),
                               (14336, 4096, "silu_mul", "gate_up"), (4096, 14336, "resid", "down")]:
        wn = 2 * Nn if epi == "silu_mul" else Nn
        ncopy = max(2, -(-(1536 << 20) // (wn * K * 2)))
        ws = [(torch.randn(wn, K, device="cuda") / math.sqrt(K)).bfloat16() for _ in range(ncopy)]
        w8 = [F8.quantize_weight(w) for w in ws]
        x = torch.randn(M, K, device="cuda").bfloat16()
        r = torch.randn(M, Nn, device="cuda").bfloat16() if epi == "resid" else None
        out = torch.empty(M, Nn, device="cuda").bfloat16()
        it = [0]

        def nxt(lst):
            it[0] = (it[0] + 1) % ncopy
            return lst[it[0]]

        res = dict(M=M, name=name)
        for S in (1, 2, 4, 8):
            if (K // 64) % S or S * M * wn > (96 << 20) // 4:
                continue
            N.STREAM_S_OVERRIDE = S
            t = timeit(lambda: N.gemm(x, nxt(ws), resid=r, epi=epi, out=out, path=5), ncopy * 4)
            res["bf16_S%d_TBps" % S] = round(wn * K * 2 / t / 1e12, 2)
            if (K // 128) % S == 0:
                t = timeit(lambda: N.gemm_fp8(x, nxt(w8), resid=r, epi=epi, out=out), ncopy * 4)
                res["fp8_S%d_TBps" % S] = round(wn * K / t / 1e12, 2)
        N.STREAM_S_OVERRIDE = 0
        t = timeit(lambda: N.gemm(x, nxt(ws), resid=r, epi=epi, out=out, path=1 if M <= 64 else 0), ncopy * 4)
        res["v1_TBps"] = round(wn * K * 2 / t / 1e12, 2)
        rows.append(res)
        print(res, flush=True)
        json.dump(rows, open("gpurun_out/tune_stream.json", "w"), indent=1)
        del ws, w8
json.dump(rows, open("gpurun_out/tune_stream.json", "w"), indent=1)
