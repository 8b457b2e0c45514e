"""Decode projection A/B inside hipGraphs (no launch overhead), weights cold (8 rotating layers):
the engine's split-K partial GEMM + its consumer vs the glds-ring stream GEMM (split S) + a plain
row kernel, for the Llama-3.1-8B o_proj / down (+ residual + RMSNorm) and qkv shapes at M = 1 / 32.

  python tools/decode_gemm_graph_ab.py            # prints one JSON line per (shape, M, variant)
"""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rag_llm_k8s_amd.ops import native as N  # noqa: E402

LAYERS = 8
H = 4096


def timed_graph(body, reps=5):
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        body()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        body()
    g.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(True), torch.cuda.Event(True)
        a.record()
        g.replay()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3 / LAYERS)
    return sorted(ts)[reps // 2]


def main():
    torch.manual_seed(0)
    res = []
    shapes = [("o_proj", 4096, 4096), ("down", 4096, 14336), ("qkv", 6144, 4096)]
    ms = [int(v) for v in os.environ.get("AB_M", "1,32").split(",")]
    only = os.environ.get("AB_VARIANTS", "")
    for (name, n, k) in shapes:
        ws = [(torch.randn(n, k, device="cuda") / math.sqrt(k)).bfloat16() for _ in range(LAYERS)]
        nw = (torch.ones(H, device="cuda")).bfloat16()
        mb = n * k * 2 / 2 ** 20
        for M in ms:
            x = torch.randn(M, k, device="cuda").bfloat16()
            h = torch.randn(M, H, device="cuda").bfloat16()
            out = torch.empty(M, n, device="cuda").bfloat16()
            variants = {}
            if name == "qkv":
                variants["part"] = lambda: [N.gemm_part(x, w) for w in ws]
                for S in (1, 2, 4, 8):
                    variants["stream_S%d" % S] = (lambda S=S: [N.gemm(x, w, out=out, path=5) for w in ws], S)
                variants["default"] = lambda: [N.gemm(x, w, out=out) for w in ws]
            else:
                def part_pair():
                    for w in ws:
                        P = N.gemm_part(x, w)
                        N.add_partials_rmsnorm(P, h, nw, 1e-5)
                variants["part+consumer"] = part_pair
                for S in (1, 2, 4, 8):
                    def stream_pair():
                        for w in ws:
                            N.gemm(x, w, resid=h, epi="resid", out=h, path=5)
                            N.rmsnorm(h, nw, 1e-5)
                    variants["stream_S%d+rmsnorm" % S] = (stream_pair, S)

                def default_pair():
                    for w in ws:
                        N.gemm(x, w, resid=h, epi="resid", out=h)
                        N.rmsnorm(h, nw, 1e-5)
                variants["default+rmsnorm"] = default_pair
            for vname, v in variants.items():
                if only and not any(vname.startswith(o) for o in only.split(",")):
                    continue
                S = 0
                if isinstance(v, tuple):
                    v, S = v
                if S and (k // 64) % S:
                    continue
                N.STREAM_S_OVERRIDE = S
                try:
                    us = timed_graph(v)
                except Exception as ex:
                    print(json.dumps(dict(name=name, M=M, variant=vname, error=str(ex)[:120])), flush=True)
                    continue
                finally:
                    N.STREAM_S_OVERRIDE = 0
                row = dict(name=name, M=M, variant=vname, us=round(us, 2), TBps=round(mb * 2 ** 20 / us / 1e6, 2))
                res.append(row)
                print(json.dumps(row), flush=True)
        del ws
        torch.cuda.empty_cache()
    os.makedirs("gpurun_out", exist_ok=True)
    json.dump(res, open("gpurun_out/decode_gemm_graph_ab.json", "w"), indent=1)


if __name__ == "__main__":
    main()
