"""Flat L2 top-k (csrc/kernels/search.hip) on one MI355X: wall time per search call (CUDA events,
median of 20, index warm in HBM/MALL as in serving; includes the host-side call), the device time
(the call captured in a hipGraph, 20 replays back to back: the two kernels and their launch gap) and
the effective read rate of the index at the device time.
Shapes of the SURVEY V2 targets: 10k x 384 (MiniLM, bench corpus) at nq = 1 / 32, 1M x 1024 (bge
scale) at nq = 1 / 32. Prints one JSON line per shape."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rag_llm_k8s_amd.ops import native as N  # noqa: E402


def timed(fn, iters=20, warmup=3):
    for _ in range(warmup):
        fn()
    ts = []
    for _ in range(iters):
        a, b = torch.cuda.Event(True), torch.cuda.Event(True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return sorted(ts)[len(ts) // 2]


def main():
    shapes = [(10000, 384, 1, 4), (10000, 384, 32, 4), (10000, 1024, 1, 5), (1000000, 1024, 1, 5),
              (1000000, 1024, 32, 5), (1000000, 384, 1, 4)]
    if os.environ.get("SB_SHAPES"):  # e.g. "10000x384x32x4,..."
        shapes = [tuple(int(v) for v in sh.split("x")) for sh in os.environ["SB_SHAPES"].split(",")]
    for n, d, nq, k in shapes:
        torch.manual_seed(0)
        xt = torch.randn(d, n, device="cuda")
        q = torch.randn(nq, d, device="cuda")
        us = timed(lambda: N.l2_search(xt, n, n, q, k))
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            N.l2_search(xt, n, n, q, k)  # workspace for this stream
            with torch.cuda.graph(g, stream=s):
                for _ in range(20):
                    N.l2_search(xt, n, n, q, k)
        torch.cuda.current_stream().wait_stream(s)
        dev = timed(g.replay, iters=10, warmup=2) / 20
        # correctness spot check vs torch (fp32 direct form) on a sample of queries
        ref = torch.cdist(q[:1].double(), xt.t().double()).pow(2)
        ri = ref.topk(k, largest=False).indices.cpu()
        D, I = N.l2_search(xt, n, n, q, k)
        print(json.dumps(dict(N=n, d=d, nq=nq, k=k, us=round(us, 1), dev_us=round(dev, 1),
                              TBps=round(n * d * 4 / dev / 1e6, 2),
                              top1_ok=bool(int(I[0, 0]) == int(ri[0, 0])))), flush=True)
        del xt
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
