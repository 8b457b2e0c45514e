"""Can the batch-32 decode's weight GEMMs gain from weights already in the Infinity Cache, and can a side
branch of a hipGraph put them there while another HBM-bound launch runs?

A stand-in for the decode attention (a 690 MB read, torch's sum over a bf16 tensor) is followed by the
o_proj-shaped split-K slab GEMM (gemm_stream_part, batch 32, 4096 x 4096 bf16). Each form is captured in
a hipGraph over 8 rotating weight copies (the weights come from HBM unless something pulls them in) and
replayed; us per (stand-in + GEMM):

  serial        stand-in, then the GEMM
  prefetched    stand-in, a read of the GEMM's weights, then the GEMM (the cache effect alone)
  side-branch   the weight read on a second stream beside the stand-in (fork / join inside the
                graph), then the GEMM: pays only if the graph runs the branches concurrently
Also the fork / join test alone: two independent 690 MB reads on two streams vs one after the other.
(profiles/mall_prefetch_probe_r6.log also holds a run with a native default-policy "touch" kernel before
the GEMM, not kept: the GEMM took the same time on touched and untouched weight copies.)

  python tools/mall_prefetch_probe.py
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from rag_llm_k8s_amd import _build
    from rag_llm_k8s_amd.ops import native

    _build.build_hip()
    dev = "cuda"
    torch.manual_seed(0)
    big = torch.randn(345 * 1024 * 1024, device=dev, dtype=torch.bfloat16)  # 690 MB
    big2 = torch.randn(345 * 1024 * 1024, device=dev, dtype=torch.bfloat16)
    acc = torch.zeros((), device=dev, dtype=torch.float32)
    acc2 = torch.zeros((), device=dev, dtype=torch.float32)
    ws = [torch.randn(4096, 4096, device=dev).bfloat16() for _ in range(8)]
    x = torch.randn(32, 4096, device=dev).bfloat16()
    sink = torch.zeros(8, device=dev, dtype=torch.float32)
    side = torch.cuda.Stream()

    def standin():
        torch.sum(big, dim=(0,), dtype=torch.float32, out=acc)

    def pull(w, i):
        torch.sum(w.view(-1), dim=(0,), dtype=torch.float32, out=sink[i])

    def serial():
        for w in ws:
            standin()
            native.gemm_stream_part(x, w)

    def prefetched():
        for i, w in enumerate(ws):
            standin()
            pull(w, i)
            native.gemm_stream_part(x, w)

    def side_branch():
        for i, w in enumerate(ws):
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                pull(w, i)
            standin()
            torch.cuda.current_stream().wait_stream(side)
            native.gemm_stream_part(x, w)

    def two_serial():
        for _ in range(4):
            torch.sum(big, dim=(0,), dtype=torch.float32, out=acc)
            torch.sum(big2, dim=(0,), dtype=torch.float32, out=acc2)

    def two_forked():
        for _ in range(4):
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                torch.sum(big2, dim=(0,), dtype=torch.float32, out=acc2)
            torch.sum(big, dim=(0,), dtype=torch.float32, out=acc)
            torch.cuda.current_stream().wait_stream(side)

    def graph_of(fn):
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            fn()
        return g

    def timed(g, n, reps=10):
        g.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            g.replay()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / reps / n * 1e6

    forms = [("serial", serial, 8), ("prefetched", prefetched, 8), ("side-branch", side_branch, 8),
             ("two reads serial", two_serial, 4), ("two reads forked", two_forked, 4)]
    graphs = [(name, graph_of(fn), n) for name, fn, n in forms]
    for rnd in range(3):
        print("round %d: %s" % (rnd, ", ".join("%s %.1f us" % (name, timed(g, n), ) for name, g, n in graphs)),
              flush=True)
    # the stand-in and the GEMM alone
    g1 = graph_of(lambda: [standin() for _ in range(8)])
    g2 = graph_of(lambda: [native.gemm_stream_part(x, w) for w in ws])
    print("stand-in alone %.1f us, GEMM alone (cold weights) %.1f us" % (timed(g1, 8), timed(g2, 8)), flush=True)

if __name__ == "__main__":
    main()
