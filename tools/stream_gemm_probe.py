"""Decode SiLU*up (gate/up) stream GEMM in isolation: Llama-3.1-8B packed [28672, 4096] weights, M rows,
NC rotating weight copies (>= 1.8 GB: nothing from the Infinity Cache), hipGraph replays. us per launch and
TB/s of weights, for the kernel (base) and its diagnostic builds (gemm_stream.hip DG): diag = the LDS-DMA
ring, waits and barriers without fragment reads / MFMA; diag_nox = also no activation staging; diag_nobar =
also no per-stage barrier.

  SP_M=32 SP_VARIANTS=base,diag,base,diag python tools/stream_gemm_probe.py
"""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from rag_llm_k8s_amd import _build
    from rag_llm_k8s_amd.ops import _lib, native

    _build.build_all()
    M = int(os.environ.get("SP_M", "32"))
    NC = int(os.environ.get("SP_NC", "8"))
    reps = int(os.environ.get("SP_REPS", "10"))
    I, H = 14336, 4096
    dev = "cuda"
    x = torch.randn(M, H, device=dev).bfloat16()
    ws = [(torch.randn(2 * I, H, device=dev) / math.sqrt(H)).bfloat16() for _ in range(NC)]
    out = torch.empty(M, I, device=dev).bfloat16()
    L = _lib.lib()
    nbytes = 2 * I * H * 2

    def run():
        for w in ws:
            native.gemm(x, w, epi="silu_mul", out=out, path=5)

    graphs = {}
    for v in [v for v in os.environ.get("SP_VARIANTS", "base,diag,base,diag").split(",") if v]:
        if v not in graphs:
            L.ragk_gemm_stream_set_diag({"diag": 1, "diag_nox": 2, "diag_nobar": 3}.get(v, 0))
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                run()
            torch.cuda.current_stream().wait_stream(s)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                run()
            graphs[v] = g
            L.ragk_gemm_stream_set_diag(0)
        g = graphs[v]
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / reps / NC
        print("M=%d %-5s %7.1f us per launch  %.2f TB/s of weights" % (M, v, us, nbytes / us / 1e6), flush=True)


if __name__ == "__main__":
    main()
