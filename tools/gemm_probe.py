"""Prefill-GEMM probe for rocprofv3 PMC passes: our ping-pong kernel vs hipBLASLt (torch.matmul) on
the Llama-3.1-8B prefill shapes, random operands. Short enough (~2 s of GPU) for one counter pass.

  rocprofv3 --pmc SQ_WAVE_CYCLES ... --kernel-trace -d gpurun_out/gp -- python3 tools/gemm_probe.py
"""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rag_llm_k8s_amd.ops import native as N  # noqa: E402

SHAPES = [(6144, 4096, "none"), (4096, 4096, "resid"), (14336, 4096, "silu_mul"), (4096, 14336, "resid"),
          (4096, 4096, "none"), (4096, 14336, "none"),
          # K scaling (fixed per-tile cost = prologue + epilogue): 6-7 vs 0, 8-9 vs 1
          (6144, 2048, "none"), (6144, 8192, "none"), (4096, 2048, "resid"), (4096, 8192, "resid")]


def main():
    M = int(os.environ.get("PROBE_M", "16384"))
    iters = int(os.environ.get("PROBE_ITERS", "5"))
    rounds = int(os.environ.get("PROBE_ROUNDS", "3"))
    paths = os.environ.get("PROBE_PATHS", "2,torch").split(",")
    shapes = [SHAPES[int(i)] for i in os.environ.get("PROBE_SHAPES", "0,1,2,3").split(",")]
    torch.manual_seed(0)
    for (n, k, epi) in shapes:
        wn = 2 * n if epi == "silu_mul" else n
        x = torch.randn(M, k, device="cuda").bfloat16()
        w = (torch.randn(wn, k, device="cuda") / math.sqrt(k)).bfloat16()
        r = torch.randn(M, n, device="cuda").bfloat16() if epi == "resid" else None
        out = torch.empty(M, n, device="cuda").bfloat16()
        fns = {}
        for p in paths:
            if p == "torch":
                fns[p] = lambda: torch.matmul(x, w.t())  # noqa: E731
            elif p == "blas":  # the library route of ops.native (resid: in-place addmm, beta = 1)
                h = r.clone() if r is not None else None
                if epi == "silu_mul":  # no library epilogue: the plain GEMM of both halves
                    o2 = torch.empty(M, wn, device="cuda").bfloat16()
                    fns[p] = lambda o2=o2: N._gemm_blas(x, w, None, o2, "none")  # noqa: E731
                else:
                    fns[p] = lambda h=h: N._gemm_blas(x, w, h, h if h is not None else out, epi)  # noqa: E731
            elif "@" in p:  # "6@0": gemm_w4 with the persistent grid set to 0 (one block per tile)
                path, grid = (int(v) for v in p.split("@"))

                def fn(path=path, grid=grid):
                    N.set_w4_grid(grid)
                    N.gemm(x, w, resid=r, epi=epi, out=out, path=path)
                    N.set_w4_grid(-1)
                fns[p] = fn
            else:
                fns[p] = lambda p=p: N.gemm(x, w, resid=r, epi=epi, out=out, path=int(p))  # noqa: E731
            fns[p]()
        times = {p: [] for p in paths}
        for _ in range(rounds):  # interleaved rounds (one process, same data): A/B deltas, not absolutes
            for p in paths:
                fn = fns[p]
                torch.cuda.synchronize()
                s, e = torch.cuda.Event(True), torch.cuda.Event(True)
                s.record()
                for _ in range(iters):
                    fn()
                e.record()
                torch.cuda.synchronize()
                times[p].append(s.elapsed_time(e) / iters * 1e-3)
        for p in paths:
            t = sorted(times[p])[len(times[p]) // 2]
            print("M=%d N=%d K=%d epi=%s path=%s  %.1f us  %.1f TF (min %.1f us)" % (
                M, wn, k, epi, p, t * 1e6, 2 * M * wn * k / t / 1e12, min(times[p]) * 1e6), flush=True)


if __name__ == "__main__":
    main()
