"""Batch-1 post-attention tail per layer: the persistent engine (csrc/kernels/mlp_engine.hip: o_proj slabs
+ residual + RMSNorm + gate/up + SiLU + down + residual) vs the separate add_partials_rmsnorm + SiLU*up +
down kernels it replaces, Llama-3.1-8B shapes, L layers of distinct random weights (1.4 GB per 4
layers, so the weights stream from HBM as in a decode step), each form captured in a hipGraph and
replayed back to back; GPU time per layer.

  python tools/mlp_engine_bench.py [layers] [replays]
  ME_NT=0,1    alternate the weight-stream cache policy of the engine
"""
import math
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from rag_llm_k8s_amd import _build
    from rag_llm_k8s_amd.ops import native
    from rag_llm_k8s_amd.ops import reference as R

    _build.build_hip()
    native.MLP_ENGINE = True
    L = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    H, I = 4096, 14336
    dev = "cuda"
    torch.manual_seed(0)
    layers = []
    for _ in range(L):
        g = (torch.randn(I, H, device=dev) / math.sqrt(H)).bfloat16()
        u = (torch.randn(I, H, device=dev) / math.sqrt(H)).bfloat16()
        layers.append((R.pack_gate_up(g, u), (torch.randn(H, I, device=dev) / math.sqrt(I)).bfloat16()))
        del g, u
    x = torch.randn(1, H, device=dev).bfloat16()
    h = torch.randn(1, H, device=dev).bfloat16()

    P = torch.randn(8, 1, H, device=dev) * 0.01
    gamma = torch.ones(H, device=dev).bfloat16()

    def separate():
        for wgu, wd in layers:
            xn = native.add_partials_rmsnorm(P, h, gamma, 1e-5)
            a = native.gemm(xn, wgu, epi="silu_mul")
            native.gemm(a, wd, resid=h, epi="resid", out=h)

    def engine():
        for wgu, wd in layers:
            native.mlp_engine_tail(P, h, gamma, 1e-5, wgu, wd)

    def graph_of(fn):
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            fn()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gr, stream=s):  # the warm-up stream (stream-keyed engine workspace)
            fn()
        return gr

    def timed(gr):
        gr.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            gr.replay()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / reps / L * 1e6

    nts = [int(t) for t in os.environ.get("ME_NT", "1").split(",") if t]
    # ME_XW="27:32,1:1": alternate the per-XCD phase-A weights (even:odd) -- engine runs per setting
    xws = [tuple(int(v) for v in s.split(":")) for s in os.environ.get("ME_XW", "").split(",") if s] or [None]
    g_sep = graph_of(separate)
    for rnd in range(2):
        print("round %d: separate kernels %.2f us/layer" % (rnd, timed(g_sep)), flush=True)
        for nt in nts:
            for xw in xws:
                from rag_llm_k8s_amd.ops import _lib
                if xw is not None:
                    _lib.lib().ragk_mlp_engine_set_xcd_weights(*xw)
                native.set_mlp_engine_nt(nt)
                g_eng = graph_of(engine)
                t = timed(g_eng)
                native.mlp_engine_check()
                print("round %d: engine nt=%d xcd weights %s %.2f us/layer (%.2f TB/s of weights)" % (
                    rnd, nt, xw, t, (3 * H * I * 2) / t / 1e6), flush=True)
                del g_eng
    native.set_mlp_engine_nt(1)
    if os.environ.get("ME_STAMPS") == "1":
        # one launch with stage stamps (s_memrealtime, 100 MHz): per-workgroup times from the earliest start
        from rag_llm_k8s_amd.ops import _lib
        G = native._cu_count()
        st = torch.zeros(G, 8, dtype=torch.int64, device=dev)
        _lib.lib().ragk_mlp_engine_set_stamps(st.data_ptr())
        runs = []
        for li in range(4):
            st.zero_()
            native.mlp_engine_tail(P, h, gamma, 1e-5, layers[li][0], layers[li][1])
            torch.cuda.synchronize()
            runs.append(st.cpu().double().clone())
        # skew structure: phase-A finish per XCD (dispatch order w % 8) and its repeatability across launches
        for k, r in enumerate(runs):
            us_r = (r[:, 2] - r[:, 0].min()) / 100.0
            per = [us_r[x::8].median().item() for x in range(8)]
            print("launch %d phase A done per XCD p50: %s" % (k, " ".join("%.1f" % v for v in per)), flush=True)
        a0 = (runs[-1][:, 2] - runs[-1][:, 0].min()) / 100.0
        a1 = (runs[-2][:, 2] - runs[-2][:, 0].min()) / 100.0
        c = torch.corrcoef(torch.stack([a0, a1]))[0, 1].item()
        print("per-workgroup phase A finish, correlation between two launches: %.2f" % c, flush=True)
        _lib.lib().ragk_mlp_engine_set_stamps(None)
        s = runs[-1]
        t0 = s[:, 0].min()
        us = (s[:, :5] - t0) / 100.0  # 100 MHz -> us
        names = ["start", "loader done", "phase A done", "act ready", "end"]
        for i, n in enumerate(names):
            col = us[:, i]
            print("stamp %-13s min %7.2f  p50 %7.2f  max %7.2f us" % (n, col.min(), col.median(), col.max()), flush=True)


if __name__ == "__main__":
    main()
