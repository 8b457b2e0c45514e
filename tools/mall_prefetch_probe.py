"""Does prefetching a GEMM's weights into the MALL while latency-bound kernels run pay off?

Synthetic decode layer, captured in a hipGraph and replayed over 8 rotating layers' gate/up
weights (8 x 224 MB, cold in HBM): [latency window: spin SPIN us] -> [gate/up GEMM, M=1].
Variant B forks a side stream at the start of each latency window that reads the first P MB of that
layer's gate/up weights (csrc/kernels/prefetch.hip); the GEMM does not wait for it.
Prints per-layer us for each (P, blocks, weight-load policy) and the no-prefetch baseline."""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rag_llm_k8s_amd.ops import _lib  # noqa: E402
from rag_llm_k8s_amd.ops import native as N  # noqa: E402

LAYERS = 8
F, K = 14336, 4096


def run(ws, x, out, spin, pf_bytes, blocks, reps=5):
    s0 = torch.cuda.Stream()
    s1 = torch.cuda.Stream()
    g = torch.cuda.CUDAGraph()
    # warm-up outside capture (allocations, first launches)
    with torch.cuda.stream(s0):
        N.gemm(x, ws[0], epi="silu_mul", out=out, path=5)
        if pf_bytes:
            N.prefetch(ws[0], pf_bytes, blocks)
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=s0):
        for l in range(LAYERS):
            if pf_bytes:
                ev = torch.cuda.Event()
                ev.record(s0)
                s1.wait_event(ev)
                with torch.cuda.stream(s1):
                    N.prefetch(ws[l], pf_bytes, blocks)
            if spin:
                N.spin_us(spin)
            N.gemm(x, ws[l], epi="silu_mul", out=out, path=5)
        if pf_bytes:
            ev = torch.cuda.Event()
            ev.record(s1)
            s0.wait_event(ev)
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


def run_fused(ws, x, out, spin, pf_bytes, blocks, reps=5):
    """Single stream: one kernel whose block 0 spins (the latency-bound window) while the other
    blocks prefetch the first pf_bytes of the layer's weights; then the GEMM."""
    L = _lib.lib()
    sink = torch.zeros(4096, dtype=torch.int32, device="cuda")
    g = torch.cuda.CUDAGraph()
    s0 = torch.cuda.Stream()

    def body():
        for l in range(LAYERS):
            N.check(L.ragk_spin_prefetch(spin, ws[l].data_ptr(), pf_bytes, blocks, sink.data_ptr(), N.stream_ptr()),
                    "spin_prefetch")
            N.gemm(x, ws[l], epi="silu_mul", out=out, path=5)
    with torch.cuda.stream(s0):
        body()
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=s0):
        body()
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
    L = _lib.lib()
    torch.manual_seed(0)
    ws = [(torch.randn(2 * F, K, device="cuda") / math.sqrt(K)).bfloat16() for _ in range(LAYERS)]
    x = torch.randn(1, K, device="cuda").bfloat16()
    out = torch.empty(1, F, device="cuda").bfloat16()
    res = []
    spin = int(os.environ.get("SPIN_US", "20"))
    for nt in (1, 0):
        L.ragk_gemm_stream_set_nt(nt)
        base_g = run(ws, x, out, 0, 0, 0)
        base = run(ws, x, out, spin, 0, 0)
        row = dict(nt=nt, spin_us=spin, gemm_only_us=round(base_g, 1), spin_plus_gemm_us=round(base, 1))
        print(json.dumps(row), flush=True)
        res.append(row)
        base_f = run_fused(ws, x, out, spin, 0, 0)
        print(json.dumps(dict(nt=nt, fused_baseline_us=round(base_f, 1))), flush=True)
        for mb in (32, 64, 96, 128, 224):
            for blocks in (64, 128, 255):
                t = run_fused(ws, x, out, spin, mb << 20, blocks)
                row = dict(nt=nt, mode="fused", spin_us=spin, prefetch_MB=mb, blocks=blocks, layer_us=round(t, 1),
                           saved_us=round(base_f - t, 1))
                print(json.dumps(row), flush=True)
                res.append(row)
        for mb in (64,):
            for blocks in (128,):
                t = run(ws, x, out, spin, mb << 20, blocks)
                row = dict(nt=nt, spin_us=spin, prefetch_MB=mb, blocks=blocks, layer_us=round(t, 1),
                           saved_us=round(base - t, 1))
                print(json.dumps(row), flush=True)
                res.append(row)
    L.ragk_gemm_stream_set_nt(1)
    os.makedirs("gpurun_out", exist_ok=True)
    json.dump(res, open("gpurun_out/mall_prefetch_probe.json", "w"), indent=1)


if __name__ == "__main__":
    main()
