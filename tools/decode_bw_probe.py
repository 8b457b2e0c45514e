"""Decode-GEMM bandwidth probe on the Llama-8B decode shapes at M=1 (the C=1 latency path):

* cold: the weight rotates over enough copies (>= 1.5 GB) that every call streams from HBM;
* warm: the same matrix back to back, i.e. what a call sees when its weights were just read (the
  256 MB Infinity Cache / MALL holds them) -- the upper bound of prefetching the next GEMM's weights
  into the MALL while attention runs;
* for the stream kernel (gate/up) with the non-temporal and the default load policy, and split-K S.
Prints one line per case (TB/s of weight bytes)."""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from rag_llm_k8s_amd.ops import _lib  # noqa: E402
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


def main():
    L = _lib.lib()
    res = []
    M = int(os.environ.get("PROBE_M", "1"))
    x = None
    for (Nn, K, epi, name) in [(6144, 4096, "none", "qkv"), (4096, 4096, "resid", "o_proj"),
                               (14336, 4096, "silu_mul", "gate_up"), (4096, 14336, "resid", "down")]:
        wn = 2 * Nn if epi == "silu_mul" else Nn
        ncopy = max(2, -(-(1536 << 20) // (wn * K * 2)))
        ws = [(torch.randn(wn, K, device="cuda") / math.sqrt(K)).bfloat16() for _ in range(ncopy)]
        x = torch.randn(M, K, device="cuda").bfloat16()
        r = torch.randn(M, Nn, device="cuda").bfloat16() if epi == "resid" else None
        out = torch.empty(M, Nn, device="cuda").bfloat16()
        it = [0]

        def nxt():
            it[0] = (it[0] + 1) % ncopy
            return ws[it[0]]

        byts = wn * K * 2
        paths = {"default": None}
        if epi == "silu_mul" or N.use_stream(M, Nn, K, epi):
            paths["stream"] = 5
        else:
            paths["part"] = "part"
        for pname, path in paths.items():
            for nt in ((0, 1) if path == 5 else (1,)):
                L.ragk_gemm_stream_set_nt(nt)
                for S in ((0, 2, 4) if path == 5 else (0,)):
                    N.STREAM_S_OVERRIDE = S
                    try:
                        if path == "part":  # split-K partials (the engine's qkv / o / down decode path)
                            tc = timeit(lambda: N.gemm_part(x, nxt()), 4 * ncopy)
                            tw = timeit(lambda: N.gemm_part(x, ws[0]), 4 * ncopy)
                        else:
                            tc = timeit(lambda: N.gemm(x, nxt(), resid=r, epi=epi, out=out, path=path), 4 * ncopy)
                            tw = timeit(lambda: N.gemm(x, ws[0], resid=r, epi=epi, out=out, path=path), 4 * ncopy)
                    except Exception as ex:  # unsupported split for this shape
                        print(name, pname, "S=%d" % S, "skipped:", ex, flush=True)
                        continue
                    row = dict(name=name, M=M, path=pname, nt=nt, S=S, MB=round(byts / 2 ** 20, 1),
                               cold_us=round(tc * 1e6, 1), cold_TBps=round(byts / tc / 1e12, 2),
                               warm_us=round(tw * 1e6, 1), warm_TBps=round(byts / tw / 1e12, 2))
                    res.append(row)
                    print(json.dumps(row), flush=True)
        N.STREAM_S_OVERRIDE = 0
        L.ragk_gemm_stream_set_nt(1)
        del ws
        torch.cuda.empty_cache()
    # raw copy bandwidth (read + write) of a 1 GiB buffer, as a roofline reference
    a = torch.empty(1 << 29, dtype=torch.bfloat16, device="cuda")
    b = torch.empty_like(a)
    t = timeit(lambda: b.copy_(a), 10)
    print(json.dumps(dict(name="copy_1GiB", TBps_read_plus_write=round(2 * a.numel() * 2 / t / 1e12, 2))), flush=True)
    os.makedirs("gpurun_out", exist_ok=True)
    json.dump(res, open("gpurun_out/decode_bw_probe.json", "w"), indent=1)


if __name__ == "__main__":
    main()
