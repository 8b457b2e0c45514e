"""Stage timeline of the fused decode launches (attention.hip attn_oproj_kernel, stamp build): batch B with
~5.2k-token contexts at Llama-3.1-8B widths. Every block's lane 0 writes s_memrealtime (10 ns ticks,
device-wide) at its stage boundaries; this prints, per role, the percentiles of each stamp in microseconds
from the launch's first block start, next to the unfused kernels' device times (hipEvents).

  python tools/fused_stamps.py            # B=1; FS_B=4 FS_MODE=qao|ao FS_LEN=5200
Stamps: attention 0 start, 1 KV prefetch issued, 2 qkv flag seen, 3 main loop done, 4 records out,
6 merged (last partition of a head), 5 arrived; o_proj 0 start, 1 weights issued, 2 flag seen, 3 slice
staged, 4 slab / columns stored, 5 end (6 norm tail done); qkv 0 start, 3 slab stored, 5 arrived.
RAGK_AO_V2=0 / RAGK_AO_MIA=0 select the older o_proj roles.
"""
import math
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from rag_llm_k8s_amd.ops import native
    from rag_llm_k8s_amd.ops import reference as R

    dev = "cuda"
    B = int(os.environ.get("FS_B", "1"))
    L = int(os.environ.get("FS_LEN", "5200"))
    mode = os.environ.get("FS_MODE", "qao")
    Hq, Hkv, D, H = 32, 8, 128, 4096
    torch.manual_seed(0)
    nb = (L + 63) // 64 + 1
    kc = torch.randn(B * nb + 4, Hkv, 64, D, device=dev).bfloat16()
    vc = torch.randn_like(kc)
    bt = torch.arange(B * nb, dtype=torch.int32, device=dev).view(B, nb) + 1
    kvl = torch.full((B,), L, dtype=torch.int32, device=dev)
    pos = kvl - 1
    slots = (bt[torch.arange(B, device=dev), (pos // 64).long()] * 64 + pos % 64).int()
    cos, sin = R.rope_tables(D, 8192, theta=500000.0)
    cos, sin = cos.to(dev), sin.to(dev)
    pt, mp = native.decode_partitions(8192, B, Hkv)
    Nq = (Hq + 2 * Hkv) * D
    wqkv = (torch.randn(Nq, H, device=dev) / 64).bfloat16()
    wo = (torch.randn(H, Hq * D, device=dev) / 64).bfloat16()
    g = torch.ones(H, device=dev).bfloat16()
    h = torch.randn(B, H, device=dev).bfloat16()
    ws_o = torch.empty((B, Hq, mp, D), dtype=torch.float32, device=dev)
    ws_ml = torch.empty((B, Hq, mp, 2), dtype=torch.float32, device=dev)
    native.attn_oproj_counters(dev)
    flush = torch.empty(512 << 20, dtype=torch.uint8, device=dev)  # evict weights / KV from the MALL

    def run():
        if mode == "qao":
            return native.qkv_attn_oproj(h, g, 1e-5, wqkv, pos, cos, sin, slots, kc, vc, bt, kvl, Hq, Hkv, D, pt, mp,
                                         ws_o, ws_ml, wo, g, 1e-5)
        P = native.gemm_part_norm(h, g, 1e-5, wqkv)
        return native.attn_oproj(P, pos, cos, sin, slots, kc, vc, bt, kvl, Hq, Hkv, D, pt, mp, ws_o, ws_ml, wo,
                                 norm=(h, g, 1e-5))

    def unfused():
        P = native.gemm_part_norm(h, g, 1e-5, wqkv)
        attn = torch.empty(B, Hq * D, device=dev).bfloat16()
        native.attn_decode_rope(P, pos, cos, sin, slots, kc, vc, bt, kvl, attn, Hq, Hkv, D, pt, mp, ws_o=ws_o,
                                ws_ml=ws_ml, defer_merge=True)
        Po = native.gemm_part_merge(attn, kvl, pt, mp, ws_o, ws_ml, Hq, wo)
        return native.add_partials_rmsnorm(Po, h, g, 1e-5)

    def timed(fn, n=20):
        ts = []
        for _ in range(n):
            flush.zero_()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        return float(np.median(ts))

    for _ in range(3):
        run(), unfused()
    print("B=%d L=%d mode=%s: fused %.1f us, unfused chain %.1f us (hipEvents, cold MALL, median of 20)"
          % (B, L, mode, timed(run), timed(unfused)), flush=True)
    nq = (Nq // 64) * (H // (64 * native.QAO_QKS)) if mode == "qao" else 0
    na = mp * Hkv * B
    no = (H // 16) if native._ao_v2(Hq * D, H) else (H // 64) * (Hq * D // (64 * native.ATTN_OPROJ_KS))
    st = torch.zeros((nq + na + no, 8), dtype=torch.int64, device=dev)
    lib = native._lib.lib()
    rows = []
    for it in range(6):
        st.zero_()
        flush.zero_()
        torch.cuda.synchronize()
        native.check(lib.ragk_fused_set_stamps(st.data_ptr(), native.stream_ptr()), "stamps")
        run()
        native.check(lib.ragk_fused_set_stamps(None, native.stream_ptr()), "stamps")
        torch.cuda.synchronize()
        if it >= 2:
            rows.append(st.cpu().numpy().astype(np.float64))
    assert not native.attn_oproj_error(dev)
    for name, lo, hi in (("qkv", 0, nq), ("attention", nq, nq + na), ("o_proj", nq + na, nq + na + no)):
        if hi <= lo:
            continue
        print("%s blocks [%d, %d):" % (name, lo, hi))
        for k in range(8):
            vals = []
            for r in rows:
                t0 = r[:, 0][r[:, 0] > 0].min()
                v = r[lo:hi, k]
                v = v[v > 0]
                vals.extend(((v - t0) / 100.0).tolist())  # 100 MHz ticks -> us
            if vals:
                q = np.percentile(vals, [0, 10, 50, 90, 100])
                print("  stamp %d: n=%5d  min %6.2f  p10 %6.2f  p50 %6.2f  p90 %6.2f  max %6.2f us" % (
                    k, len(vals) // len(rows), *q))


if __name__ == "__main__":
    main()
