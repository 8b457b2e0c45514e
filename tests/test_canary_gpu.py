"""GPU out-of-bounds canaries ("HIP kernels checked for OOB with guard pages in unit tests").

Every output of a kernel with ragged tails is a view into a larger allocation whose head and tail are
filled with a sentinel; after the launch the sentinel must be intact, and the view must hold the
right values. Covered: the GEMM family at M / N tails (tile GEMM, 256x256 w4 and ping-pong, skinny,
glds-ring stream, LDS-activation decode GEMM, split-K partial slabs, prefill split-K slabs, fused
epilogues), the norm / residual consumers, prefill attention over ragged tile lists, split-K decode
attention, the paged KV writes (untouched cache blocks stay sentinel), the top-k / sampler buffers.
The reference's analogue is the unguarded read-modify-write at /root/reference/llm/rag.py:68-86.
"""
import math

import pytest
import torch

from rag_llm_k8s_amd.ops import reference as R

pytestmark = pytest.mark.gpu
DEV = "cuda"
PAD = 4096  # elements of sentinel on each side


def guarded(shape, dtype, sentinel=-7.0):
    n = 1
    for s in shape:
        n *= s
    buf = torch.full((2 * PAD + n,), sentinel, dtype=dtype, device=DEV)
    return buf, buf[PAD:PAD + n].view(*shape)


def intact(buf, sentinel=-7.0):
    torch.cuda.synchronize()
    s = torch.tensor(sentinel, dtype=buf.dtype)
    return bool(buf[:PAD].cpu().eq(s).all()) and bool(buf[-PAD:].cpu().eq(s).all())


def rel_err(a, b):
    a, b = a.float().cpu(), b.float().cpu()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


@pytest.mark.parametrize("M,N,K,path,epi", [
    (1111, 1032, 512, 6, "none"),      # 256x256 w4: ragged M and N tiles
    (1111, 1032, 512, 6, "resid"),
    (777, 1280, 384, 6, "silu_mul"),    # N = 2 x 640 packed gate/up
    (513, 4104, 256, 2, "none"),        # 8-wave ping-pong
    (300, 1000, 768, None, "none"),     # 128^2 tile GEMM
    (7, 1000, 768, None, "resid"),      # skinny decode GEMM
    (33, 14336, 4096, 5, "silu_mul"),   # glds-ring stream (gate/up shape)
    (40, 32776, 1024, 4, "none"),       # LDS-activation decode GEMM (lm_head-like, N % 256 != 0)
])
def test_gemm_outputs_stay_in_bounds(native, M, N, K, path, epi):
    torch.manual_seed(M + N)
    x = torch.randn(M, K, device=DEV).bfloat16()
    rows = 2 * N if epi == "silu_mul" else N
    w = (torch.randn(rows, K, device=DEV) / math.sqrt(K)).bfloat16()
    buf, out = guarded((M, N), torch.bfloat16)
    r = torch.randn(M, N, device=DEV).bfloat16() if epi == "resid" else None
    native.gemm(x, w, resid=r, epi=epi, out=out, path=path)
    assert intact(buf)
    ref = R.linear(x.float().cpu(), w.float().cpu(), None, r.float().cpu() if r is not None else None, epi=epi)
    assert rel_err(out, ref) < 2e-2


@pytest.mark.parametrize("M,N,K", [(13, 1000, 1024), (1, 6144, 4096), (33, 4096, 14336), (64, 512, 512)])
def test_gemm_part_slabs_in_bounds(native, M, N, K):
    torch.manual_seed(K)
    x = torch.randn(M, K, device=DEV).bfloat16()
    w = (torch.randn(N, K, device=DEV) / math.sqrt(K)).bfloat16()
    ks, S = native.gemm_part_slabs(M, N, K)
    assert S > 0
    buf, P = guarded((S, M, N), torch.float32)
    native.gemm_part(x, w, out=P)
    assert intact(buf)
    assert rel_err(P.sum(0), x.float() @ w.float().t()) < 1e-4


@pytest.mark.parametrize("M,I,H", [(1, 1792, 4096), (3, 3584, 4096), (4, 7168, 4096)])
def test_gemm_part_silu_slabs_in_bounds(native, M, I, H):
    torch.manual_seed(I)
    x = torch.randn(M, H, device=DEV).bfloat16()
    wgu = (torch.randn(2 * I, H, device=DEV) / math.sqrt(H)).bfloat16()
    wd = (torch.randn(H, I, device=DEV) / math.sqrt(I)).bfloat16()
    pgu = native.gemm_part_gu(x, wgu)
    P0 = native.gemm_part_silu(pgu, wd)
    buf, P = guarded(tuple(P0.shape), torch.float32)
    native.gemm_part_silu(pgu, wd, out=P)
    assert intact(buf)
    assert torch.equal(P, P0)


def test_prefill_splitk_slabs_in_bounds(native):
    torch.manual_seed(3)
    M, N, K, ns = 1300, 1032, 1024, 2
    x = torch.randn(M, K, device=DEV).bfloat16()
    w = (torch.randn(N, K, device=DEV) / math.sqrt(K)).bfloat16()
    buf, P = guarded((ns, M, N), torch.float32)
    native.gemm_splitk(x, w, ns, out=P)
    assert intact(buf)
    assert rel_err(P.sum(0), x.float() @ w.float().t()) < 1e-4


@pytest.mark.parametrize("M,H", [(5, 4096), (1, 8192), (17, 384)])
def test_norm_consumers_in_bounds(native, M, H):
    torch.manual_seed(M)
    h = torch.randn(M, H, device=DEV).bfloat16()
    g = (1 + 0.1 * torch.randn(H, device=DEV)).bfloat16()
    buf, out = guarded((M, H), torch.bfloat16)
    native.rmsnorm(h, g, 1e-5, out=out)
    assert intact(buf)
    assert rel_err(out, R.rmsnorm(h.cpu(), g.cpu(), 1e-5)) < 1e-2
    P = torch.randn(3, M, H, device=DEV) * 0.1
    hbuf, hh = guarded((M, H), torch.bfloat16)
    hh.copy_(h)
    buf2, out2 = guarded((M, H), torch.bfloat16)
    native.add_partials_rmsnorm(P, hh, g, 1e-5, out=out2)
    assert intact(buf2) and intact(hbuf)


def _paged(lens, Hkv, D, sentinel):
    nb = sum((L + 63) // 64 for L in lens) + 2
    kbuf, kc = guarded((nb, Hkv, 64, D), torch.bfloat16, sentinel)
    vbuf, vc = guarded((nb, Hkv, 64, D), torch.bfloat16, sentinel)
    maxb = max((L + 63) // 64 for L in lens)
    bt = torch.zeros(len(lens), maxb, dtype=torch.int32)
    b = 1
    for i, L in enumerate(lens):
        n = (L + 63) // 64
        bt[i, :n] = torch.arange(b, b + n)
        b += n
    return kbuf, kc, vbuf, vc, bt.to(DEV)


def test_prefill_attention_and_kv_writes_in_bounds(native):
    """rope_kv writes exactly the prompt slots (every other cache element stays sentinel); the
    attention output over a ragged tile list stays inside its [T, Hq*D] view."""
    torch.manual_seed(9)
    Hq, Hkv, D = 8, 2, 128
    lens = [37, 100, 1]
    T = sum(lens)
    kbuf, kc, vbuf, vc, bt = _paged(lens, Hkv, D, 3.0)
    qkv = torch.randn(T, (Hq + 2 * Hkv) * D, device=DEV).bfloat16()
    pos = torch.cat([torch.arange(L) for L in lens]).int().to(DEV)
    slots = torch.cat([bt[i, torch.arange(L) // 64].cpu() * 64 + torch.arange(L) % 64
                       for i, L in enumerate(lens)]).int().to(DEV)
    cos, sin = R.rope_tables(D, 4096, theta=500000.0)
    native.rope_kv(qkv, pos, cos.to(DEV), sin.to(DEV), slots, kc, vc, Hq, Hkv, D)
    assert intact(kbuf, 3.0) and intact(vbuf, 3.0)
    written = torch.zeros(kc.shape[0] * 64, dtype=torch.bool)
    written[slots.long().cpu()] = True
    untouched = (~written).view(kc.shape[0], 64)
    kcc = kc.cpu().permute(0, 2, 1, 3)  # [nb, 64, Hkv, D]
    assert bool(kcc[untouched].eq(3.0).all())
    cu = torch.tensor([0, 37, 137, 138], dtype=torch.int32, device=DEV)
    kvl = torch.tensor(lens, dtype=torch.int32, device=DEV)
    tiles = native.build_prefill_tiles(lens, Hq, Hkv).to(DEV)
    obuf, out = guarded((T, Hq * D), torch.bfloat16)
    native.attn_prefill(qkv, kc, vc, cu, kvl, tiles, out, Hq, Hkv, D, causal=True, paged=True, block_tables=bt)
    assert intact(obuf)
    assert bool(torch.isfinite(out.float()).all())


@pytest.mark.parametrize("Hq,Hkv", [(32, 8), (4, 1)])
@pytest.mark.parametrize("single", [False, True])
def test_decode_attention_in_bounds(native, Hq, Hkv, single, monkeypatch):
    """single: the single-partition grid (the batch-32 path: K tiles by LDS-DMA in 4-wave blocks)."""
    if single:
        monkeypatch.setattr(native, "DECODE_NW8_MIN_PAIRS", 1)
    torch.manual_seed(10)
    D = 128
    lens = [65, 3000, 1]
    kbuf, kc, vbuf, vc, bt = _paged(lens, Hkv, D, 0.5)
    B = len(lens)
    kvl = torch.tensor(lens, dtype=torch.int32, device=DEV)
    pt, mp = native.decode_partitions(max(lens), B, Hkv, target_blocks=1024)
    ws_o = torch.empty((B, Hq, mp, D), dtype=torch.float32, device=DEV)
    ws_ml = torch.empty((B, Hq, mp, 2), dtype=torch.float32, device=DEV)
    q = torch.randn(B, Hq * D, device=DEV).bfloat16()
    obuf, out = guarded((B, Hq * D), torch.bfloat16)
    native.attn_decode(q, kc, vc, bt, kvl, out, Hq, Hkv, D, pt, mp, ws_o, ws_ml)
    assert intact(obuf) and intact(kbuf, 0.5) and intact(vbuf, 0.5)
    assert bool(torch.isfinite(out.float()).all())


def test_topk_and_sampler_buffers_in_bounds(native):
    torch.manual_seed(11)
    B, V, K, chunks = 3, 30011, 64, 7
    logits = torch.randn(B, V, device=DEV)
    vbuf, cv = guarded((B, chunks * K), torch.float32)
    ibuf, ci = guarded((B, chunks * K), torch.int32, -7)
    native.topk_candidates(logits, K, chunks=chunks, cand_v=cv, cand_i=ci)
    assert intact(vbuf) and intact(ibuf, -7)
    assert bool((ci >= 0).all()) and bool((ci < V).all())
    temps = torch.full((B,), 0.7, device=DEV)
    ks = torch.full((B,), 50, dtype=torch.int32, device=DEV)
    ps = torch.full((B,), 0.9, device=DEV)
    seeds = torch.arange(B, dtype=torch.int64, device=DEV) + 5
    steps = torch.zeros(B, dtype=torch.int32, device=DEV)
    tbuf, tok = guarded((B,), torch.int32, -7)
    native.sample_candidates(cv, ci, temps, ks, ps, seeds, steps, out_tok=tok, list_len=K)
    assert intact(tbuf, -7)
    assert bool((tok >= 0).all()) and bool((tok < V).all())
