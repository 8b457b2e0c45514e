"""Shape-checked Python entry points of the gfx950 kernels (GPU tensors only).

Every function validates dtype / contiguity / shapes on the host *before* the launch
(a mis-shaped launch could fault the GPU), then calls the C ABI with the current
HIP stream, so everything here is capturable in a hipGraph (torch.cuda.CUDAGraph).
"""
from __future__ import annotations

import math
import os
import threading

import torch

from . import _lib
from ._lib import check, ptr, stream_ptr
from .reference import EPI


def _req(cond, msg):
    if not cond:
        raise ValueError(msg)


def _bf16_2d(t, name):
    _req(t.is_cuda and t.dtype == torch.bfloat16 and t.dim() == 2, "%s must be a 2-D bf16 GPU tensor" % name)
    _req(t.stride(1) == 1, "%s must be row-contiguous" % name)


# ----------------------------------------------------------------------------- GEMM
# large-M GEMMs (prefill) go to the 256x256 MFMA kernels from this many rows
PP_MIN_M = 1024


def set_w4_grid(g):
    """gemm_w4 persistent grid: -1 = one block per CU (default), 0 = one block per output tile,
    g > 0 = at most g blocks (each block loops over tiles g apart)."""
    check(_lib.lib().ragk_gemm_w4_set_grid(int(g)), "ragk_gemm_w4_set_grid")




DEC_DEFAULT = True
DEC_WS_BYTES = 96 << 20
_dec_ws = {}


def dec_workspace(device):
    """Per-device split-K workspace for the decode GEMM: fp32 slabs + ticket counters (zeroed once;
    the last-arriving block resets its counter). Allocated eagerly, before any graph capture."""
    key = str(device)
    if key not in _dec_ws:
        _dec_ws[key] = (torch.empty(DEC_WS_BYTES // 4, dtype=torch.float32, device=device),
                        torch.zeros(65536, dtype=torch.int32, device=device))
    return _dec_ws[key]


def use_dec(M, N, K, epi):
    """v3 (LDS-shared activations) wins over v1 only on vocab-sized N at M > 16 (lm_head: 5.1 vs
    3.1 TB/s at M=32, cache-cold); v1 stays the default elsewhere (profiles/kernels_r1_decode.json)."""
    return 16 < M <= 64 and N >= 32768 and K % 256 == 0 and epi != "silu_mul"


STREAM_DEFAULT = True
STREAM_MIN_ROWS = 16384
# vocab-sized weights (>= 32768 rows, the lm_head) go to the stream GEMM (nt weights) only above batch 16:
# batch 32 6.97 -> 6.94 ms per decode step, batch 4 slower (profiles/decode_lmhead_stream_r4.log)
STREAM_MAX_ROWS = 262144
STREAM_VOCAB_MIN_M = 17


def use_stream(M, N, K, epi, fp8=False):
    """Decode GEMM v4 (glds ring) wins where one launch has >= ~128 n-tiles of long K-streams and
    no split-K: the packed gate/up projection (4.5 vs 3.4 TB/s bf16 at M=32, 4.4 vs 2.2 at M=64;
    fp8 2.6 vs 1.5 at M=32) and other 16k-32k-row weights. Below that, the fixed pipeline-fill +
    split-K reduction latencies lose to the register-streaming kernels (profiles/tune_stream_r1.json)."""
    rows = 2 * N if epi == "silu_mul" else N
    if M > 64 or not (STREAM_MIN_ROWS <= rows < STREAM_MAX_ROWS) or K % 128:
        return False
    if rows >= 32768 and M < STREAM_VOCAB_MIN_M:
        return False
    return M > 16 if fp8 else True


def use_pp(M, N, K, epi):
    """Large-M GEMMs go to a 256x256 MFMA kernel: gemm_w4.hip (default, 4 waves x 128x128, 9-16 %
    faster on the Llama-8B prefill shapes, profiles/gemm_w4_r1.txt) or the 8-wave ping-pong gemm_pp.hip."""
    if M < PP_MIN_M or K % 64 or K < 192:  # gemm_w4's continuous ring needs three K-tiles per tile
        return False
    return N % 128 == 0 if epi == "silu_mul" else N % 8 == 0


# Large-M GEMMs through hipBLASLt (torch) instead of gemm_w4, by epilogue (A/B only). "none" (default):
# every large-M GEMM on the hand-written gemm_w4, no library kernel on the prefill path. "resid": the
# residual-add projections (o_proj, down: h += x @ W^T as one in-place addmm, beta = 1) on hipBLASLt --
# its K-loop is 4-6 % faster on those two shapes, worth 0.85 % of the headline bench (1644 / 1648 vs
# 1660 / 1661 tok/s, same box alternating, profiles/bench_prefill_blas_ab_r5.log); "plain": no-epilogue
# GEMMs only; "all": both. The fused SiLU*up gate/up GEMM has no library form (gemm_w4 is 2.8 % faster
# than hipBLASLt's plain GEMM of the same shape, profiles/gemm_silu_rcp_r5.log).
PREFILL_BLAS = os.environ.get("RAGK_PREFILL_BLAS", "none")


# The prefill qkv projection with rope_kv's work in the gemm_w4 epilogue (RoPE on q / k, k and v rows into
# the paged cache; bit-identical to gemm + rope_kv): one pass over the 32k-token chunk's qkv fewer.
PREFILL_ROPE_FUSED = os.environ.get("RAGK_PREFILL_ROPE", "1") != "0"


def gemm_rope_kv_ok(x, w, positions, cos_t, sin_t, slots, k_cache, v_cache, Hq, Hkv, D):
    """Whether gemm_rope_kv takes these operands (else: gemm + rope_kv)."""
    if not PREFILL_ROPE_FUSED or D != 128 or slots is None or k_cache is None or v_cache is None:
        return False
    if not (isinstance(x, torch.Tensor) and isinstance(w, torch.Tensor) and x.is_cuda and w.dim() == 2):
        return False
    M, K = x.shape
    N = w.shape[0]
    if N != (Hq + 2 * Hkv) * D or N % 256 or w.shape[1] != K or not use_pp(M, N, K, "none"):
        return False
    if PREFILL_BLAS in ("plain", "all"):
        return False
    if x.dtype != torch.bfloat16 or w.dtype != torch.bfloat16 or x.stride(1) != 1 or w.stride(1) != 1:
        return False
    if x.stride(0) * M * 2 >= 2 ** 31 or w.stride(0) * N * 2 >= 2 ** 31:
        return False
    if not (k_cache.is_contiguous() and v_cache.is_contiguous() and k_cache.dim() == 4 and k_cache.shape[1] == Hkv
            and k_cache.shape[3] == D and v_cache.shape == k_cache.shape and k_cache.dtype == torch.bfloat16):
        return False
    if not (cos_t.dtype == torch.float32 and sin_t.dtype == torch.float32 and cos_t.is_contiguous()
            and sin_t.is_contiguous() and cos_t.shape[-1] == D // 2):
        return False
    return (positions.dtype == torch.int32 and slots.dtype == torch.int32 and positions.is_contiguous()
            and slots.is_contiguous() and positions.numel() == M and slots.numel() == M)


def gemm_rope_kv(x, w, positions, cos_t, sin_t, slots, k_cache, v_cache, Hq, Hkv, D, out=None):
    """qkv = x @ w^T with RoPE applied to q and k and the k / v rows written to the paged cache at `slots`
    (gemm + rope_kv in one launch; callers check gemm_rope_kv_ok first)."""
    _req(gemm_rope_kv_ok(x, w, positions, cos_t, sin_t, slots, k_cache, v_cache, Hq, Hkv, D), "gemm_rope_kv operands")
    M, K = x.shape
    N = w.shape[0]
    if out is None:
        out = torch.empty((M, N), dtype=torch.bfloat16, device=x.device)
    _req(out.shape == (M, N) and out.stride(1) == 1 and out.stride(0) % 8 == 0, "gemm_rope_kv out")
    check(_lib.lib().ragk_gemm_w4_rope_kv(x.data_ptr(), x.stride(0), w.data_ptr(), w.stride(0), out.data_ptr(),
                                          out.stride(0), M, K, positions.data_ptr(), slots.data_ptr(),
                                          cos_t.data_ptr(), sin_t.data_ptr(), k_cache.data_ptr(), v_cache.data_ptr(),
                                          Hq, Hkv, k_cache.shape[2], stream_ptr()), "ragk_gemm_w4_rope_kv")
    return out


def _gemm_blas(x, w, resid, out, epi):
    if epi == "resid":
        if out.data_ptr() == resid.data_ptr() and out.stride() == resid.stride():
            return out.addmm_(x, w.t())
        return torch.addmm(resid, x, w.t(), out=out)
    return torch.mm(x, w.t(), out=out)


def gemm(x, w, bias=None, resid=None, epi="none", out=None, out_f32=False, path=None):
    """out[M,N] = epi(x[M,K] @ w[N,K]^T). For epi='silu_mul', w is the packed
    gate/up weight [2N, K] (see reference.pack_gate_up) and out has N columns."""
    _bf16_2d(x, "x")
    _bf16_2d(w, "w")
    M, K = x.shape
    e = EPI[epi]
    N = w.shape[0] // 2 if epi == "silu_mul" else w.shape[0]
    _req(w.shape[1] == K, "K mismatch %s vs %s" % (tuple(x.shape), tuple(w.shape)))
    _req(K % 128 == 0, "K must be a multiple of 128 (got %d)" % K)
    if epi == "silu_mul":
        _req(N % 64 == 0, "silu_mul needs N % 64 == 0")
    if "bias" in epi:
        _req(bias is not None and bias.is_cuda and bias.dtype == torch.bfloat16 and bias.numel() == N
             and bias.is_contiguous(), "bias must be bf16[N]")
    if "resid" in epi:
        _bf16_2d(resid, "resid")
        _req(resid.shape == (M, N), "resid shape")
    odt = torch.float32 if out_f32 else torch.bfloat16
    if out is None:
        out = torch.empty((M, N), dtype=odt, device=x.device)
    _req(out.dtype == odt and out.shape == (M, N) and out.stride(1) == 1, "out shape/dtype")
    if M > 64 and N % 8 != 0 and epi != "silu_mul":
        raise ValueError("tile GEMM needs N % 8 == 0")
    if M == 0:
        return out
    L = _lib.lib()
    ldr = resid.stride(0) if resid is not None else 0
    if (path is None and PREFILL_BLAS != "none" and not out_f32 and bias is None and use_pp(M, N, K, epi)
            and ((epi == "none" and PREFILL_BLAS in ("plain", "all"))
                 or (epi == "resid" and PREFILL_BLAS in ("resid", "all")))):
        return _gemm_blas(x, w, resid, out, epi)
    if path is None and use_pp(M, N, K, epi):
        rows = w.shape[0]
        # gemm_w4 addresses operands with 32-bit buffer offsets
        fits = x.stride(0) * M * 2 < 2 ** 31 and w.stride(0) * rows * 2 < 2 ** 31
        path = 6 if fits else 2  # gemm_pp (8-wave ping-pong, 64-bit addressing): operands past 2 GiB
    if path is None and STREAM_DEFAULT and use_stream(M, N, K, epi):
        path = 5
    if path is None and DEC_DEFAULT and use_dec(M, N, K, epi):
        path = 4
    if path == 5:
        rc = _gemm_stream(x, w, None, out, bias, resid, ldr, M, N, K, epi, e, out_f32)
    elif path == 4:
        ws, cnt = dec_workspace(x.device)
        S = L.ragk_gemm_dec_splits(N, K, e)
        need = S * (2 if epi == "silu_mul" else 1) * M * N
        _req(S == 1 or need <= ws.numel(), "decode GEMM workspace too small (%d > %d floats)" % (need, ws.numel()))
        _req(-(-N // 128) <= cnt.numel(), "too many n-tiles for the counter buffer")
        rc = L.ragk_gemm_dec(x.data_ptr(), x.stride(0), w.data_ptr(), w.stride(0), out.data_ptr(), out.stride(0),
                             ptr(bias), ptr(resid), ldr, M, N, K, e, int(out_f32), S, ws.data_ptr(), cnt.data_ptr(),
                             stream_ptr())
    elif path == 2:
        rc = L.ragk_gemm_pp(x.data_ptr(), x.stride(0), w.data_ptr(), w.stride(0), out.data_ptr(), out.stride(0),
                            ptr(bias), ptr(resid), ldr, M, N, K, e, int(out_f32), stream_ptr())
    elif path == 6:
        rc = L.ragk_gemm_w4(x.data_ptr(), x.stride(0), w.data_ptr(), w.stride(0), out.data_ptr(), out.stride(0),
                            ptr(bias), ptr(resid), ldr, M, N, K, e, int(out_f32), stream_ptr())
    elif path is None:
        rc = L.ragk_gemm(x.data_ptr(), x.stride(0), w.data_ptr(), w.stride(0), out.data_ptr(), out.stride(0),
                         ptr(bias), ptr(resid), ldr, M, N, K, e, int(out_f32), stream_ptr())
    else:
        rc = L.ragk_gemm_path(path, x.data_ptr(), x.stride(0), w.data_ptr(), w.stride(0), out.data_ptr(),
                              out.stride(0), ptr(bias), ptr(resid), ldr, M, N, K, e, stream_ptr())
    check(rc, "ragk_gemm")
    return out


PART_MIN_BLOCKS = 512
_part_cfg = [False]


def gemm_part_slabs(M, N, K, ks=None):
    """(ks_steps, S) of the split-K partial GEMM for this shape (0, 0 if unsupported)."""
    if not _part_cfg[0]:
        check(_lib.lib().ragk_gemm_part_set_min_blocks(PART_MIN_BLOCKS), "ragk_gemm_part_set_min_blocks")
        _part_cfg[0] = True
    ks = ks or _lib.lib().ragk_gemm_part_ksteps(M, N, K)
    if ks <= 0 or K % (64 * ks):
        return 0, 0
    return ks, K // (64 * ks)


def gemm_part_norm(h, gamma, eps, w, out=None, ks=None):
    """gemm_part of rmsnorm(h) * gamma (the norm applied inside the GEMM's activation staging, same
    math as rmsnorm): decode batches <= 4, bf16 weights, K <= 8192."""
    _bf16_2d(h, "h")
    _bf16_2d(w, "w")
    M, K = h.shape
    N = w.shape[0]
    _req(w.shape[1] == K and M <= 4 and K <= 8192 and gamma.numel() == K and gamma.dtype == torch.bfloat16
         and gamma.is_contiguous(), "gemm_part_norm shape")
    ks, S = gemm_part_slabs(1, N, K, ks)
    if ks not in (8, 16):  # the norm variant is built for 8- and 16-step K-slices
        ks, S = gemm_part_slabs(1, N, K, 16)
    _req(S > 0 and K in (4096, 8192), "gemm_part_norm: unsupported K=%d" % K)
    if out is None:
        out = torch.empty((S, M, N), dtype=torch.float32, device=h.device)
    check(_lib.lib().ragk_gemm_part_norm(h.data_ptr(), h.stride(0), gamma.data_ptr(), float(eps), w.data_ptr(),
                                         w.stride(0), out.data_ptr(), M, N, K, ks, stream_ptr()),
          "ragk_gemm_part_norm")
    return out


# Split-K partial slabs through the LDS-DMA weight ring (gemm_stream.hip SLAB) instead of gemm_part's
# register-streaming blocks, at decode batches above STREAM_PART_MIN_M: the down projection's 1792-deep
# activation slice needs 114 KB of LDS per gemm_part block at batch 32 (one block per CU, two rounds).
# Batch 32: decode step 7.35 / 7.33 -> 6.91 / 6.98 ms, bench 1568 / 1570 -> 1597 / 1595 tok/s (same box,
# alternating; profiles/bench_stream_part_ab_r4.log).
STREAM_PART = True
STREAM_PART_MIN_M = 5  # batch 8 / 16 -3 %, batch 4 +0.6 %
STREAM_PART_ROWS = 0  # 0: by occupancy (ties: 128)
STREAM_PART_MAX_S = 64  # slabs the consumer sums


def stream_part_cfg(M, N, K):
    """(rows, S) of the slab-mode stream GEMM: the most blocks that are co-resident (128-row tiles one
    block per CU, 64-row tiles two), at least 8 K-steps of 64 per block; (0, 0) if nothing fits."""
    cus = _cu_count()
    steps = K // 64
    best = (0, 0, 0)
    for rows, per_cu in ((128, 1), (64, 2)):
        if STREAM_PART_ROWS and rows != STREAM_PART_ROWS:
            continue
        tiles = -(-N // rows)
        S = 1
        while (tiles * S * 2 <= per_cu * cus and steps % (S * 2) == 0 and steps // (S * 2) >= 8
               and S * 2 <= STREAM_PART_MAX_S):
            S *= 2
        blocks = tiles * S
        if blocks <= per_cu * cus and (blocks / per_cu, rows) > (best[2], best[0]):
            best = (rows, S, blocks / per_cu)
    # a grid that fills less than half the CUs (tensor-parallel shards: o_proj K = 512 cannot be split
    # into 8-step slices) stays on gemm_part, whose 64-column blocks split finer
    if best[2] < 0.5 * cus:
        return 0, 0
    return best[0], best[1]


def gemm_stream_part(x, w, out=None, rows=None, S=None):
    """Partial slabs P[S, M, N] (fp32) with P.sum(0) = x @ w^T from the LDS-DMA stream GEMM (bf16 weights)."""
    _bf16_2d(x, "x")
    _bf16_2d(w, "w")
    M, K = x.shape
    N = w.shape[0]
    _req(w.shape[1] == K and M <= 64 and K % 64 == 0 and N % 4 == 0, "gemm_stream_part shape")
    r0, s0 = stream_part_cfg(M, N, K)
    rows, S = rows or r0, S or s0
    _req(rows in (64, 128) and S >= 1 and (K // 64) % S == 0, "gemm_stream_part config")
    if out is None:
        out = torch.empty((S, M, N), dtype=torch.float32, device=x.device)
    check(_lib.lib().ragk_gemm_stream_part(x.data_ptr(), x.stride(0), w.data_ptr(), w.stride(0), out.data_ptr(), M, N,
                                           K, S, rows, stream_ptr()), "ragk_gemm_stream_part")
    return out


def gemm_part(x, w, out=None, ks=None):
    """Decode GEMM v5 (csrc/kernels/gemm_part.hip): fp32 split-K partials P[S, M, N] with
    P.sum(0) = x @ w^T. The consumer (add_partials_rmsnorm / rope_kv_partials) does the reduction.
    w: bf16 [N, K], or an :class:`ops.fp8.Fp8Weight` (W8A16: e4m3fn rows, per-row scale applied to
    the partials)."""
    from .fp8 import Fp8Weight

    _bf16_2d(x, "x")
    fp8 = isinstance(w, Fp8Weight)
    wt = w.w8 if fp8 else w
    if fp8:
        _req(wt.is_cuda and wt.dim() == 2 and wt.stride(1) == 1 and wt.element_size() == 1, "fp8 weight rows")
        _req(w.scale.dtype == torch.float32 and w.scale.is_contiguous(), "fp8 weight scales fp32")
    else:
        _bf16_2d(wt, "w")
    M, K = x.shape
    N = wt.shape[0]
    _req(wt.shape[1] == K and M <= 64, "gemm_part shape %s x %s" % (tuple(x.shape), tuple(wt.shape)))
    if (STREAM_PART and not fp8 and ks is None and out is None and M >= STREAM_PART_MIN_M and K % 64 == 0
            and N % 4 == 0 and stream_part_cfg(M, N, K)[1] > 0):
        return gemm_stream_part(x, wt)
    ks, S = gemm_part_slabs(M, N, K, ks)
    _req(S > 0, "gemm_part: unsupported K=%d" % K)
    if out is None:
        out = torch.empty((S, M, N), dtype=torch.float32, device=x.device)
    _req(out.dtype == torch.float32 and out.is_contiguous() and out.numel() >= S * M * N, "gemm_part out")
    if fp8:
        check(_lib.lib().ragk_gemm_part_fp8(x.data_ptr(), x.stride(0), wt.data_ptr(), wt.stride(0),
                                            w.scale.data_ptr(), out.data_ptr(), M, N, K, ks, stream_ptr()),
              "ragk_gemm_part_fp8")
    else:
        check(_lib.lib().ragk_gemm_part(x.data_ptr(), x.stride(0), wt.data_ptr(), wt.stride(0), out.data_ptr(), M, N,
                                        K, ks, stream_ptr()), "ragk_gemm_part")
    return out[:S] if out.dim() == 3 else out


PREFILL_SPLITK = True
# measured: M = 5.2k (one RAG prompt) 2 slabs win (o_proj + down 760 -> 656 us per layer); a ~2.2k-token
# tail step with 4 slabs was no faster than unsplit in the bench profile -> split only M >= 4096, 2 slabs
PREFILL_SPLITK_MIN_M = 4096
_n_cus = [0]


def _cu_count():
    if not _n_cus[0]:
        try:
            _n_cus[0] = torch.cuda.get_device_properties(torch.cuda.current_device()).multi_processor_count
        except Exception:
            _n_cus[0] = 256
    return _n_cus[0]


def prefill_nsplit(M, N, K):
    """K-slabs for a prefill GEMM whose 256x256 tile grid fills the CUs poorly (gemm_w4c KSPLIT):
    the split with the best wave efficiency (tiles / (waves * CUs)), 2 % charged per extra slab for
    the fp32 slab traffic; 1 = no split. M = 5.2k (a C=1 RAG prompt), N = 4096: 336 tiles = 1.31 waves
    (66 %) -> 2 slabs = 2.6 waves (88 %). The 32k-token bench steps (2048 tiles) never split."""
    if not PREFILL_SPLITK or M < PREFILL_SPLITK_MIN_M:
        return 1
    cus = _cu_count()
    tiles = -(-M // 256) * -(-N // 256)
    best, best_s = 0.0, 1
    for s in (1, 2):
        if K % (64 * s) or K // s < 4 * 64:
            continue
        wt = tiles * s
        eff = wt / (-(-wt // cus) * cus) - 0.02 * (s - 1)
        if eff > best + 1e-9:
            best, best_s = eff, s
    return best_s


def gemm_splitk(x, w, nsplit, out=None):
    """fp32 split-K slabs P[nsplit, M, N] with P.sum(0) = x @ w^T, one persistent gemm_w4 launch
    (csrc/kernels/gemm_w4.hip KSPLIT); consumed by add_partials_rmsnorm (residual add + norm)."""
    _bf16_2d(x, "x")
    _bf16_2d(w, "w")
    M, K = x.shape
    N = w.shape[0]
    _req(w.shape[1] == K and K % (64 * nsplit) == 0 and K // nsplit >= 256 and N % 8 == 0, "gemm_splitk shape")
    if out is None:
        out = torch.empty((nsplit, M, N), dtype=torch.float32, device=x.device)
    _req(out.dtype == torch.float32 and out.is_contiguous() and out.numel() >= nsplit * M * N, "gemm_splitk out")
    check(_lib.lib().ragk_gemm_w4_splitk(x.data_ptr(), x.stride(0), w.data_ptr(), w.stride(0), out.data_ptr(), M, N, K,
                                         nsplit, stream_ptr()), "ragk_gemm_w4_splitk")
    return out


def gemm_part_merge_ok(M, w, Hq, max_parts, ws_o):
    """Whether the o_proj split-K GEMM can merge the decode attention's partitions itself
    (gemm_part.hip MergeArgs): batch <= 4, head dim 128, a partition workspace present."""
    from .fp8 import Fp8Weight

    if ws_o is None or max_parts < 2:
        return False
    wt = w.w8 if isinstance(w, Fp8Weight) else w
    N, K = wt.shape
    ks, S = gemm_part_slabs(M, N, K)
    return S > 0 and bool(_lib.lib().ragk_gemm_part_merge_ok(M, K, Hq, max_parts, ks))


def gemm_part_merge(attn_out, kv_lens, part_tiles, max_parts, ws_o, ws_ml, Hq, w, out=None):
    """o_proj partials P[S, M, N] = merge(attention partitions) @ w^T: the decode attention ran with its
    split-K merge deferred (attn_decode_rope(..., defer_merge=True)) and every GEMM block merges the
    heads of its K-slice from ws_o / ws_ml (attn_decode_reduce's math); rows with a single partition
    are read from attn_out, where the attention kernel wrote them. Replaces the reduce launch."""
    from .fp8 import Fp8Weight

    fp8 = isinstance(w, Fp8Weight)
    wt = w.w8 if fp8 else w
    M = kv_lens.numel()
    N, K = wt.shape
    _req(attn_out.dtype == torch.bfloat16 and attn_out.stride(1) == 1 and attn_out.shape[0] >= M
         and attn_out.shape[1] == K, "attention output rows")
    _req(ws_o is not None and ws_o.dtype == torch.float32 and ws_o.numel() >= M * Hq * max_parts * 128
         and ws_ml.numel() >= M * Hq * max_parts * 2, "partition workspace")
    ks, S = gemm_part_slabs(M, N, K)
    _req(S > 0 and _lib.lib().ragk_gemm_part_merge_ok(M, K, Hq, max_parts, ks), "gemm_part_merge shape")
    if out is None:
        out = torch.empty((S, M, N), dtype=torch.float32, device=attn_out.device)
    check(_lib.lib().ragk_gemm_part_merge(
        ws_o.data_ptr(), ws_ml.data_ptr(), attn_out.data_ptr(), attn_out.stride(0), kv_lens.data_ptr(), Hq,
        part_tiles, max_parts, wt.data_ptr(), wt.stride(0), w.scale.data_ptr() if fp8 else None, out.data_ptr(), M, N,
        K, ks, stream_ptr()), "ragk_gemm_part_merge")
    return out


SILU_MAX_SLABS = 4  # gemm_part.hip SG_MAXS


def gemm_part_gu_ks(K):
    """K-slice steps of the packed gate/up partial GEMM feeding gemm_part_silu: at most SILU_MAX_SLABS
    slabs. (8 slabs: the TP=8 shard's gate/up 8.2 -> 7.9 us with 448 blocks, but the down GEMM's
    staging of 8 slabs 7.2 -> 9.4 us; docs/PERF_NOTES.md, TP decode.)"""
    for ks in (4, 8, 16, 32):
        if K % (64 * ks) == 0 and K // (64 * ks) <= SILU_MAX_SLABS:
            return ks
    return 0


def _silu_ks(M, N, K):
    """K-slice steps of gemm_part_silu: the SG variant is built for 4/8/16-step slices with one staging
    item per thread (M * 8 * ks <= 512); as gemm_part_slabs, the widest slice reaching PART_MIN_BLOCKS."""
    legal = [ks for ks in (16, 8, 4) if K % (64 * ks) == 0 and M * 8 * ks <= 512]
    nb = -(-N // 64)
    for ks in legal:
        if nb * (K // (64 * ks)) >= PART_MIN_BLOCKS:
            return ks
    return legal[-1] if legal else 0


def gemm_part_silu_ok(M, w_gu, w_down):
    """Whether the down projection can take silu(gate) * up straight from the gate/up partial slabs."""
    if not (isinstance(w_gu, torch.Tensor) and isinstance(w_down, torch.Tensor)):
        return False
    N, K = w_down.shape
    ks_gu = gemm_part_gu_ks(w_gu.shape[1])
    if w_gu.shape[0] != 2 * K or K % 64 or ks_gu == 0 or M > 4:
        return False
    S1 = w_gu.shape[1] // (64 * ks_gu)
    ks = _silu_ks(M, N, K)
    return ks > 0 and bool(_lib.lib().ragk_gemm_part_silu_ok(M, S1, K, ks))


def gemm_part_gu(x, w_gu):
    """Split-K partials of the packed gate/up projection with at most SILU_MAX_SLABS slabs (gemm_part_silu's input)."""
    return gemm_part(x, w_gu, ks=gemm_part_gu_ks(x.shape[1]))


def gemm_part_silu(pgu, w, out=None):
    """Down-projection partials P[S, M, N] of silu(gate) * up, where gate / up are the sums of the slabs
    of pgu [S1, M, 2K] (gemm_part_gu output, packed [64 gate | 64 up] column tiles): the reduction and
    the activation happen in the down GEMM's LDS staging (gemm_part.hip SG) -- no silu_mul launch and
    the gate/up GEMM streams its weights split-K."""
    _bf16_2d(w, "w")
    _req(pgu.dtype == torch.float32 and pgu.is_cuda and pgu.is_contiguous() and pgu.dim() == 3, "pgu fp32 [S1, M, 2K]")
    S1, M, K2 = pgu.shape
    N, K = w.shape
    _req(K2 == 2 * K, "pgu holds packed gate/up columns of width 2K")
    ks = _silu_ks(M, N, K)
    _req(ks > 0 and _lib.lib().ragk_gemm_part_silu_ok(M, S1, K, ks), "gemm_part_silu shape")
    S = K // (64 * ks)
    if out is None:
        out = torch.empty((S, M, N), dtype=torch.float32, device=pgu.device)
    _req(out.shape == (S, M, N) and out.dtype == torch.float32, "out [S, M, N] fp32")
    check(_lib.lib().ragk_gemm_part_silu(pgu.data_ptr(), S1, w.data_ptr(), w.stride(0), out.data_ptr(), M, N, K, ks,
                                         stream_ptr()), "ragk_gemm_part_silu")
    return out


# ----------------------------------------------------------------------------- persistent decode MLP
# Batch-1 decode MLP as one persistent launch (csrc/kernels/mlp_engine.hip): h += W_down (silu(W_gate x) *
# (W_up x)) with both weight streams going through one LDS ring per CU (RAGK_MLP_ENGINE=0 turns it off). Batch-1 decode step 3.47 -> 3.34 ms (profiles/mlp_engine_r5.log).
MLP_ENGINE = os.environ.get("RAGK_MLP_ENGINE", "1") != "0"
_me_ws = {}


class _MeWorkspace:
    """One launch stream's engine state: act [I] bf16 (the hand-off), the monotonic arrival counters, the
    device error word (a set word makes later launches exit at entry), the deadline word (test hook) and a
    host-mapped pinned error word the engine reads after every step without a device sync."""

    def __init__(self, dev, I):
        L = _lib.lib()
        self.nb = int(L.ragk_mlp_engine_ctr_bytes())
        # int64 words: counters | error (u32 at byte nb) | deadline ticks (u32 at byte nb + 8)
        self.words = torch.zeros(self.nb // 8 + 2, dtype=torch.int64, device=dev)
        self.act = torch.zeros(I, dtype=torch.bfloat16, device=dev)
        self.host = L.ragk_host_word_alloc()
        _req(bool(self.host), "mlp_engine: hipHostMalloc of the host error word failed")
        self.host_dev = L.ragk_host_word_dev(self.host)
        _req(bool(self.host_dev), "mlp_engine: no device address for the host error word")
        import ctypes

        self._host_word = ctypes.c_uint.from_address(self.host)

    @property
    def err_ptr(self):
        return self.words.data_ptr() + self.nb

    @property
    def tmo_ptr(self):
        return self.words.data_ptr() + self.nb + 8

    def fault(self) -> int:
        return int(self._host_word.value)

    def rearm(self):
        """Zero the counters and both error words (the device must be idle: no launch of this workspace in
        flight)."""
        self.words[: self.nb // 8 + 1].zero_()
        self._host_word.value = 0

    def __del__(self):  # pragma: no cover - interpreter shutdown order
        try:
            if self.host:
                _lib.lib().ragk_host_word_free(self.host)
                self.host = None
        except Exception:
            pass


def _me_workspace(dev, I):
    """The workspace of the launching stream: two streams (two engines, or two captured graphs of one
    process) never share arrival counters. Allocated by an eager launch, never inside a hipGraph capture
    (a graph-pool allocation, with its zero-fill captured, would be handed to later eager launches after
    the graph is gone): warm up on the stream the graph is then captured on."""
    key = (str(dev), stream_ptr(), I)
    ws = _me_ws.get(key)
    if ws is None:
        _req(not torch.cuda.is_current_stream_capturing(),
             "mlp_engine workspace: run one eager step on the capture stream before capture")
        ws = _me_ws[key] = _MeWorkspace(dev, I)
    return ws


def mlp_engine_ok(M, w_gu, w_down):
    if not MLP_ENGINE or not (isinstance(w_gu, torch.Tensor) and isinstance(w_down, torch.Tensor)):
        return False
    if w_gu.dtype != torch.bfloat16 or w_down.dtype != torch.bfloat16 or not w_gu.is_cuda:
        return False
    H, I = w_down.shape
    if w_gu.shape != (2 * I, H) or not (w_gu.is_contiguous() and w_down.is_contiguous()):
        return False
    return bool(_lib.lib().ragk_mlp_engine_ok(M, H, I, _cu_count()))


def mlp_engine(xn, w_gu, w_down, h):
    """h += W_down . (silu(gate) * up) for ONE row (xn = the post-attention RMSNorm of h, bf16 [1, H])."""
    _bf16_2d(xn, "xn")
    _req(xn.shape == (1, w_down.shape[0]) and xn.is_contiguous(), "xn [1, H]")
    return _mlp_engine_launch(xn.data_ptr(), None, 0, None, 0.0, w_gu, w_down, h)


def mlp_engine_tail(P, h, gamma, eps, w_gu, w_down):
    """The batch-1 post-attention tail in one launch: h += bf16(sum of the o_proj slabs P [S, 1, H]);
    x = rmsnorm(h) * gamma (add_partials_rmsnorm's math); h += W_down . (silu(gate) * up)."""
    H = w_down.shape[0]
    _req(P.dtype == torch.float32 and P.is_cuda and P.is_contiguous() and P.dim() == 3 and P.shape[1:] == (1, H),
         "P [S, 1, H] fp32")
    _req(gamma.dtype == torch.bfloat16 and gamma.is_contiguous() and gamma.numel() == H, "gamma [H] bf16")
    return _mlp_engine_launch(None, P.data_ptr(), P.shape[0], gamma.data_ptr(), float(eps), w_gu, w_down, h)


def _mlp_engine_launch(xn_ptr, P_ptr, S, g_ptr, eps, w_gu, w_down, h):
    _bf16_2d(h, "h")
    H, I = w_down.shape
    _req(h.shape == (1, H) and h.is_contiguous(), "h [1, H]")
    _req(mlp_engine_ok(1, w_gu, w_down), "mlp_engine shape")
    ws = _me_workspace(h.device, I)
    check(_lib.lib().ragk_mlp_engine(xn_ptr, P_ptr, S, g_ptr, eps, w_gu.data_ptr(), w_down.data_ptr(), h.data_ptr(),
                                     ws.act.data_ptr(), ws.words.data_ptr(), ws.err_ptr, ws.host_dev, ws.tmo_ptr, 1,
                                     H, I, _cu_count(), stream_ptr()),
          "ragk_mlp_engine")
    return h


def mlp_engine_fault(dev=None) -> int:
    """Error code of a persistent MLP launch on `dev` that gave up a wait (0 = healthy). Reads the
    host-mapped words only: no device sync, so the engine checks it after every step's event sync."""
    d = torch.device(dev) if dev is not None else None
    for key, ws in list(_me_ws.items()):
        if d is not None and d.index is not None and torch.device(key[0]) != d:
            continue
        e = ws.fault()
        if e:
            return e
    return 0


def mlp_engine_rearm(dev=None):
    """Re-arm every workspace on `dev` after a fault (call with the device idle)."""
    d = torch.device(dev) if dev is not None else None
    for key, ws in list(_me_ws.items()):
        if d is None or d.index is None or torch.device(key[0]) == d:
            ws.rearm()


def mlp_engine_check(dev=None):
    """Raise if a persistent MLP launch on `dev` timed out in a wait (then re-arm its counters). Syncs."""
    if not _me_ws:
        return
    torch.cuda.synchronize(dev)
    e = mlp_engine_fault(dev)
    if e:
        mlp_engine_rearm(dev)
        raise RuntimeError("persistent decode MLP: wait timed out (code %d); counters reset" % e)


def mlp_engine_force_timeout(ticks, dev=None):
    """Test hook: deadline of the following launches in s_memrealtime ticks (0 = the kernel's default). A
    device-side word written on the current stream, so launches captured in a hipGraph see it too."""
    d = torch.device(dev) if dev is not None else None
    for key, ws in list(_me_ws.items()):
        if d is None or d.index is None or torch.device(key[0]) == d:
            ws.words[ws.nb // 8 + 1].fill_(int(ticks))


def set_mlp_engine_nt(nt):
    check(_lib.lib().ragk_mlp_engine_set_nt(int(nt)), "ragk_mlp_engine_set_nt")


STREAM_S_OVERRIDE = 0  # tuning hook (tools/tune_stream.py)


def _gemm_stream(x, w, wscale, out, bias, resid, ldr, M, N, K, epi, e, out_f32):
    """Decode GEMM v4 (csrc/kernels/gemm_stream.hip): glds-ring weight streaming, split-K."""
    L = _lib.lib()
    fp8 = wscale is not None
    S = STREAM_S_OVERRIDE or L.ragk_gemm_stream_splits(N, K, e, int(fp8))
    ws, cnt = dec_workspace(x.device)
    rows = 2 * N if epi == "silu_mul" else N
    _req(S == 1 or S * M * (-(-rows // 128) * 128) <= ws.numel(), "stream GEMM workspace too small")
    _req(-(-rows // 64) <= cnt.numel(), "too many n-tiles for the counter buffer")
    return L.ragk_gemm_stream(x.data_ptr(), x.stride(0), w.data_ptr(), w.stride(0), ptr(wscale), out.data_ptr(),
                              out.stride(0), ptr(bias), ptr(resid), ldr, M, N, K, e, int(out_f32), S, ws.data_ptr(),
                              cnt.data_ptr(), stream_ptr())


# ----------------------------------------------------------------------------- fp8 GEMM
def quant_fp8_rows(x, q=None, scale=None):
    """bf16 [M,K] -> (e4m3fn [M,K], fp32 [M]) with one dynamic scale per row."""
    _bf16_2d(x, "x")
    M, K = x.shape
    _req(K % 8 == 0, "K % 8")
    q = torch.empty((M, K), dtype=torch.float8_e4m3fn, device=x.device) if q is None else q
    scale = torch.empty(M, dtype=torch.float32, device=x.device) if scale is None else scale
    _req(q.shape == (M, K) and q.is_contiguous() and scale.numel() == M, "quant buffers")
    check(_lib.lib().ragk_quant_fp8_rows(x.data_ptr(), x.stride(0), q.data_ptr(), q.stride(0), scale.data_ptr(), M, K,
                                         stream_ptr()), "ragk_quant_fp8_rows")
    return q, scale


FP8_DEC_STREAM = True


def gemm_fp8(x, w, bias=None, resid=None, epi="none", out=None, out_f32=False):
    """out[M,N] = epi(x[M,K] @ dequant(w)^T) for an :class:`ops.fp8.Fp8Weight` w (rows = N, or 2N
    packed gate/up for epi='silu_mul'). M <= 64: W8A16 decode kernel; else W8A8 prefill kernel."""
    from .fp8 import DEC_MAX_M

    _bf16_2d(x, "x")
    M, K = x.shape
    w8, sw = w.w8, w.scale
    _req(w8.dtype == torch.float8_e4m3fn and w8.is_cuda and w8.is_contiguous() and w8.shape[1] == K, "fp8 weight")
    _req(sw.dtype == torch.float32 and sw.numel() == w8.shape[0], "fp8 scale")
    _req(K % 128 == 0, "K must be a multiple of 128")
    e = EPI[epi]
    N = w8.shape[0] // 2 if epi == "silu_mul" else w8.shape[0]
    if epi == "silu_mul":
        _req(N % 64 == 0 and not out_f32, "silu_mul needs N % 64 == 0, bf16 out")
    elif M > DEC_MAX_M:
        _req(N % 8 == 0, "N % 8")
    if "bias" in epi:
        _req(bias is not None and bias.dtype == torch.bfloat16 and bias.numel() == N, "bias bf16[N]")
    if "resid" in epi:
        _bf16_2d(resid, "resid")
        _req(resid.shape == (M, N), "resid shape")
    odt = torch.float32 if out_f32 else torch.bfloat16
    out = torch.empty((M, N), dtype=odt, device=x.device) if out is None else out
    _req(out.dtype == odt and out.shape == (M, N) and out.stride(1) == 1, "out shape/dtype")
    if M == 0:
        return out
    ldr = resid.stride(0) if resid is not None else 0
    if M <= DEC_MAX_M and FP8_DEC_STREAM and use_stream(M, N, K, epi, fp8=True):
        rc = _gemm_stream(x, w8, sw, out, bias, resid, ldr, M, N, K, epi, e, out_f32)
    elif M <= DEC_MAX_M:
        rc = _lib.lib().ragk_gemm_fp8(x.data_ptr(), x.stride(0), None, 0, None, w8.data_ptr(), w8.stride(0),
                                      sw.data_ptr(), out.data_ptr(), out.stride(0), ptr(bias), ptr(resid), ldr, M, N,
                                      K, e, int(out_f32), stream_ptr())
    else:
        q, sa = quant_fp8_rows(x)
        rc = _lib.lib().ragk_gemm_fp8(None, 0, q.data_ptr(), q.stride(0), sa.data_ptr(), w8.data_ptr(), w8.stride(0),
                                      sw.data_ptr(), out.data_ptr(), out.stride(0), ptr(bias), ptr(resid), ldr, M, N,
                                      K, e, int(out_f32), stream_ptr())
    check(rc, "ragk_gemm_fp8")
    return out


# ----------------------------------------------------------------------------- norms
def rmsnorm(x, w, eps, out=None, resid=None):
    _bf16_2d(x, "x")
    T, H = x.shape
    _req(w.numel() == H and w.dtype == torch.bfloat16, "weight")
    _req(H % 8 == 0 and H <= 8192, "H must be a multiple of 8, <= 8192")
    if resid is not None:
        _bf16_2d(resid, "resid")
        _req(resid.shape == x.shape, "resid shape")
    out = torch.empty_like(x) if out is None else out
    check(_lib.lib().ragk_rmsnorm(x.data_ptr(), x.stride(0), ptr(resid), resid.stride(0) if resid is not None else 0,
                                  w.data_ptr(), out.data_ptr(), out.stride(0), T, H, float(eps), stream_ptr()),
          "ragk_rmsnorm")
    return out


def layernorm(x, g, b, eps, out=None, resid=None):
    _bf16_2d(x, "x")
    T, H = x.shape
    _req(H % 8 == 0 and H <= 8192, "H")
    out = torch.empty_like(x) if out is None else out
    check(_lib.lib().ragk_layernorm(x.data_ptr(), x.stride(0), ptr(resid), resid.stride(0) if resid is not None else 0,
                                    g.data_ptr(), b.data_ptr(), out.data_ptr(), out.stride(0), T, H, float(eps),
                                    stream_ptr()), "ragk_layernorm")
    return out


def embed(ids, table, out=None, carry=None, prev=None):
    """Embedding gather. carry/prev (asynchronous decode): rows with carry[t] >= 0 take their token id
    from prev[carry[t]] (the previous step's sampled tokens on the device) and store it into ids[t]."""
    _req(ids.dtype == torch.int32 and ids.is_cuda and ids.is_contiguous(), "ids int32")
    V, H = table.shape
    out = torch.empty((ids.numel(), H), dtype=table.dtype, device=table.device) if out is None else out
    if carry is None:
        check(_lib.lib().ragk_embed(ids.data_ptr(), table.data_ptr(), out.data_ptr(), ids.numel(), H, V,
                                    stream_ptr()), "ragk_embed")
        return out
    _req(carry.dtype == torch.int32 and prev.dtype == torch.int32 and carry.numel() >= ids.numel(), "carry int32")
    check(_lib.lib().ragk_embed_carry(ids.data_ptr(), carry.data_ptr(), prev.data_ptr(), table.data_ptr(),
                                      out.data_ptr(), ids.numel(), H, V, stream_ptr()), "ragk_embed_carry")
    return out


def embed_ln(ids, pos_ids, word, pos, type_row, g, b, eps, do_ln=True, out=None):
    _req(ids.dtype == torch.int32 and pos_ids.dtype == torch.int32, "int32 ids")
    _req(int(ids.numel()) == int(pos_ids.numel()), "ids/pos_ids")
    H = word.shape[1]
    out = torch.empty((ids.numel(), H), dtype=word.dtype, device=word.device) if out is None else out
    check(_lib.lib().ragk_embed_ln(ids.data_ptr(), pos_ids.data_ptr(), word.data_ptr(), pos.data_ptr(),
                                   ptr(type_row), ptr(g), ptr(b), out.data_ptr(), ids.numel(), H, float(eps),
                                   int(do_ln), stream_ptr()), "ragk_embed_ln")
    return out


def rope_kv(qkv, positions, cos_t, sin_t, slots, k_cache, v_cache, Hq, Hkv, D, apply_rope=True):
    """In-place RoPE on q and k (inside qkv [T, (Hq+2Hkv)*D]) + paged cache write."""
    _bf16_2d(qkv, "qkv")
    T = qkv.shape[0]
    _req(qkv.shape[1] >= (Hq + 2 * Hkv) * D, "qkv width")
    _req(positions.dtype == torch.int32 and positions.numel() == T, "positions")
    if slots is not None:
        _req(slots.dtype == torch.int32 and slots.numel() == T, "slots")
        _req(k_cache.dim() == 4 and k_cache.shape[1] == Hkv and k_cache.shape[3] == D, "cache layout")
    BS = k_cache.shape[2] if k_cache is not None else 64
    check(_lib.lib().ragk_rope_kv(qkv.data_ptr(), qkv.stride(0), positions.data_ptr(), ptr(cos_t), ptr(sin_t),
                                  ptr(slots), ptr(k_cache), ptr(v_cache), T, Hq, Hkv, D, BS, int(apply_rope),
                                  stream_ptr()), "ragk_rope_kv")


def add_partials_rmsnorm(P, h, w, eps, out=None):
    """h <- bf16(h + bf16(P.sum(0))) in place; returns rmsnorm(h) * w (split-K decode consumer)."""
    _bf16_2d(h, "h")
    M, H = h.shape
    _req(P.dtype == torch.float32 and P.is_contiguous() and P.dim() == 3 and P.shape[1:] == (M, H), "partials shape")
    _req(w.is_cuda and w.dtype == torch.bfloat16 and w.numel() == H, "norm weight")
    out = torch.empty_like(h) if out is None else out
    _req(out.shape == (M, H) and out.stride(1) == 1, "out")
    check(_lib.lib().ragk_add_partials_rmsnorm(P.data_ptr(), P.shape[0], M, h.data_ptr(), h.stride(0), w.data_ptr(),
                                               out.data_ptr(), out.stride(0), H, float(eps), stream_ptr()),
          "ragk_add_partials_rmsnorm")
    return out


def rope_kv_partials(P, q_out, positions, cos_t, sin_t, slots, k_cache, v_cache, Hq, Hkv, D):
    """qkv = bf16(P.sum(0)); RoPE'd q -> q_out[:, :Hq*D]; RoPE'd k and v -> paged cache."""
    _req(P.dtype == torch.float32 and P.is_contiguous() and P.dim() == 3, "partials")
    S, T, ldp = P.shape
    _req(ldp >= (Hq + 2 * Hkv) * D, "qkv width")
    _bf16_2d(q_out, "q_out")
    _req(q_out.shape[0] == T and q_out.shape[1] >= Hq * D, "q_out shape")
    _req(positions.dtype == torch.int32 and positions.numel() == T, "positions")
    _req(slots is not None and slots.dtype == torch.int32 and slots.numel() == T, "slots")
    _req(k_cache.dim() == 4 and k_cache.shape[1] == Hkv and k_cache.shape[3] == D, "cache layout")
    check(_lib.lib().ragk_rope_kv_partials(P.data_ptr(), S, T, ldp, q_out.data_ptr(), q_out.stride(0),
                                           positions.data_ptr(), ptr(cos_t), ptr(sin_t), slots.data_ptr(),
                                           k_cache.data_ptr(), v_cache.data_ptr(), Hq, Hkv, D, k_cache.shape[2],
                                           stream_ptr()), "ragk_rope_kv_partials")


def pool_l2norm(hidden, cu, mode="cls", normalize=True, out=None):
    _bf16_2d(hidden, "hidden")
    B = cu.numel() - 1
    H = hidden.shape[1]
    _req(H <= 2048, "H <= 2048")
    m = {"cls": 0, "mean": 1, "last": 2}[mode]
    out = torch.empty((B, H), dtype=torch.float32, device=hidden.device) if out is None else out
    check(_lib.lib().ragk_pool_l2norm(hidden.data_ptr(), hidden.stride(0), cu.data_ptr(), out.data_ptr(), B, H, m,
                                      int(normalize), stream_ptr()), "ragk_pool_l2norm")
    return out


def silu_mul(x, out=None):
    _bf16_2d(x, "x")
    T, I2 = x.shape
    I = I2 // 2
    out = torch.empty((T, I), dtype=x.dtype, device=x.device) if out is None else out
    check(_lib.lib().ragk_silu_mul(x.data_ptr(), x.stride(0), out.data_ptr(), out.stride(0), T, I, stream_ptr()),
          "ragk_silu_mul")
    return out


def gather_rows(x, idx, out=None):
    _bf16_2d(x, "x")
    _req(idx.dtype == torch.int32 and idx.is_cuda, "idx int32")
    n = idx.numel()
    out = torch.empty((n, x.shape[1]), dtype=x.dtype, device=x.device) if out is None else out
    check(_lib.lib().ragk_gather_rows(x.data_ptr(), x.stride(0), idx.data_ptr(), out.data_ptr(), out.stride(0), n,
                                      x.shape[1], stream_ptr()), "ragk_gather_rows")
    return out


# ----------------------------------------------------------------------------- attention
def prefill_qtile(Hq, Hkv):
    """Query rows per prefill-attention block (the tile list must be built with the kernel's value):
    64 when 4 query heads share a KV head (the 8-wave kernels, two 32-row groups per K/V tile), else
    128 / heads-per-block (attention.hip ragk_attn_prefill_qtile)."""
    G = Hq // Hkv
    GB = 4 if G % 4 == 0 else (2 if G % 2 == 0 else 1)
    return 32 * ((8 if GB == 4 else 4) // GB)


def build_prefill_tiles(q_lens, Hq, Hkv):
    """(seq, q_start) work list, heaviest (latest query positions) first."""
    import numpy as np

    qt = prefill_qtile(Hq, Hkv)
    ql = np.asarray(q_lens, dtype=np.int64)
    nt = (ql + qt - 1) // qt
    seq = np.repeat(np.arange(len(ql)), nt)
    first = np.repeat(np.cumsum(nt) - nt, nt)
    q0 = (np.arange(int(nt.sum())) - first) * qt
    order = np.argsort(-q0, kind="stable")
    return torch.from_numpy(np.stack([seq[order], q0[order]], 1).astype(np.int32)).reshape(-1, 2)


def attn_prefill(q, k, v, cu_q, kv_lens, tiles, out, Hq, Hkv, D, causal=True, paged=True, block_tables=None,
                 cu_kv=None, kv_stride=0, scale=None):
    """q: [T, >=Hq*D] bf16 (row stride arbitrary). paged: k/v caches [nb, Hkv, 64, D];
    else packed k/v row pointers with `kv_stride` (element stride per token)."""
    _req(q.dtype == torch.bfloat16 and q.stride(-1) == 1, "q")
    _req(tiles.dtype == torch.int32 and tiles.is_cuda and tiles.is_contiguous(), "tiles int32 on GPU")
    _req(D in (32, 64, 128), "head_dim must be 32/64/128")
    if paged:
        _req(k.dim() == 4 and k.shape[2] == 64 and k.shape[1] == Hkv and k.shape[3] == D, "paged cache [nb,Hkv,64,D]")
        _req(block_tables is not None and block_tables.dtype == torch.int32, "block_tables int32")
        _req(block_tables.stride(0) <= 2048, "prefill block tables wider than 2048 blocks (128k tokens)")
    scale = 1.0 / math.sqrt(D) if scale is None else scale
    n_tiles = tiles.shape[0]
    if paged:
        _req(v.shape == k.shape, "paged k/v caches differ in shape")
        kv_stride = k.shape[0]  # paged: the cache block count (sizes the kernel's buffer descriptors)
    check(_lib.lib().ragk_attn_prefill(
        q.data_ptr(), q.stride(0), k.data_ptr(), v.data_ptr(), kv_stride, ptr(block_tables),
        block_tables.stride(0) if block_tables is not None else 0, cu_q.data_ptr(), ptr(cu_kv), kv_lens.data_ptr(),
        tiles.data_ptr(), n_tiles, out.data_ptr(), out.stride(0), Hq, Hkv, D, int(causal), int(paged), float(scale),
        stream_ptr()), "ragk_attn_prefill")
    return out


DECODE_TARGET_BLOCKS = 512
DECODE_MIN_TILES = 4


def decode_partitions(max_kv_len, batch, Hkv, target_blocks=None, min_tiles=None):
    """(part_tiles, max_parts) for split-K decode: grid = max_parts x Hkv x batch >= target_blocks.

    The kernel spreads each sequence's actual KV tiles evenly over the max_parts partitions
    (at least ``part_tiles`` = min_tiles tiles each, attention.hip:decode_part_tiles), so the grid can
    be sized once for the longest allowed context (hipGraph capture) without idle partitions."""
    target_blocks = DECODE_TARGET_BLOCKS if target_blocks is None else target_blocks
    min_tiles = DECODE_MIN_TILES if min_tiles is None else min_tiles
    max_kt = max(1, (max_kv_len + 63) // 64)
    if DECODE_NW8_MIN_PAIRS > 0 and batch * Hkv >= DECODE_NW8_MIN_PAIRS:
        return min_tiles, 1  # one 8-wave block per (sequence, KV head), no merge (attention.hip NW = 8)
    mp = max(1, min(-(-target_blocks // (batch * Hkv)), -(-max_kt // min_tiles)))
    return min_tiles, mp


# One partition per (sequence, KV head) in 8-wave blocks once batch x KV heads reaches this (>= one block
# per CU): the same KV bytes in flight as two 4-wave partition blocks, and no merge launch (0 = off).
# Batch 32: decode step 6.96 -> 6.86-6.90 ms (profiles/decode_nw8_ab_r4.log).
DECODE_NW8_MIN_PAIRS = 256


# Non-temporal K / V loads in the split-K decode attention once batch x KV heads reaches this: at batch 32
# over 5.2k-token contexts (TP=1, 8 KV heads) the KV stream (681 MB per layer) is read once per step, and
# the nt policy keeps it from evicting the L2 / Infinity Cache lines the other kernels reuse: decode step
# 7.60 -> 7.33 ms (profiles/decode_nt_ab_r4.log); batch 1 / 4 neutral-to-worse, and the TP=8 shard's
# 1-KV-head stream at batch 32 (85 MB per layer) 2.33 -> 2.40 ms with nt (profiles/tp_nt_ab_r4.log).
DECODE_NT_MIN_BH = 64


# The single-partition grid (DECODE_NW8_MIN_PAIRS) on 4-wave blocks whose K tiles arrive by LDS-DMA in 1 KiB
# pieces like the V tiles (attention.hip KL), instead of 8-wave blocks loading K as 64-B row pieces into
# registers: batch-32 decode attention over 5.2k-token contexts 114.2-116.8 -> 109.5-110.1 us per layer
# (5.9-6.0 -> 6.3 TB/s of KV; with +-150-token context jitter 116-118 -> 110-111 us),
# tools/attn_decode_probe.py, profiles/attn_decode_probe_r6.log.
DECODE_KL = os.environ.get("RAGK_DECODE_KL", "1") != "0"


def _set_decode_nt(B, Hkv):
    L = _lib.lib()
    check(L.ragk_attn_decode_set_nt(1 if B * Hkv >= DECODE_NT_MIN_BH else 0), "ragk_attn_decode_set_nt")
    check(L.ragk_attn_decode_set_nw8(DECODE_NW8_MIN_PAIRS), "ragk_attn_decode_set_nw8")
    check(L.ragk_attn_decode_set_kl(1 if DECODE_KL else 0), "ragk_attn_decode_set_kl")


def attn_decode(q, k_cache, v_cache, block_tables, kv_lens, out, Hq, Hkv, D, part_tiles, max_parts, ws_o=None,
                ws_ml=None, scale=None):
    B = kv_lens.numel()
    _req(k_cache.dim() == 4 and k_cache.shape[2] == 64 and k_cache.shape[3] == D, "paged cache")
    _req(block_tables.dtype == torch.int32 and block_tables.shape[0] >= B, "block_tables")
    _req(kv_lens.dtype == torch.int32, "kv_lens int32")
    G = Hq // Hkv
    _req(G <= 16, "G <= 16")
    if max_parts > 1:
        if ws_o is None:
            ws_o = torch.empty((B, Hq, max_parts, D), dtype=torch.float32, device=q.device)
            ws_ml = torch.empty((B, Hq, max_parts, 2), dtype=torch.float32, device=q.device)
        _req(ws_o.numel() >= B * Hq * max_parts * D and ws_ml.numel() >= B * Hq * max_parts * 2, "workspace")
    scale = 1.0 / math.sqrt(D) if scale is None else scale
    _set_decode_nt(B, Hkv)
    check(_lib.lib().ragk_attn_decode(
        q.data_ptr(), q.stride(0), k_cache.data_ptr(), v_cache.data_ptr(), block_tables.data_ptr(),
        block_tables.stride(0), kv_lens.data_ptr(), ptr(ws_o), ptr(ws_ml), out.data_ptr(), out.stride(0), B, Hq, Hkv,
        D, part_tiles, max_parts, float(scale), stream_ptr()), "ragk_attn_decode")
    return out


def attn_decode_rope(P, positions, cos_t, sin_t, slots, k_cache, v_cache, block_tables, kv_lens, out, Hq, Hkv, D,
                     part_tiles, max_parts, ws_o=None, ws_ml=None, scale=None, defer_merge=False):
    """Decode attention straight from the qkv projection's split-K partial slabs P [S, B, ldp] (fp32):
    q / k RoPE, the KV append at `slots` and the attention in one launch -- the same result as
    rope_kv_partials followed by attn_decode (bit-identical), one kernel fewer per layer."""
    _req(P.dtype == torch.float32 and P.is_contiguous() and P.dim() == 3, "partials")
    S, B, ldp = P.shape
    _req(ldp >= (Hq + 2 * Hkv) * D and D % 64 == 0, "qkv width")
    _req(kv_lens.numel() == B, "one partial row per sequence")
    _req(positions.dtype == torch.int32 and positions.numel() == B, "positions")
    _req(slots is not None and slots.dtype == torch.int32 and slots.numel() == B, "slots")
    _req(k_cache.dim() == 4 and k_cache.shape[1] == Hkv and k_cache.shape[2] == 64 and k_cache.shape[3] == D,
         "paged cache")
    _req(block_tables.dtype == torch.int32 and block_tables.shape[0] >= B, "block_tables")
    _req(kv_lens.dtype == torch.int32, "kv_lens int32")
    _req(Hq // Hkv <= 16, "G <= 16")
    if max_parts > 1:
        if ws_o is None:
            ws_o = torch.empty((B, Hq, max_parts, D), dtype=torch.float32, device=P.device)
            ws_ml = torch.empty((B, Hq, max_parts, 2), dtype=torch.float32, device=P.device)
        _req(ws_o.numel() >= B * Hq * max_parts * D and ws_ml.numel() >= B * Hq * max_parts * 2, "workspace")
    scale = 1.0 / math.sqrt(D) if scale is None else scale
    if defer_merge:  # the partitions stay unmerged for gemm_part_merge (no reduce launch)
        _req(max_parts > 1 and ws_o is not None, "deferred merge needs a partition workspace")
    lib = _lib.lib()
    _set_decode_nt(B, Hkv)
    if defer_merge:
        lib.ragk_attn_decode_set_defer(1)
    try:
        check(lib.ragk_attn_decode_rope(
            P.data_ptr(), S, ldp, positions.data_ptr(), slots.data_ptr(), cos_t.data_ptr(), sin_t.data_ptr(),
            k_cache.data_ptr(), v_cache.data_ptr(), block_tables.data_ptr(), block_tables.stride(0),
            kv_lens.data_ptr(), ptr(ws_o), ptr(ws_ml), out.data_ptr(), out.stride(0), B, Hq, Hkv, D, part_tiles,
            max_parts, float(scale), stream_ptr()), "ragk_attn_decode_rope")
    finally:
        if defer_merge:
            lib.ragk_attn_decode_set_defer(0)
    return out


# ----------------------------------------------------------------------------- sampling
TOPK_CHUNK = 16384  # vocab entries per top-k workgroup (128k vocab -> 7 workgroups per row)


def topk_chunks(V, K, max_cand=512):
    """Workgroups per row for the candidate top-k: enough to fill the chip at decode batch
    sizes, few enough that chunks*K candidates (x TP ranks) stay cheap to merge."""
    return max(1, min(V // TOPK_CHUNK, max_cand // K, 64))


def topk_candidates(logits, K, vocab_offset=0, max_cand=512, chunks=None, cand_v=None, cand_i=None):
    """Per-row top-K of a (vocab-shard of) fp32 logits -> (values, global ids) [B, chunks*K]:
    `chunks` sorted-descending lists of K, one per vocab chunk; the sampler merges them."""
    _req(logits.dtype == torch.float32 and logits.is_cuda and logits.stride(1) == 1, "logits fp32")
    B, V = logits.shape
    _req(1 <= K <= 256, "1 <= K <= 256")
    chunks = topk_chunks(V, K, max_cand) if chunks is None else int(chunks)
    _req(1 <= chunks <= 64, "1 <= chunks <= 64")
    if cand_v is None:
        cand_v = torch.empty((B, chunks * K), dtype=torch.float32, device=logits.device)
        cand_i = torch.empty((B, chunks * K), dtype=torch.int32, device=logits.device)
    _req(cand_v.shape == (B, chunks * K) and cand_i.shape == (B, chunks * K), "candidate buffers [B, chunks*K]")
    check(_lib.lib().ragk_topk_candidates(logits.data_ptr(), logits.stride(0), B, V, K, vocab_offset, chunks,
                                          cand_v.data_ptr(), cand_i.data_ptr(), stream_ptr()), "ragk_topk_candidates")
    return cand_v, cand_i


# candidate lists rank-merged in the sampler (no full sort) when rows ask for top_k <= 64
SAMPLE_LIST_MERGE = True


def sample_candidates(cand_v, cand_i, temps, top_ks, top_ps, seeds, steps, out_tok=None, out_lp=None, list_len=None):
    """list_len: the candidates are n / list_len sorted lists of list_len (topk_candidates output);
    lets rows with top_k <= 64 merge the lists by rank instead of sorting every candidate."""
    B, n = cand_v.shape
    _req(n <= 2048, "<= 2048 candidates")
    _req(temps.dtype == torch.float32 and top_ks.dtype == torch.int32 and top_ps.dtype == torch.float32, "param dtypes")
    _req(seeds.dtype == torch.int64 and steps.dtype == torch.int32, "seeds int64 / steps int32")
    out_tok = torch.empty(B, dtype=torch.int32, device=cand_v.device) if out_tok is None else out_tok
    if list_len and SAMPLE_LIST_MERGE:
        _req(n % list_len == 0, "candidate lists")
        check(_lib.lib().ragk_sample_candidates_lists(cand_v.data_ptr(), cand_i.data_ptr(), B, n, int(list_len),
                                                      temps.data_ptr(), top_ks.data_ptr(), top_ps.data_ptr(),
                                                      seeds.data_ptr(), steps.data_ptr(), out_tok.data_ptr(),
                                                      ptr(out_lp), stream_ptr()), "ragk_sample_candidates_lists")
        return out_tok
    check(_lib.lib().ragk_sample_candidates(cand_v.data_ptr(), cand_i.data_ptr(), B, n, temps.data_ptr(),
                                            top_ks.data_ptr(), top_ps.data_ptr(), seeds.data_ptr(), steps.data_ptr(),
                                            out_tok.data_ptr(), ptr(out_lp), stream_ptr()), "ragk_sample_candidates")
    return out_tok


# ----------------------------------------------------------------------------- search
def l2_search_set_mfma_min_nq(n):
    """Batches of at least n queries (k <= 8, d % 32 == 0) take the MFMA ||x||^2+||q||^2-2x.q path."""
    check(_lib.lib().ragk_l2_search_set_mfma_min_nq(int(n)), "ragk_l2_search_set_mfma_min_nq")


_search_ws = {}
_search_lock = threading.Lock()


def _search_out(nq, k, device):
    """(D fp32 [nq, k], I int64 [nq, k]) as views of ONE allocation (the merge kernel writes int64 ids)."""
    buf = torch.empty(nq * k * 3, dtype=torch.int32, device=device)
    return buf[2 * nq * k:].view(torch.float32).view(nq, k), buf[:2 * nq * k].view(torch.int64).view(nq, k)


def _search_partials(n_entries, device):
    """Per-(device, stream) grow-only partial-list workspace (fp32 distances + int32 ids). Callers hold
    _search_lock from here until both kernels of the search are enqueued, so two searches on one stream
    never interleave their scan / merge pair over the same buffer."""
    key = (str(device), stream_ptr())
    ws = _search_ws.get(key)
    if ws is None or ws.numel() < 2 * n_entries:
        ws = torch.empty(max(2 * n_entries, 1 << 16), dtype=torch.int32, device=device)
        _search_ws[key] = ws
    return ws[:n_entries].view(torch.float32), ws[n_entries:2 * n_entries]


def l2_search(xt, cap, n, q, k, row_begin=0, ids_map=None):
    """Exact squared-L2 top-k over rows [row_begin, n) of a column-major store xt[d][cap]
    (csrc/kernels/search.hip: l2_scan with wave-resident running top lists + one list merge; batches
    of >= 16 queries with k <= 8 on the fp32-MFMA distance GEMM, faiss' BLAS form).
    Returns (D fp32 [nq,k], I int64 [nq,k]) with faiss padding semantics (-1, FLT_MAX).
    Host cost per call: one output allocation and two ctypes calls (the partial lists live in a
    cached workspace), so a single-query search is not dominated by launch overhead."""
    _req(xt.is_cuda and xt.dtype == torch.float32 and xt.is_contiguous() and xt.dim() == 2, "xt fp32 [d, cap]")
    _req(q.is_cuda and q.dtype == torch.float32 and q.is_contiguous() and q.dim() == 2, "q fp32 [nq, d]")
    d = xt.shape[0]
    nq = q.shape[0]
    _req(q.shape[1] == d, "dim mismatch")
    _req(1 <= k <= 64, "1 <= k <= 64")
    _req(xt.shape[1] == cap and 0 <= row_begin <= max(row_begin, n) <= cap, "rows within the store")
    _req(ids_map is None or (ids_map.dtype == torch.int32 and ids_map.is_cuda and ids_map.numel() >= n), "ids_map")
    L = _lib.lib()
    od, oi = _search_out(nq, k, q.device)
    if nq == 0:
        return od, oi
    G = L.ragk_l2_search_groups(row_begin, max(n, row_begin), nq, k, d)
    with _search_lock:
        pd, pi = _search_partials(nq * G * k, q.device)
        check(L.ragk_l2_search(xt.data_ptr(), cap, d, row_begin, max(n, row_begin), q.data_ptr(), nq, k,
                               ptr(ids_map), pd.data_ptr(), pi.data_ptr(), od.data_ptr(), oi.data_ptr(), stream_ptr()),
              "ragk_l2_search")
    return od, oi


def ivf_search(xt, cap, q, probes, offsets, ids_map, k, max_list=None, ends=None):
    """IVF-Flat scan of the probed lists (one block per (query, probe), wave-resident top lists,
    then one list merge). probes int32 [nq, nprobe] (device; -1 = no list); list i occupies store rows
    [offsets[i], ends[i]) (ends None: packed lists, offsets has nlist+1 entries); ids_map int32 [cap]
    original id of every store row. max_list is accepted for API compatibility (unused)."""
    _req(xt.dtype == torch.float32 and q.dtype == torch.float32 and q.is_contiguous(), "fp32")
    _req(probes.dtype == torch.int32 and offsets.dtype == torch.int32 and ids_map.dtype == torch.int32, "int32")
    _req(probes.is_contiguous() and probes.is_cuda and offsets.is_cuda and ids_map.is_cuda, "device int32")
    _req(ends is None or (ends.dtype == torch.int32 and ends.is_cuda), "ends int32")
    d = xt.shape[0]
    nq, nprobe = probes.shape
    _req(1 <= k <= 64 and d <= 2048 and nprobe >= 1, "k <= 64, d <= 2048")
    od, oi = _search_out(nq, k, q.device)
    if nq == 0:
        return od, oi
    with _search_lock:
        pd, pi = _search_partials(nq * nprobe * k, q.device)
        check(_lib.lib().ragk_ivf_search(xt.data_ptr(), cap, d, q.data_ptr(), nq, probes.data_ptr(), nprobe,
                                         offsets.data_ptr(), ptr(ends), ids_map.data_ptr(), k, pd.data_ptr(),
                                         pi.data_ptr(), od.data_ptr(), oi.data_ptr(), stream_ptr()), "ragk_ivf_search")
    return od, oi


def kmeans_assign(x, c, cnorm=None, scores=None):
    """argmin_j ||x_i - c_j||^2 (ties -> lower j) and that squared distance, on the MFMA distance-GEMM
    kernel (exact fp32 products). x [n, d], c [k, d] fp32 contiguous on the GPU; d % 64 == 0, <= 1024.
    scores (optional fp32 [n, k]): receives -(||c_j||^2 - 2 x_i.c_j), the numbers the argmin ranks."""
    _req(x.is_cuda and x.dtype == torch.float32 and x.is_contiguous() and x.dim() == 2, "x fp32 [n, d]")
    _req(c.is_cuda and c.dtype == torch.float32 and c.is_contiguous() and c.shape[1] == x.shape[1], "c fp32 [k, d]")
    n, d = x.shape
    _req(d % 64 == 0 and d <= 1024, "d % 64 == 0 and d <= 1024")
    _req(scores is None or (scores.is_cuda and scores.dtype == torch.float32 and scores.is_contiguous()
                            and tuple(scores.shape) == (n, c.shape[0])), "scores fp32 [n, k]")
    if cnorm is None:
        cnorm = (c * c).sum(1)
    a = torch.empty(n, dtype=torch.int32, device=x.device)
    dist = torch.empty(n, dtype=torch.float32, device=x.device)
    check(_lib.lib().ragk_kmeans_assign(x.data_ptr(), n, d, c.data_ptr(), cnorm.contiguous().data_ptr(), c.shape[0],
                                        a.data_ptr(), dist.data_ptr(), ptr(scores), stream_ptr()), "ragk_kmeans_assign")
    return a, dist


def coarse_probes(x, c, cnorm, nprobe):
    """IVF coarse search: the nprobe nearest centroids of every row of x (int32 [n, nprobe], ties ->
    lower id), ranked by the SAME scores kmeans_assign's argmin uses, so top-1 == the list assignment."""
    n, nl = x.shape[0], c.shape[0]
    _req(1 <= nprobe <= min(256, nl) and nl <= 24576, "1 <= nprobe <= min(256, nlist), nlist <= 24576")
    sc = torch.empty((n, nl), dtype=torch.float32, device=x.device)
    kmeans_assign(x, c, cnorm, scores=sc)
    _, idx = topk_candidates(sc, nprobe, chunks=1)
    return idx


def l2_scatter(xt, cap, pos, x):
    """Store rows x [n, d] at slots pos (int32, each < cap) of the column-major store xt[d][cap]."""
    _req(x.dtype == torch.float32 and x.is_contiguous() and x.shape[1] == xt.shape[0], "x fp32 [n,d]")
    _req(pos.dtype == torch.int32 and pos.is_cuda and pos.numel() == x.shape[0], "pos int32 [n]")
    check(_lib.lib().ragk_l2_scatter(xt.data_ptr(), cap, xt.shape[0], pos.data_ptr(), x.data_ptr(), x.shape[0],
                                     stream_ptr()), "ragk_l2_scatter")


def l2_append(xt, cap, n0, x):
    _req(x.dtype == torch.float32 and x.is_contiguous() and x.shape[1] == xt.shape[0], "x fp32 [n,d]")
    check(_lib.lib().ragk_l2_append(xt.data_ptr(), cap, xt.shape[0], n0, x.data_ptr(), x.shape[0], stream_ptr()),
          "ragk_l2_append")


