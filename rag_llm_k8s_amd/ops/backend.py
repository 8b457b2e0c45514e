"""Compute backends used by the model code.

``NativeBackend``  -- GPU: every op is a gfx950 HIP kernel from ``libragk_hip.so``
                      (no eager/torch fallback: a missing library raises).
``TorchBackend``   -- CPU: the fp32-accumulating torch reference ops (BASELINE config 1,
                      CPU plumbing), also used as the oracle in tests.

Both expose the same methods with the same tensor layouts (paged KV cache
[nblocks, Hkv, 64, D], packed gate/up weights, fused qkv rows), so the Llama /
encoder / GPT-2 model code and the serving engine are device-agnostic.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import List, Optional

import torch

from . import reference as R
from .fp8 import Fp8Weight, reference_linear

KV_BLOCK = 64


@dataclass
class AttnMeta:
    """Attention metadata for one forward step (device tensors + host mirrors)."""
    kind: str  # "prefill" | "decode"
    kv_lens: torch.Tensor  # int32 [S]
    block_tables: torch.Tensor  # int32 [S, maxb]
    cu_q: Optional[torch.Tensor] = None  # int32 [S+1] (prefill)
    tiles: Optional[torch.Tensor] = None  # int32 [n,2] (prefill)
    part_tiles: int = 4  # decode split-K
    max_parts: int = 1
    ws_o: Optional[torch.Tensor] = None
    ws_ml: Optional[torch.Tensor] = None
    host_kv_lens: List[int] = field(default_factory=list)
    host_q_lens: List[int] = field(default_factory=list)


class TorchBackend:
    name = "torch"

    def __init__(self, device="cpu"):
        self.device = torch.device(device)

    # GEMM family ---------------------------------------------------------------
    def gemm(self, x, w, bias=None, resid=None, epi="none", out=None, out_f32=False):
        if isinstance(w, Fp8Weight):
            y = reference_linear(x, w, bias, resid, epi=epi, out_f32=out_f32)
        else:
            y = R.linear(x, w, bias, resid, epi=epi, out_f32=out_f32)
        if out is not None:
            out.copy_(y)
            return out
        return y

    def rmsnorm(self, x, w, eps, out=None):
        y = R.rmsnorm(x, w, eps)
        if out is not None:
            out.copy_(y)
            return out
        return y

    def layernorm(self, x, g, b, eps, out=None, resid=None):
        y = R.layernorm(x, g, b, eps, resid=resid)
        if out is not None:
            out.copy_(y)
            return out
        return y

    def embed(self, ids, table, out=None, carry=None, prev=None):
        if carry is not None:
            c = carry[:ids.numel()].long()
            ids.copy_(torch.where(c >= 0, prev.long()[c.clamp(min=0)], ids.long()).to(ids.dtype))
        y = table[ids.long()]
        if out is not None:
            out.copy_(y)
            return out
        return y

    def embed_ln(self, ids, pos_ids, word, pos, type_row, g, b, eps, do_ln=True):
        h = word[ids.long()].float() + pos[pos_ids.long()].float()
        if type_row is not None:
            h = h + type_row.float().reshape(1, -1)
        if do_ln:
            h = torch.nn.functional.layer_norm(h, (h.shape[-1],), g.float(), b.float(), eps)
        return h.to(word.dtype)

    def gather_rows(self, x, idx):
        return x[idx.long()]

    def silu_mul(self, x):
        I = x.shape[1] // 2
        return (torch.nn.functional.silu(x[:, :I].float()) * x[:, I:].float()).to(x.dtype)

    def rope_kv(self, qkv, positions, cos_t, sin_t, slots, kc, vc, Hq, Hkv, D, apply_rope=True):
        T = qkv.shape[0]
        q = qkv[:, :Hq * D].reshape(T, Hq, D)
        k = qkv[:, Hq * D:(Hq + Hkv) * D].reshape(T, Hkv, D)
        v = qkv[:, (Hq + Hkv) * D:(Hq + 2 * Hkv) * D].reshape(T, Hkv, D)
        if apply_rope:
            p = positions.long()
            q.copy_(R.apply_rope(q, p, cos_t, sin_t))
            k.copy_(R.apply_rope(k, p, cos_t, sin_t))
        if slots is not None and kc is not None:
            s = slots.long()
            ok = s >= 0
            s = s[ok]
            kc[s // KV_BLOCK, :, s % KV_BLOCK] = k[ok]
            vc[s // KV_BLOCK, :, s % KV_BLOCK] = v[ok]

    def gemm_rope_kv(self, x, w, positions, cos_t, sin_t, slots, kc, vc, Hq, Hkv, D):
        """qkv projection + rope_kv (the GPU backend fuses them into the GEMM epilogue)."""
        qkv = self.gemm(x, w)
        self.rope_kv(qkv, positions, cos_t, sin_t, slots, kc, vc, Hq, Hkv, D)
        return qkv


    # split-K decode path (GPU: gemm_part.hip + the consumers in norm.hip) ----------------
    enable_part = False  # the torch oracle runs the same dataflow when a test switches it on

    def part_ok(self, M, w):
        return self.enable_part and M <= 64

    def gemm_part(self, x, w):
        wf = w.dequant() if isinstance(w, Fp8Weight) else w.float()
        return (x.float() @ wf.t()).unsqueeze(0)

    def part_norm_ok(self, M, w):
        return self.enable_part and M <= 4 and not isinstance(w, Fp8Weight) and w.shape[1] <= 8192

    def part_silu_ok(self, M, w_gu, w_down):
        return (self.enable_part and M <= 4 and not isinstance(w_gu, Fp8Weight) and not isinstance(w_down, Fp8Weight)
                and w_down.shape[1] % 64 == 0)

    def gemm_part_gu(self, x, w):
        return self.gemm_part(x, w)

    def gemm_part_silu(self, pgu, w):
        gu = pgu.float().sum(0)
        M, K2 = gu.shape
        t = gu.view(M, K2 // 128, 2, 64)
        a = (torch.nn.functional.silu(t[:, :, 0, :]) * t[:, :, 1, :]).reshape(M, K2 // 2).to(torch.bfloat16)
        return self.gemm_part(a, w)

    def gemm_part_norm(self, h, gamma, eps, w):
        return self.gemm_part(R.rmsnorm(h, gamma, eps), w)

    def mlp_engine_ok(self, M, w_gu, w_down):
        return (self.enable_part and M == 1 and not isinstance(w_gu, Fp8Weight) and not isinstance(w_down, Fp8Weight)
                and w_down.shape[1] % 64 == 0)

    def mlp_engine(self, xn, w_gu, w_down, h):
        """h += W_down (silu(gate) * up) for one row: bf16 activations, one rounding of the residual add."""
        t = (xn.float() @ w_gu.float().t()).view(xn.shape[0], -1, 2, 64)  # packed [64 gate | 64 up] tiles
        a = (torch.nn.functional.silu(t[:, :, 0, :]) * t[:, :, 1, :]).reshape(xn.shape[0], -1).to(torch.bfloat16)
        h.copy_((h.float() + a.float() @ w_down.float().t()).to(h.dtype))
        return h

    def mlp_engine_tail(self, P, h, gamma, eps, w_gu, w_down):
        """add_partials_rmsnorm (o_proj slabs + residual + post-attention norm) then mlp_engine, one op."""
        return self.mlp_engine(self.add_partials_rmsnorm(P, h, gamma, eps), w_gu, w_down, h)

    def add_partials_rmsnorm(self, P, h, w, eps):
        h.copy_((h.float() + P.sum(0).to(h.dtype).float()).to(h.dtype))
        return R.rmsnorm(h, w, eps)

    def rope_kv_partials(self, P, q_out, positions, cos_t, sin_t, slots, kc, vc, Hq, Hkv, D):
        qkv = P.sum(0).to(q_out.dtype)
        self.rope_kv(qkv, positions, cos_t, sin_t, slots, kc, vc, Hq, Hkv, D)
        q_out[:, :Hq * D].copy_(qkv[:, :Hq * D])

    def attn_prefill(self, q, kc, vc, meta: AttnMeta, out, Hq, Hkv, D):
        T = q.shape[0]
        qq = q[:, :Hq * D].reshape(T, Hq, D)
        bt = meta.block_tables.cpu()
        lens = meta.host_kv_lens
        o = R.attention_varlen(qq, None, None, meta.cu_q.cpu(), lens, True, 1.0 / math.sqrt(D),
                               k_full=lambda s: R.paged_kv_view(kc, bt[s], lens[s], KV_BLOCK),
                               v_full=lambda s: R.paged_kv_view(vc, bt[s], lens[s], KV_BLOCK))
        out.copy_(o.reshape(T, Hq * D))
        return out

    def attn_decode_rope(self, P, positions, cos_t, sin_t, slots, kc, vc, meta: AttnMeta, out, Hq, Hkv, D,
                         defer_merge=False):
        q = torch.empty((P.shape[1], Hq * D), dtype=out.dtype, device=out.device)
        self.rope_kv_partials(P, q, positions, cos_t, sin_t, slots, kc, vc, Hq, Hkv, D)
        return self.attn_decode(q, kc, vc, meta, out, Hq, Hkv, D)

    def part_merge_ok(self, M, meta: AttnMeta, w, Hq, D):
        return False

    def prefill_nsplit(self, M, w):
        return 1

    def attn_decode(self, q, kc, vc, meta: AttnMeta, out, Hq, Hkv, D):
        B = q.shape[0]
        cu = torch.arange(B + 1, dtype=torch.int32)
        m = AttnMeta("prefill", meta.kv_lens, meta.block_tables, cu_q=cu, host_kv_lens=meta.host_kv_lens)
        return self.attn_prefill(q, kc, vc, m, out, Hq, Hkv, D)

    def attn_encoder(self, qkv, cu, lens_host, tiles, out, H, D):
        T = qkv.shape[0]
        q = qkv[:, :H * D].reshape(T, H, D)
        k = qkv[:, H * D:2 * H * D].reshape(T, H, D)
        v = qkv[:, 2 * H * D:3 * H * D].reshape(T, H, D)
        o = R.attention_varlen(q, k, v, cu.cpu(), lens_host, False, 1.0 / math.sqrt(D), cu_kv=cu.cpu())
        out.copy_(o.reshape(T, H * D))
        return out

    def pool_l2norm(self, hidden, cu, mode="cls", normalize=True):
        return R.pool_l2norm(hidden, cu.cpu(), mode=mode, normalize=normalize)

    # sampling -----------------------------------------------------------------
    def topk_candidates(self, logits, K, vocab_offset=0, max_cand=512, chunks=None):
        k = min(K, logits.shape[1])
        v, i = torch.topk(logits.float(), k, dim=-1)
        if k < K:
            v = torch.cat([v, torch.full((v.shape[0], K - k), float("-inf"))], 1)
            i = torch.cat([i, torch.full((i.shape[0], K - k), -1)], 1)
        return v, (i + vocab_offset).int()

    def sample_candidates(self, cand_v, cand_i, temps, top_ks, top_ps, seeds, steps, list_len=None):
        out = torch.empty(cand_v.shape[0], dtype=torch.int32)
        for b in range(cand_v.shape[0]):
            order = torch.argsort(cand_v[b], descending=True, stable=True)
            v, i = cand_v[b][order], cand_i[b][order]
            k = int(top_ks[b])
            k = len(v) if k <= 0 or k > len(v) else k
            v, i = v[:k], i[:k]
            t = float(temps[b])
            if t <= 0:
                out[b] = int(i[0])
                continue
            g = torch.Generator().manual_seed((int(seeds[b]) * 1000003 + int(steps[b])) & 0x7FFFFFFFFFFFFFFF)
            u = float(torch.rand(1, generator=g))
            _, _, pick = R.sample_from_logits_candidates(v, i, t, float(top_ps[b]), u)
            out[b] = pick
        return out


class NativeBackend(TorchBackend):
    name = "native"

    def __init__(self, device="cuda"):
        super().__init__(device)
        from . import native

        self.n = native
        native._lib.lib()  # fail loudly now if the gfx950 library is missing

    def gemm(self, x, w, bias=None, resid=None, epi="none", out=None, out_f32=False):
        if isinstance(w, Fp8Weight):
            return self.n.gemm_fp8(x, w, bias=bias, resid=resid, epi=epi, out=out, out_f32=out_f32)
        return self.n.gemm(x, w, bias=bias, resid=resid, epi=epi, out=out, out_f32=out_f32)

    def rmsnorm(self, x, w, eps, out=None):
        return self.n.rmsnorm(x, w, eps, out=out)

    def layernorm(self, x, g, b, eps, out=None, resid=None):
        return self.n.layernorm(x, g, b, eps, out=out, resid=resid)

    def embed(self, ids, table, out=None, carry=None, prev=None):
        return self.n.embed(ids, table, out=out, carry=carry, prev=prev)

    def embed_ln(self, ids, pos_ids, word, pos, type_row, g, b, eps, do_ln=True):
        return self.n.embed_ln(ids, pos_ids, word, pos, type_row, g, b, eps, do_ln=do_ln)

    def gather_rows(self, x, idx):
        return self.n.gather_rows(x, idx)

    def silu_mul(self, x):
        return self.n.silu_mul(x)

    def rope_kv(self, qkv, positions, cos_t, sin_t, slots, kc, vc, Hq, Hkv, D, apply_rope=True):
        self.n.rope_kv(qkv, positions, cos_t, sin_t, slots, kc, vc, Hq, Hkv, D, apply_rope=apply_rope)

    def gemm_rope_kv(self, x, w, positions, cos_t, sin_t, slots, kc, vc, Hq, Hkv, D):
        if self.n.gemm_rope_kv_ok(x, w, positions, cos_t, sin_t, slots, kc, vc, Hq, Hkv, D):
            return self.n.gemm_rope_kv(x, w, positions, cos_t, sin_t, slots, kc, vc, Hq, Hkv, D)
        qkv = self.gemm(x, w)
        self.rope_kv(qkv, positions, cos_t, sin_t, slots, kc, vc, Hq, Hkv, D)
        return qkv

    enable_part = __import__("os").environ.get("RAGK_DECODE_PART", "1") == "1"

    def part_ok(self, M, w):
        if not self.enable_part or M > 64:
            return False
        return self.n.gemm_part_slabs(M, w.shape[0], w.shape[1])[1] > 0

    def gemm_part(self, x, w):
        return self.n.gemm_part(x, w)

    def part_norm_ok(self, M, w):
        return self.enable_part and M <= 4 and not isinstance(w, Fp8Weight) and w.shape[1] in (4096, 8192)

    def gemm_part_norm(self, h, gamma, eps, w):
        return self.n.gemm_part_norm(h, gamma, eps, w)

    def part_silu_ok(self, M, w_gu, w_down):
        return self.enable_part and self.n.gemm_part_silu_ok(M, w_gu, w_down)

    def gemm_part_gu(self, x, w):
        return self.n.gemm_part_gu(x, w)

    def gemm_part_silu(self, pgu, w):
        return self.n.gemm_part_silu(pgu, w)

    def add_partials_rmsnorm(self, P, h, w, eps):
        return self.n.add_partials_rmsnorm(P, h, w, eps)

    def mlp_engine_ok(self, M, w_gu, w_down):
        return self.n.mlp_engine_ok(M, w_gu, w_down)

    def mlp_engine(self, xn, w_gu, w_down, h):
        return self.n.mlp_engine(xn, w_gu, w_down, h)

    def mlp_engine_tail(self, P, h, gamma, eps, w_gu, w_down):
        return self.n.mlp_engine_tail(P, h, gamma, eps, w_gu, w_down)

    def rope_kv_partials(self, P, q_out, positions, cos_t, sin_t, slots, kc, vc, Hq, Hkv, D):
        self.n.rope_kv_partials(P, q_out, positions, cos_t, sin_t, slots, kc, vc, Hq, Hkv, D)

    def attn_prefill(self, q, kc, vc, meta: AttnMeta, out, Hq, Hkv, D):
        return self.n.attn_prefill(q, kc, vc, meta.cu_q, meta.kv_lens, meta.tiles, out, Hq, Hkv, D, causal=True,
                                   paged=True, block_tables=meta.block_tables)

    def attn_decode_rope(self, P, positions, cos_t, sin_t, slots, kc, vc, meta: AttnMeta, out, Hq, Hkv, D,
                         defer_merge=False):
        return self.n.attn_decode_rope(P, positions, cos_t, sin_t, slots, kc, vc, meta.block_tables, meta.kv_lens, out,
                                       Hq, Hkv, D, meta.part_tiles, meta.max_parts, meta.ws_o, meta.ws_ml,
                                       defer_merge=defer_merge)

    def prefill_nsplit(self, M, w):
        if isinstance(w, Fp8Weight):
            return 1
        return self.n.prefill_nsplit(M, w.shape[0], w.shape[1])

    def gemm_splitk(self, x, w, nsplit):
        return self.n.gemm_splitk(x, w, nsplit)

    def part_merge_ok(self, M, meta: AttnMeta, w, Hq, D):
        return (self.enable_part and D == 128
                and self.n.gemm_part_merge_ok(M, w, Hq, meta.max_parts, meta.ws_o))

    def gemm_part_merge(self, attn_out, meta: AttnMeta, w, Hq):
        return self.n.gemm_part_merge(attn_out, meta.kv_lens, meta.part_tiles, meta.max_parts, meta.ws_o, meta.ws_ml,
                                      Hq, w)

    def attn_decode(self, q, kc, vc, meta: AttnMeta, out, Hq, Hkv, D):
        return self.n.attn_decode(q, kc, vc, meta.block_tables, meta.kv_lens, out, Hq, Hkv, D, meta.part_tiles,
                                  meta.max_parts, meta.ws_o, meta.ws_ml)

    def attn_encoder(self, qkv, cu, lens_host, tiles, out, H, D):
        return self.n.attn_prefill(qkv, qkv[:, H * D:], qkv[:, 2 * H * D:], cu, _lens_dev(cu), tiles, out, H, H, D,
                                   causal=False, paged=False, cu_kv=cu, kv_stride=qkv.stride(0))

    def pool_l2norm(self, hidden, cu, mode="cls", normalize=True):
        return self.n.pool_l2norm(hidden, cu, mode=mode, normalize=normalize)

    def topk_candidates(self, logits, K, vocab_offset=0, max_cand=512, chunks=None):
        return self.n.topk_candidates(logits, K, vocab_offset=vocab_offset, max_cand=max_cand, chunks=chunks)

    def sample_candidates(self, cand_v, cand_i, temps, top_ks, top_ps, seeds, steps, list_len=None):
        return self.n.sample_candidates(cand_v, cand_i, temps, top_ks, top_ps, seeds, steps, list_len=list_len)


def _lens_dev(cu):
    return (cu[1:] - cu[:-1]).contiguous()


def get_backend(device) -> TorchBackend:
    dev = torch.device(device)
    return NativeBackend(dev) if dev.type == "cuda" else TorchBackend(dev)
