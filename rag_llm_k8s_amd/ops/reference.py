"""Pure-torch reference implementations of every kernel in ``csrc/kernels``.

Two roles:
* numerics oracle for the GPU kernel tests (computed in fp32 on the same inputs);
* the CPU execution path (BASELINE config 1: CPU plumbing, no GPU).

Semantics follow the reference's dependencies (transformers' Llama / XLM-R / BERT /
GPT-2 modules, sentence-transformers pooling, faiss IndexFlatL2) as catalogued in
SURVEY.md §2.4.
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

EPI = {"none": 0, "bias": 1, "resid": 2, "bias_resid": 3, "bias_gelu": 4, "silu_mul": 5, "gelu": 6,
       "bias_gelu_tanh": 7}


def pack_gate_up(gate: torch.Tensor, up: torch.Tensor) -> torch.Tensor:
    """Pack [I,K] gate and up weights into the kernel layout: 128-row tiles of
    [64 gate rows | 64 up rows]. Requires I % 64 == 0."""
    I, K = gate.shape
    assert up.shape == gate.shape and I % 64 == 0, (gate.shape, up.shape)
    g = gate.reshape(I // 64, 64, K)
    u = up.reshape(I // 64, 64, K)
    return torch.stack([g, u], dim=1).reshape(2 * I, K).contiguous()


def unpack_gate_up(w: torch.Tensor):
    n2, K = w.shape
    t = w.reshape(n2 // 128, 2, 64, K)
    return t[:, 0].reshape(n2 // 2, K), t[:, 1].reshape(n2 // 2, K)


def linear(x, w, bias=None, resid=None, epi="none", out_f32=False):
    """C = x @ w^T with the fused epilogues of ragk_gemm (fp32 accumulate)."""
    xf = x.float()
    if epi == "silu_mul":
        g, u = unpack_gate_up(w)
        y = F.silu(xf @ g.float().t()) * (xf @ u.float().t())
    else:
        y = xf @ w.float().t()
        if bias is not None and "bias" in epi:
            y = y + bias.float()
        if resid is not None and "resid" in epi:
            y = y + resid.float()
        if epi in ("bias_gelu", "gelu"):
            y = F.gelu(y)
        elif epi == "bias_gelu_tanh":
            y = F.gelu(y, approximate="tanh")
    return y if out_f32 else y.to(x.dtype)


def rmsnorm(x, w, eps, resid=None):
    """HF LlamaRMSNorm; with resid: resid <- bf16(x + resid) first (in place)."""
    if resid is not None:
        resid.copy_((x.float() + resid.float()).to(resid.dtype))
        x = resid
    h = x.float()
    var = h.pow(2).mean(-1, keepdim=True)
    h = (h * torch.rsqrt(var + eps)).to(x.dtype)
    return (w.float() * h.float()).to(x.dtype)


def layernorm(x, g, b, eps, resid=None):
    h = x.float() if resid is None else x.float() + resid.float()
    return F.layer_norm(h, (h.shape[-1],), g.float(), b.float(), eps).to(x.dtype)


def rope_tables(head_dim, max_pos, theta=10000.0, scaling=None, dtype=torch.bfloat16):
    """cos/sin tables [max_pos, head_dim/2] (fp32 storing `dtype`-rounded values), with
    optional llama3 scaling dict {factor, low_freq_factor, high_freq_factor,
    original_max_position_embeddings} ([dep] modeling_rope_utils.py llama3 rule)."""
    inv_freq = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.int64).float() / head_dim))
    if scaling is not None and scaling.get("rope_type", scaling.get("type")) == "llama3":
        factor = scaling["factor"]
        low = scaling["low_freq_factor"]
        high = scaling["high_freq_factor"]
        old = scaling["original_max_position_embeddings"]
        low_wl, high_wl = old / low, old / high
        wavelen = 2 * math.pi / inv_freq
        inv_l = torch.where(wavelen > low_wl, inv_freq / factor, inv_freq)
        smooth = (old / wavelen - low) / (high - low)
        smoothed = (1 - smooth) * inv_l / factor + smooth * inv_l
        is_medium = (~(wavelen < high_wl)) & (~(wavelen > low_wl))
        inv_freq = torch.where(is_medium, smoothed, inv_l)
    pos = torch.arange(max_pos, dtype=torch.float32)
    freqs = torch.outer(pos, inv_freq.float())
    return freqs.cos().to(dtype).float().contiguous(), freqs.sin().to(dtype).float().contiguous()


def apply_rope(x, positions, cos_t, sin_t):
    """x: [T, H, D] -> rotate_half RoPE with bf16 op rounding (HF apply_rotary_pos_emb)."""
    dt = x.dtype
    c = cos_t[positions].to(dt)[:, None, :]
    s = sin_t[positions].to(dt)[:, None, :]
    c = torch.cat([c, c], -1)
    s = torch.cat([s, s], -1)
    half = x.shape[-1] // 2
    rot = torch.cat([-x[..., half:], x[..., :half]], -1)
    return (x * c) + (rot * s)


def attention_varlen(q, k, v, cu_q, kv_lens, causal, scale, cu_kv=None, k_full=None, v_full=None):
    """Reference attention over packed sequences.
    q: [Tq, Hq, D]; for each sequence s, keys are k_full(s)/v_full(s) of length kv_lens[s]
    (callables returning [L, Hkv, D]) or slices of packed k/v by cu_kv. Queries are the
    LAST q_len positions of the context."""
    Hq = q.shape[1]
    out = torch.empty_like(q)
    n = len(kv_lens)
    for s in range(n):
        q0, q1 = int(cu_q[s]), int(cu_q[s + 1])
        L = int(kv_lens[s])
        if k_full is not None:
            ks, vs = k_full(s), v_full(s)
        else:
            k0 = int(cu_kv[s])
            ks, vs = k[k0:k0 + L], v[k0:k0 + L]
        Hkv = ks.shape[1]
        rep = Hq // Hkv
        kk = ks.float().repeat_interleave(rep, dim=1).transpose(0, 1)  # [Hq, L, D]
        vv = vs.float().repeat_interleave(rep, dim=1).transpose(0, 1)
        qq = q[q0:q1].float().transpose(0, 1)  # [Hq, ql, D]
        att = (qq @ kk.transpose(1, 2)) * scale
        ql = q1 - q0
        if causal:
            qpos = torch.arange(L - ql, L)[:, None]
            kpos = torch.arange(L)[None, :]
            att = att.masked_fill(kpos > qpos, float("-inf"))
        p = att.softmax(-1)
        out[q0:q1] = (p @ vv).transpose(0, 1).to(q.dtype)
    return out


def paged_kv_view(cache, block_table, L, block_size):
    """Gather [L, Hkv, D] from a paged cache [nblocks, Hkv, BS, D]."""
    nb = (L + block_size - 1) // block_size
    blocks = cache[block_table[:nb].long()]  # [nb, Hkv, BS, D]
    return blocks.permute(0, 2, 1, 3).reshape(nb * block_size, cache.shape[1], cache.shape[3])[:L]


def pool_l2norm(hidden, cu, mode="cls", normalize=True):
    outs = []
    for b in range(len(cu) - 1):
        h = hidden[int(cu[b]):int(cu[b + 1])].float()
        if mode == "cls":
            v = h[0]
        elif mode == "mean":
            v = h.mean(0)
        else:
            v = h[-1]
        outs.append(v)
    o = torch.stack(outs)
    return F.normalize(o, p=2, dim=-1) if normalize else o


def sample_from_logits(logits, temperature, top_k, top_p, u=None):
    """Single-row HF-order sampler (temperature -> top-k -> top-p). Returns (kept token
    ids in descending-prob order, probabilities, pick). `u` in [0,1) draws the token."""
    x = logits.float()
    if temperature <= 0:
        return None, None, int(torch.argmax(x))
    x = x / temperature
    k = min(top_k if top_k > 0 else x.numel(), x.numel())
    vals, idx = torch.topk(x, k)
    probs = torch.softmax(vals, -1)
    cum_before = torch.cumsum(probs, 0) - probs
    keep = cum_before < top_p
    keep[0] = True
    kv, ki = vals[keep], idx[keep]
    p = torch.softmax(kv, -1)
    pick = None
    if u is not None:
        c = torch.cumsum(p, 0)
        j = int(torch.searchsorted(c, torch.tensor([u * float(c[-1])]), right=True)[0])
        pick = int(ki[min(j, len(ki) - 1)])
    return ki, p, pick


def sample_from_logits_candidates(vals, idx, temperature, top_p, u):
    """vals/idx: top-k candidates sorted descending. Applies temperature and top-p, then
    draws with uniform `u` (inverse CDF). Returns (kept ids, probs, picked id)."""
    x = vals.float() / temperature
    probs = torch.softmax(x, -1)
    cum_before = torch.cumsum(probs, 0) - probs
    keep = cum_before < top_p
    keep[0] = True
    ki = idx[keep]
    p = torch.softmax(x[keep], -1)
    c = torch.cumsum(p, 0)
    j = int(torch.searchsorted(c, torch.tensor([u * float(c[-1])]), right=True)[0])
    return ki, p, int(ki[min(j, len(ki) - 1)])


def l2_knn(xb, q, k):
    """faiss IndexFlatL2.search: squared L2, ascending; pad (-1, FLT_MAX)."""
    n = xb.shape[0]
    nq = q.shape[0]
    D = torch.full((nq, k), torch.finfo(torch.float32).max)
    I = torch.full((nq, k), -1, dtype=torch.int64)
    if n == 0:
        return D, I
    d = ((q[:, None, :].double() - xb[None, :, :].double()) ** 2).sum(-1).float()
    kk = min(k, n)
    dv, di = torch.sort(d, dim=1, stable=True)
    D[:, :kk] = dv[:, :kk]
    I[:, :kk] = di[:, :kk]
    return D, I
