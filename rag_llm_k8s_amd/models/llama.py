"""Llama-3.x decoder (8B / 70B / tiny) for the serving engine.

Reference: transformers' LlamaForCausalLM as loaded by /root/reference/llm/rag.py:24 and
driven by model.generate at :172 (per-layer structure [dep] modeling_llama.py:284-323).

MI355X-first design:
  * q/k/v fused into one [ (Hq+2Hkv)*D, H ] weight; gate/up packed into the
    [64 gate | 64 up]-row tile layout so SiLU(gate)*up is the GEMM epilogue;
  * residual adds are GEMM epilogues (o_proj, down_proj write h += x @ W^T in place);
  * RoPE + paged-KV write is one kernel; attention reads K/V only from the paged cache;
  * Megatron tensor parallelism: qkv / gate-up column-parallel, o / down row-parallel
    (2 all-reduces per layer over RCCL/xGMI), lm_head vocab-parallel (the sampler
    all-gathers only the per-rank top-k candidates -- exact because top-k precedes top-p).
"""
from __future__ import annotations

import json
import math
import os
from dataclasses import dataclass, field
from typing import List, Optional

import torch

from ..ops.backend import AttnMeta, get_backend
from ..ops.reference import pack_gate_up, rope_tables

# decode batches up to this size run the down projection on the register-streaming GEMM (fused residual)
DECODE_DOWN_SKINNY_MAX_M = 4
# decode batch <= DECODE_OPROJ_MERGE_MAX_M: the o_proj split-K GEMM merges the attention's split-K
# partitions itself (gemm_part_merge), so the attention's separate merge launch disappears
DECODE_OPROJ_MERGE_MAX_M = 2
# decode batch <= 4 under tensor parallelism: gate/up as split-K partials, silu(gate) * up formed inside
# the down GEMM's staging (gemm_part.hip SG); the TP=1 batch <= 4 path keeps the skinny down GEMM with
# its fused residual (batch 4 at TP=1: 2 merge rounds, slower)


@dataclass
class LlamaConfig:
    vocab_size: int = 128256
    hidden_size: int = 4096
    intermediate_size: int = 14336
    num_hidden_layers: int = 32
    num_attention_heads: int = 32
    num_key_value_heads: int = 8
    head_dim: int = 128
    rms_norm_eps: float = 1e-5
    rope_theta: float = 500000.0
    rope_scaling: Optional[dict] = field(default_factory=lambda: {
        "rope_type": "llama3", "factor": 8.0, "low_freq_factor": 1.0, "high_freq_factor": 4.0,
        "original_max_position_embeddings": 8192})
    max_position_embeddings: int = 131072
    tie_word_embeddings: bool = False
    bos_token_id: int = 128000
    eos_token_id: List[int] = field(default_factory=lambda: [128001, 128008, 128009])
    model_type: str = "llama"

    @classmethod
    def from_dict(cls, d):
        c = cls()
        for k in ("vocab_size", "hidden_size", "intermediate_size", "num_hidden_layers", "num_attention_heads",
                  "rms_norm_eps", "rope_theta", "max_position_embeddings", "tie_word_embeddings", "bos_token_id",
                  "model_type"):
            if k in d and d[k] is not None:
                setattr(c, k, d[k])
        c.num_key_value_heads = d.get("num_key_value_heads") or c.num_attention_heads
        c.head_dim = d.get("head_dim") or c.hidden_size // c.num_attention_heads
        c.rope_scaling = d.get("rope_scaling")
        eos = d.get("eos_token_id")
        if eos is not None:
            c.eos_token_id = eos if isinstance(eos, list) else [eos]
        return c

    @classmethod
    def from_json(cls, path):
        with open(path) as f:
            return cls.from_dict(json.load(f))

    def to_hf_dict(self):
        return {
            "architectures": ["LlamaForCausalLM"], "model_type": "llama", "vocab_size": self.vocab_size,
            "hidden_size": self.hidden_size, "intermediate_size": self.intermediate_size,
            "num_hidden_layers": self.num_hidden_layers, "num_attention_heads": self.num_attention_heads,
            "num_key_value_heads": self.num_key_value_heads, "head_dim": self.head_dim,
            "rms_norm_eps": self.rms_norm_eps, "rope_theta": self.rope_theta, "rope_scaling": self.rope_scaling,
            "max_position_embeddings": self.max_position_embeddings,
            "tie_word_embeddings": self.tie_word_embeddings, "bos_token_id": self.bos_token_id,
            "eos_token_id": self.eos_token_id, "hidden_act": "silu", "attention_bias": False, "mlp_bias": False,
            "torch_dtype": "bfloat16",
        }


def llama31_8b():
    return LlamaConfig()


def llama31_70b():
    return LlamaConfig(hidden_size=8192, intermediate_size=28672, num_hidden_layers=80, num_attention_heads=64,
                       num_key_value_heads=8)


def llama_tiny(vocab=512, layers=2, hidden=256, heads=4, kv_heads=2, inter=512):
    return LlamaConfig(vocab_size=vocab, hidden_size=hidden, intermediate_size=inter, num_hidden_layers=layers,
                       num_attention_heads=heads, num_key_value_heads=kv_heads, head_dim=hidden // heads,
                       max_position_embeddings=4096, bos_token_id=1, eos_token_id=[2])


# ------------------------------------------------------------------------------------- weights
class LlamaWeights:
    """Rank-local (TP-sharded) device tensors in kernel layouts."""

    def __init__(self, cfg: LlamaConfig, tp_rank=0, tp_size=1):
        self.cfg, self.tp_rank, self.tp_size = cfg, tp_rank, tp_size
        self.layers = []
        self.embed = self.norm = self.lm_head = None

    # ---- shard geometry
    def geom(self):
        c, tp = self.cfg, self.tp_size
        assert c.num_attention_heads % tp == 0 and c.num_key_value_heads % tp == 0, "heads % tp"
        assert c.intermediate_size % tp == 0 and (c.intermediate_size // tp) % 64 == 0, "intermediate % (64*tp)"
        return dict(Hq=c.num_attention_heads // tp, Hkv=c.num_key_value_heads // tp, D=c.head_dim,
                    I=c.intermediate_size // tp, V=-(-c.vocab_size // tp))

    @classmethod
    def from_hf(cls, cfg, get, device, tp_rank=0, tp_size=1, dtype=torch.bfloat16):
        """`get(name, rows=None, cols=None)` returns (a slice of) an HF-named tensor."""
        w = cls(cfg, tp_rank, tp_size)
        g = w.geom()
        r = tp_rank
        D, Hq, Hkv, I, Vl = g["D"], g["Hq"], g["Hkv"], g["I"], g["V"]

        def dev(t):
            return t.to(device=device, dtype=dtype, non_blocking=False).contiguous()

        w.embed = dev(get("model.embed_tokens.weight"))
        for i in range(cfg.num_hidden_layers):
            p = "model.layers.%d." % i
            q = get(p + "self_attn.q_proj.weight", rows=(r * Hq * D, (r + 1) * Hq * D))
            k = get(p + "self_attn.k_proj.weight", rows=(r * Hkv * D, (r + 1) * Hkv * D))
            v = get(p + "self_attn.v_proj.weight", rows=(r * Hkv * D, (r + 1) * Hkv * D))
            o = get(p + "self_attn.o_proj.weight", cols=(r * Hq * D, (r + 1) * Hq * D))
            gt = get(p + "mlp.gate_proj.weight", rows=(r * I, (r + 1) * I))
            up = get(p + "mlp.up_proj.weight", rows=(r * I, (r + 1) * I))
            dn = get(p + "mlp.down_proj.weight", cols=(r * I, (r + 1) * I))
            w.layers.append(dict(
                ln_in=dev(get(p + "input_layernorm.weight")), ln_post=dev(get(p + "post_attention_layernorm.weight")),
                wqkv=dev(torch.cat([q, k, v], 0)), wo=dev(o), wgu=dev(pack_gate_up(gt, up)), wdown=dev(dn)))
        w.norm = dev(get("model.norm.weight"))
        V = cfg.vocab_size
        lo, hi = r * Vl, min(V, (r + 1) * Vl)
        name = "model.embed_tokens.weight" if cfg.tie_word_embeddings else "lm_head.weight"
        lm = get(name, rows=(lo, hi))
        if lm.shape[0] < Vl:  # pad the last vocab shard
            lm = torch.cat([lm, torch.zeros(Vl - lm.shape[0], lm.shape[1], dtype=lm.dtype, device=lm.device)], 0)
        w.lm_head = dev(lm)
        w.vocab_offset = lo
        w.vocab_valid = hi - lo
        return w

    @classmethod
    def from_checkpoint(cls, path, cfg, device, tp_rank=0, tp_size=1):
        from ..runtime.safetensors_io import CheckpointReader

        rd = CheckpointReader(path)
        try:
            return cls.from_hf(cfg, rd.get, device, tp_rank, tp_size)
        finally:
            rd.close()

    @classmethod
    def from_state_dict(cls, cfg, sd, device, tp_rank=0, tp_size=1):
        def get(name, rows=None, cols=None):
            t = sd[name]
            if rows is not None:
                t = t[rows[0]:rows[1]]
            if cols is not None:
                t = t[:, cols[0]:cols[1]]
            return t

        return cls.from_hf(cfg, get, device, tp_rank, tp_size)

    @classmethod
    def random(cls, cfg, device, tp_rank=0, tp_size=1, seed=0, dtype=torch.bfloat16):
        """Random-init weights of the architecture, generated directly on `device` in the
        rank-local shard shapes (no host round trip: 16 GB for 8B in well under a second)."""
        w = cls(cfg, tp_rank, tp_size)
        g = w.geom()
        D, Hq, Hkv, I, Vl = g["D"], g["Hq"], g["Hkv"], g["I"], g["V"]
        H = cfg.hidden_size
        gen = torch.Generator(device=device).manual_seed(seed * 1000 + tp_rank)

        def rnd(*shape, std=0.02):
            return (torch.randn(*shape, device=device, generator=gen, dtype=torch.float32) * std).to(dtype)

        def ones(n):
            return (1.0 + 0.1 * torch.randn(n, device=device, generator=gen)).to(dtype)

        w.embed = rnd(cfg.vocab_size, H)
        for _ in range(cfg.num_hidden_layers):
            w.layers.append(dict(ln_in=ones(H), ln_post=ones(H), wqkv=rnd((Hq + 2 * Hkv) * D, H),
                                 wo=rnd(H, Hq * D), wgu=rnd(2 * I, H), wdown=rnd(H, I)))
        w.norm = ones(H)
        w.lm_head = rnd(Vl, H)
        w.vocab_offset = tp_rank * Vl
        w.vocab_valid = min(cfg.vocab_size - tp_rank * Vl, Vl)
        return w

    def quantize_fp8(self, lm_head=False):
        """BASELINE config 5: e4m3fn weights with per-row scales for every linear layer (qkv, o,
        packed gate/up, down; optionally lm_head). Embedding and norms stay bf16."""
        from ..ops.fp8 import quantize_weight

        for L in self.layers:
            for k in ("wqkv", "wo", "wgu", "wdown"):
                L[k] = quantize_weight(L[k])
        if lm_head:
            self.lm_head = quantize_weight(self.lm_head)
        self.dtype = "fp8"
        return self

    def nbytes(self):
        t = [self.embed, self.norm, self.lm_head] + [v for l in self.layers for v in l.values()]
        return sum(x.nbytes() if hasattr(x, "dequant") else x.numel() * x.element_size() for x in t)


# ------------------------------------------------------------------------------------- model
@dataclass
class StepInput:
    ids: torch.Tensor  # int32 [T]
    positions: torch.Tensor  # int32 [T]
    slots: torch.Tensor  # int32 [T]
    meta: AttnMeta
    logits_idx: Optional[torch.Tensor] = None  # int32 [n] rows that need logits (None = all)
    # asynchronous decode: carry[i] >= 0 -> ids[i] = carry_src[carry[i]] (previous step's sampled token,
    # resolved on the device by the embedding kernel)
    carry: Optional[torch.Tensor] = None
    carry_src: Optional[torch.Tensor] = None


class LlamaModel:
    def __init__(self, cfg: LlamaConfig, weights: LlamaWeights, device, comm=None, max_positions=None):
        self.cfg, self.w, self.device = cfg, weights, torch.device(device)
        self.be = get_backend(self.device)
        g = weights.geom()
        self.Hq, self.Hkv, self.D, self.I, self.Vl = g["Hq"], g["Hkv"], g["D"], g["I"], g["V"]
        self.comm = comm  # tensor-parallel communicator (None at TP=1)
        self.tp_rank = weights.tp_rank
        mp = max_positions or cfg.max_position_embeddings
        cos, sin = rope_tables(self.D, mp, cfg.rope_theta, cfg.rope_scaling)
        self.cos, self.sin = cos.to(self.device), sin.to(self.device)
        self.kv_cache = None  # list of (k, v) per layer: [nblocks, Hkv, 64, D]
        self.seq_parallel = os.environ.get("RAGK_SEQ_PARALLEL", "0") == "1"
        self.sp_min_tokens = int(os.environ.get("RAGK_SP_MIN_TOKENS", "256"))

    def allocate_kv_cache(self, num_blocks, dtype=torch.bfloat16):
        self.kv_cache = [(torch.zeros(num_blocks, self.Hkv, 64, self.D, dtype=dtype, device=self.device),
                          torch.zeros(num_blocks, self.Hkv, 64, self.D, dtype=dtype, device=self.device))
                         for _ in range(self.cfg.num_hidden_layers)]
        return self.kv_cache

    def kv_bytes_per_block(self, dtype=torch.bfloat16):
        return 2 * self.cfg.num_hidden_layers * self.Hkv * 64 * self.D * torch.tensor([], dtype=dtype).element_size()

    def _allreduce(self, x):
        if self.comm is not None:
            self.comm.all_reduce(x)

    # one decoder layer in two halves, so tensor-parallel prefill can interleave micro-batches
    def _attn_block(self, li, L, h, inp: StepInput, attn):
        """h <- (rank 0: h +) o_proj(attention(rmsnorm(h))): this rank's partial sum before the all-reduce."""
        be, c = self.be, self.cfg
        Hq, Hkv, D = self.Hq, self.Hkv, self.D
        kc, vc = self.kv_cache[li]
        xn = be.rmsnorm(h, L["ln_in"], c.rms_norm_eps)
        qkv = be.gemm_rope_kv(xn, L["wqkv"], inp.positions, self.cos, self.sin, inp.slots, kc, vc, Hq, Hkv, D)
        if inp.meta.kind == "decode":
            be.attn_decode(qkv, kc, vc, inp.meta, attn, Hq, Hkv, D)
        else:
            be.attn_prefill(qkv, kc, vc, inp.meta, attn, Hq, Hkv, D)
        if self.tp_rank == 0:
            be.gemm(attn, L["wo"], resid=h, epi="resid", out=h)
        else:
            be.gemm(attn, L["wo"], out=h)

    def _mlp_block(self, L, h):
        be, c = self.be, self.cfg
        xn = be.rmsnorm(h, L["ln_post"], c.rms_norm_eps)
        a = be.gemm(xn, L["wgu"], epi="silu_mul")
        if self.tp_rank == 0:
            be.gemm(a, L["wdown"], resid=h, epi="resid", out=h)
        else:
            be.gemm(a, L["wdown"], out=h)

    def _final(self, h, inp: StepInput):
        if inp.logits_idx is not None:
            h = self.be.gather_rows(h, inp.logits_idx)
        return self.be.rmsnorm(h, self.w.norm, self.cfg.rms_norm_eps)

    def _tp(self):
        return self.comm is not None and self.comm.size > 1

    def _decode_part_ok(self, inp: StepInput, h):
        if inp.meta is None or inp.meta.kind != "decode" or inp.slots is None:
            return False
        L, M = self.w.layers[0], h.shape[0]
        if self._tp() and not self.comm.fused_decode_ok(M, h.shape[1]):
            return False
        return self.be.part_ok(M, L["wqkv"]) and self.be.part_ok(M, L["wo"]) and self.be.part_ok(M, L["wdown"])

    def hidden_states_decode_part(self, inp: StepInput, h):
        """Decode step with the split-K partial GEMM (csrc/kernels/gemm_part.hip) for the three
        small-N projections: qkv / o_proj / down write fp32 partial slabs and the following row
        kernel reduces them -- rope_kv_partials (qkv) and add_partials_rmsnorm (o_proj -> post-attention
        norm, down -> next layer's input norm / the final norm), so the reduction adds no launch and
        the GEMMs stream their weights with every load in flight (qkv 26.7 -> 15 us, o_proj 15 -> 11.6,
        down 43 -> 30 at batch 32; tools/bench_decode_gemm.py). Same math and bf16 rounding points as
        hidden_states (bf16 linear outputs, bf16 residual adds).

        Tensor parallel: the same path on this rank's shard (its heads, its slices of the FFN). The
        row-parallel o_proj / down reductions happen INSIDE their consumer: comm.add_partials_rmsnorm
        sums every rank's fp32 slabs over the xGMI peer mappings, adds the residual and normalises in
        one kernel (csrc/comm/allreduce.hip ar_add_rmsnorm) -- no standalone all-reduce launch, and
        the row-parallel sum is rounded to bf16 once, as at TP=1. Per layer: qkv GEMM, attention (+RoPE
        + KV append), o_proj (+ partition merge at batch <= 2), reduce+norm, gate/up, down,
        reduce+norm. (The batch <= 4 TP=1 fusions that put the input norm into the qkv GEMM and the
        residual into the down GEMM need the full-rank sum first, so they stay TP=1-only.)"""
        be, w, c = self.be, self.w, self.cfg
        Hq, Hkv, D = self.Hq, self.Hkv, self.D
        M = h.shape[0]
        tp = self._tp()

        def reduce_norm(P, gamma):
            if tp:
                return self.comm.add_partials_rmsnorm(P, h, gamma, c.rms_norm_eps, be)
            return be.add_partials_rmsnorm(P, h, gamma, c.rms_norm_eps)

        attn = torch.empty((M, Hq * D), dtype=h.dtype, device=h.device)
        layers = w.layers
        # batch <= 4: the input norm runs inside the qkv GEMM (gemm_part_norm) -- one launch fewer per layer
        fuse_norm = M <= DECODE_DOWN_SKINNY_MAX_M and not tp and be.part_norm_ok(M, layers[0]["wqkv"])
        # batch <= 4 (TP): silu(gate) * up inside the down GEMM; the down partials then go through the
        # reduce + norm consumer, so the next layer's input norm is not fused into its qkv GEMM
        silu_fused = tp and be.part_silu_ok(M, layers[0]["wgu"], layers[0]["wdown"])
        xn = None if fuse_norm else be.rmsnorm(h, layers[0]["ln_in"], c.rms_norm_eps)
        merge = M <= DECODE_OPROJ_MERGE_MAX_M and be.part_merge_ok(M, inp.meta, layers[0]["wo"], Hq, D)
        # batch 1: gate/up + SiLU + down + residual as ONE persistent launch (csrc/kernels/mlp_engine.hip)
        mlp_eng = M == 1 and not tp and be.mlp_engine_ok(M, layers[0]["wgu"], layers[0]["wdown"])
        for li, L in enumerate(layers):
            kc, vc = self.kv_cache[li]
            P = be.gemm_part_norm(h, L["ln_in"], c.rms_norm_eps, L["wqkv"]) if fuse_norm else be.gemm_part(xn, L["wqkv"])
            # RoPE + KV append inside the attention kernel; at batch <= 2 its split-K merge inside the o_proj GEMM
            be.attn_decode_rope(P, inp.positions, self.cos, self.sin, inp.slots, kc, vc, inp.meta, attn, Hq, Hkv, D,
                                defer_merge=merge)
            P = be.gemm_part_merge(attn, inp.meta, L["wo"], Hq) if merge else be.gemm_part(attn, L["wo"])
            nxt = layers[li + 1]["ln_in"] if li + 1 < len(layers) else w.norm
            if mlp_eng:
                # o_proj slabs + residual + post-attention norm + gate/up + SiLU + down + residual: one launch
                be.mlp_engine_tail(P, h, L["ln_post"], c.rms_norm_eps, L["wgu"], L["wdown"])
                if not fuse_norm or li + 1 == len(layers):
                    xn = be.rmsnorm(h, nxt, c.rms_norm_eps)
                continue
            xn = reduce_norm(P, L["ln_post"])
            if silu_fused:
                P = be.gemm_part_silu(be.gemm_part_gu(xn, L["wgu"]), L["wdown"])
                xn = reduce_norm(P, nxt)
                continue
            a = be.gemm(xn, L["wgu"], epi="silu_mul")
            if M <= DECODE_DOWN_SKINNY_MAX_M and not tp:
                # tiny batch: the register-streaming GEMM with the fused residual + a plain norm beats
                # the split-K partials + consumer by ~2 us (profiles/decode_gemm_graph_ab_M_r2.log)
                be.gemm(a, L["wdown"], resid=h, epi="resid", out=h)
                if not fuse_norm or li + 1 == len(layers):
                    xn = be.rmsnorm(h, nxt, c.rms_norm_eps)
                continue
            P = be.gemm_part(a, L["wdown"])
            xn = reduce_norm(P, nxt)
        if inp.logits_idx is not None:
            xn = be.gather_rows(xn, inp.logits_idx)
        return xn

    def hidden_states(self, inp: StepInput):
        """Run the decoder stack; returns the final-norm'ed rows selected by logits_idx."""
        be, w = self.be, self.w
        h = be.embed(inp.ids, w.embed, carry=inp.carry, prev=inp.carry_src)
        if self._decode_part_ok(inp, h):
            return self.hidden_states_decode_part(inp, h)
        attn = torch.empty((h.shape[0], self.Hq * self.D), dtype=h.dtype, device=h.device)
        if self.comm is None and inp.meta is not None and inp.meta.kind != "decode":
            L0 = w.layers[0]
            ns = (be.prefill_nsplit(h.shape[0], L0["wo"]), be.prefill_nsplit(h.shape[0], L0["wdown"]))
            if max(ns) > 1:
                return self.hidden_states_splitk(inp, h, attn, *ns)
        for li, L in enumerate(w.layers):
            self._attn_block(li, L, h, inp, attn)
            self._allreduce(h)
            self._mlp_block(L, h)
            self._allreduce(h)
        return self._final(h, inp)

    def hidden_states_splitk(self, inp: StepInput, h, attn, ns_o, ns_d):
        """TP=1 prefill of a step too small to fill the CUs with 256x256 output tiles (a single ~5k-token
        RAG prompt): o_proj / down run as split-K GEMMs into fp32 slabs (ops/native.py:prefill_nsplit,
        gemm_w4c KSPLIT) and the residual add moves into the following RMSNorm kernel
        (add_partials_rmsnorm), which the layer needs anyway -- same rounding points as the residual
        epilogue path (bf16 projection output, bf16 residual add)."""
        be, w, c = self.be, self.w, self.cfg
        Hq, Hkv, D = self.Hq, self.Hkv, self.D
        layers = w.layers
        xn = be.rmsnorm(h, layers[0]["ln_in"], c.rms_norm_eps)
        for li, L in enumerate(layers):
            kc, vc = self.kv_cache[li]
            qkv = be.gemm_rope_kv(xn, L["wqkv"], inp.positions, self.cos, self.sin, inp.slots, kc, vc, Hq, Hkv, D)
            be.attn_prefill(qkv, kc, vc, inp.meta, attn, Hq, Hkv, D)
            if ns_o > 1:
                xn = be.add_partials_rmsnorm(be.gemm_splitk(attn, L["wo"], ns_o), h, L["ln_post"], c.rms_norm_eps)
            else:
                be.gemm(attn, L["wo"], resid=h, epi="resid", out=h)
                xn = be.rmsnorm(h, L["ln_post"], c.rms_norm_eps)
            a = be.gemm(xn, L["wgu"], epi="silu_mul")
            nxt = layers[li + 1]["ln_in"] if li + 1 < len(layers) else w.norm
            if ns_d > 1:
                xn = be.add_partials_rmsnorm(be.gemm_splitk(a, L["wdown"], ns_d), h, nxt, c.rms_norm_eps)
            else:
                be.gemm(a, L["wdown"], resid=h, epi="resid", out=h)
                xn = be.rmsnorm(h, nxt, c.rms_norm_eps)
        if inp.logits_idx is not None:
            xn = be.gather_rows(xn, inp.logits_idx)
        return xn

    def hidden_states_sp(self, inp: StepInput):
        """Tensor-parallel prefill with Megatron sequence parallelism: the residual
        stream stays sharded over tokens -- rank r owns rows [r*S, (r+1)*S) of the (padded) batch --
        so embedding, both RMSNorms and both residual adds run on T/tp rows per rank, and each
        row-parallel projection's all-reduce becomes a reduce-scatter into the owner's rows, paired
        with an all-gather of the normed rows in front of the next column-parallel GEMM:
            h_r -> rmsnorm -> AG -> qkv/rope/attention -> o_proj (partial) -> RS -> h_r +=
                -> rmsnorm -> AG -> gate/up/SiLU -> down (partial) -> RS -> h_r +=
        Same bytes on xGMI as the two all-reduces (RS + AG), a tp-th of the norm/residual traffic, and
        a [T/tp, H] residual per rank. Attention, the paged KV cache and the GEMMs see all T tokens of
        this rank's heads, exactly as in hidden_states. Returns the final-norm'ed logits rows."""
        be, w, c, comm = self.be, self.w, self.cfg, self.comm
        tp, r = comm.size, comm.rank
        Hq, Hkv, D, H = self.Hq, self.Hkv, self.D, c.hidden_size
        T = inp.ids.shape[0]
        S = -(-T // tp)
        Tp = S * tp
        ids = inp.ids
        if Tp != T:
            ids = torch.cat([ids, ids.new_zeros(Tp - T)])
        h = be.embed(ids[r * S:(r + 1) * S].contiguous(), w.embed)  # [S, H] this rank's rows
        dev, dt = h.device, h.dtype
        xg = torch.empty((Tp, H), dtype=dt, device=dev)  # gathered normed rows
        part = torch.zeros((Tp, H), dtype=dt, device=dev)  # row-parallel partial sums (pad rows stay 0)
        attn = torch.empty((T, Hq * D), dtype=dt, device=dev)
        rs = torch.empty((S, H), dtype=dt, device=dev)
        for li, L in enumerate(w.layers):
            kc, vc = self.kv_cache[li]
            comm.all_gather_into(xg, be.rmsnorm(h, L["ln_in"], c.rms_norm_eps))
            qkv = be.gemm_rope_kv(xg[:T], L["wqkv"], inp.positions, self.cos, self.sin, inp.slots, kc, vc, Hq, Hkv, D)
            be.attn_prefill(qkv, kc, vc, inp.meta, attn, Hq, Hkv, D)
            be.gemm(attn, L["wo"], out=part[:T])
            h += comm.reduce_scatter(part, rs)
            comm.all_gather_into(xg, be.rmsnorm(h, L["ln_post"], c.rms_norm_eps))
            a = be.gemm(xg[:T], L["wgu"], epi="silu_mul")
            be.gemm(a, L["wdown"], out=part[:T])
            h += comm.reduce_scatter(part, rs)
        comm.all_gather_into(xg, be.rmsnorm(h, w.norm, c.rms_norm_eps))
        x = xg[:T]
        return be.gather_rows(x, inp.logits_idx) if inp.logits_idx is not None else x

    def hidden_states_microbatched(self, inps):
        """Tensor-parallel prefill with communication/compute overlap: the token
        batch is split into micro-batches (consecutive pieces of the packed prompt chunks; a later
        micro-batch's queries read the earlier one's K/V from the paged cache, which this layer has
        already written). Every all-reduce is issued asynchronously (RCCL stream / the peer-mapped
        kernel on a side stream) and waited on only when its micro-batch needs the result, so the
        all-reduce of micro-batch m overlaps the GEMMs and attention of micro-batch m+1:
            attn(A) | AR(A) ~ attn(B) | AR(B) ~ mlp(A) | AR(A) ~ mlp(B) | AR(B) ~ attn(A, next layer)
        Returns one hidden-state tensor per micro-batch."""
        be, w = self.be, self.w
        hs = [be.embed(i.ids, w.embed) for i in inps]
        attn = [torch.empty((h.shape[0], self.Hq * self.D), dtype=h.dtype, device=h.device) for h in hs]
        pend = [None] * len(hs)
        for li, L in enumerate(w.layers):
            for m, inp in enumerate(inps):
                if pend[m] is not None:
                    pend[m].wait()
                self._attn_block(li, L, hs[m], inp, attn[m])
                pend[m] = self.comm.all_reduce_async(hs[m])
            for m in range(len(inps)):
                pend[m].wait()
                self._mlp_block(L, hs[m])
                pend[m] = self.comm.all_reduce_async(hs[m])
        for p in pend:
            p.wait()
        return [self._final(h, inp) for h, inp in zip(hs, inps)]

    def logits(self, hs):
        """Rank-local vocab-shard logits (fp32)."""
        return self.be.gemm(hs, self.w.lm_head, out_f32=True)

    def forward(self, inp: StepInput):
        if self.use_sp(inp):
            return self.logits(self.hidden_states_sp(inp))
        return self.logits(self.hidden_states(inp))

    def use_sp(self, inp: StepInput):
        """Sequence-parallel prefill: TP > 1, RAGK_SEQ_PARALLEL=1 (default off: same xGMI bytes as the
        all-reduce path, which overlaps micro-batches), at least sp_min_tokens tokens."""
        return (self.seq_parallel and self.comm is not None and self.comm.size > 1 and inp.meta is not None
                and inp.meta.kind == "prefill" and inp.ids.shape[0] >= self.sp_min_tokens)
