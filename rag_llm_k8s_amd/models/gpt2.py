"""GPT-2 decoder (BASELINE config 1: "all-MiniLM-L6-v2 embed + gpt2 generate ... on CPU").

Not used by the reference itself (it only runs Llama-3.1-8B, /root/reference/llm/download_model.py:5);
it is the CPU plumbing generator. Same engine interface as LlamaModel (paged KV cache,
StepInput), so it also runs on the GPU through the native kernels: learned positions
(embed without LayerNorm), pre-LN blocks, fused qkv + bias, bias+residual epilogues,
tanh-GELU MLP epilogue, tied lm_head (padded to a multiple of 8 rows).
HF weights use Conv1D ([in, out]) -> transposed once at load.
"""
from __future__ import annotations

import json
from dataclasses import dataclass

import torch

from ..ops.backend import get_backend


@dataclass
class GPT2Config:
    vocab_size: int = 50257
    n_positions: int = 1024
    n_embd: int = 768
    n_layer: int = 12
    n_head: int = 12
    layer_norm_epsilon: float = 1e-5
    bos_token_id: int = 50256
    eos_token_id: int = 50256
    model_type: str = "gpt2"

    @classmethod
    def from_dict(cls, d):
        c = cls()
        for k in ("vocab_size", "n_positions", "n_embd", "n_layer", "n_head", "layer_norm_epsilon", "bos_token_id",
                  "eos_token_id"):
            if d.get(k) is not None:
                setattr(c, k, d[k])
        return c

    def to_hf_dict(self):
        return {"architectures": ["GPT2LMHeadModel"], "model_type": "gpt2", "vocab_size": self.vocab_size,
                "n_positions": self.n_positions, "n_ctx": self.n_positions, "n_embd": self.n_embd,
                "n_layer": self.n_layer, "n_head": self.n_head, "layer_norm_epsilon": self.layer_norm_epsilon,
                "bos_token_id": self.bos_token_id, "eos_token_id": self.eos_token_id,
                "activation_function": "gelu_new"}

    @property
    def head_dim(self):
        return self.n_embd // self.n_head


class GPT2Weights:
    @classmethod
    def from_hf(cls, cfg, get, has, device, dtype=torch.bfloat16):
        w = cls()
        pre = "transformer." if has("transformer.wte.weight") else ""

        def g(n, t=False):
            x = get(pre + n)
            if t:
                x = x.t()
            return x.to(device=device, dtype=dtype).contiguous()

        w.wte = g("wte.weight")
        w.wpe = g("wpe.weight")
        w.layers = []
        for i in range(cfg.n_layer):
            p = "h.%d." % i
            w.layers.append(dict(
                ln1_g=g(p + "ln_1.weight"), ln1_b=g(p + "ln_1.bias"),
                wqkv=g(p + "attn.c_attn.weight", True), bqkv=g(p + "attn.c_attn.bias"),
                wo=g(p + "attn.c_proj.weight", True), bo=g(p + "attn.c_proj.bias"),
                ln2_g=g(p + "ln_2.weight"), ln2_b=g(p + "ln_2.bias"),
                wfc=g(p + "mlp.c_fc.weight", True), bfc=g(p + "mlp.c_fc.bias"),
                wpr=g(p + "mlp.c_proj.weight", True), bpr=g(p + "mlp.c_proj.bias")))
        w.lnf_g, w.lnf_b = g("ln_f.weight"), g("ln_f.bias")
        V = w.wte.shape[0]
        pad = (-V) % 8
        w.lm_head = torch.cat([w.wte, torch.zeros(pad, w.wte.shape[1], dtype=dtype, device=device)], 0) if pad \
            else w.wte
        w.vocab_offset, w.vocab_valid = 0, V
        w.tp_rank = 0
        return w

    @classmethod
    def from_checkpoint(cls, path, cfg, device):
        from ..runtime.safetensors_io import CheckpointReader

        rd = CheckpointReader(path)
        try:
            return cls.from_hf(cfg, rd.get, rd.has, device)
        finally:
            rd.close()

    @classmethod
    def from_state_dict(cls, cfg, sd, device):
        return cls.from_hf(cfg, lambda n: sd[n], lambda n: n in sd, device)


class GPT2Model:
    def __init__(self, cfg: GPT2Config, weights: GPT2Weights, device, comm=None, max_positions=None):
        self.cfg, self.w, self.device = cfg, weights, torch.device(device)
        self.be = get_backend(self.device)
        self.Hq = self.Hkv = cfg.n_head
        self.D = cfg.head_dim
        self.tp_rank = 0
        self.kv_cache = None

    def allocate_kv_cache(self, num_blocks, dtype=torch.bfloat16):
        self.kv_cache = [(torch.zeros(num_blocks, self.Hkv, 64, self.D, dtype=dtype, device=self.device),
                          torch.zeros(num_blocks, self.Hkv, 64, self.D, dtype=dtype, device=self.device))
                         for _ in range(self.cfg.n_layer)]
        return self.kv_cache

    def kv_bytes_per_block(self):
        return 2 * self.cfg.n_layer * self.Hkv * 64 * self.D * 2

    def hidden_states(self, inp):
        be, w, c = self.be, self.w, self.cfg
        H, D, nh = c.n_embd, self.D, c.n_head
        h = be.embed_ln(inp.ids, inp.positions, w.wte, w.wpe, None, None, None, 0.0, do_ln=False)
        T = h.shape[0]
        attn = torch.empty((T, H), dtype=h.dtype, device=h.device)
        for li, L in enumerate(w.layers):
            kc, vc = self.kv_cache[li]
            x = be.layernorm(h, L["ln1_g"], L["ln1_b"], c.layer_norm_epsilon)
            qkv = be.gemm(x, L["wqkv"], bias=L["bqkv"], epi="bias")
            be.rope_kv(qkv, inp.positions, None, None, inp.slots, kc, vc, nh, nh, D, apply_rope=False)
            if inp.meta.kind == "decode":
                be.attn_decode(qkv, kc, vc, inp.meta, attn, nh, nh, D)
            else:
                be.attn_prefill(qkv, kc, vc, inp.meta, attn, nh, nh, D)
            h = be.gemm(attn, L["wo"], bias=L["bo"], resid=h, epi="bias_resid")
            x = be.layernorm(h, L["ln2_g"], L["ln2_b"], c.layer_norm_epsilon)
            f = be.gemm(x, L["wfc"], bias=L["bfc"], epi="bias_gelu_tanh")
            h = be.gemm(f, L["wpr"], bias=L["bpr"], resid=h, epi="bias_resid")
        if inp.logits_idx is not None:
            h = be.gather_rows(h, inp.logits_idx)
        return be.layernorm(h, w.lnf_g, w.lnf_b, c.layer_norm_epsilon)

    def logits(self, hs):
        return self.be.gemm(hs, self.w.lm_head, out_f32=True)

    def forward(self, inp):
        return self.logits(self.hidden_states(inp))


def gpt2_tiny(vocab=512):
    return GPT2Config(vocab_size=vocab, n_positions=1024, n_embd=128, n_layer=2, n_head=2, bos_token_id=vocab - 2,
                      eos_token_id=vocab - 1)


def gpt2_state_dict(cfg: GPT2Config, seed=0, std=0.02):
    g = torch.Generator().manual_seed(seed)
    H = cfg.n_embd

    def r(*s):
        return (torch.randn(*s, generator=g) * std).bfloat16()

    def one(n):
        return (1 + 0.05 * torch.randn(n, generator=g)).bfloat16()

    sd = {"transformer.wte.weight": r(cfg.vocab_size, H), "transformer.wpe.weight": r(cfg.n_positions, H),
          "transformer.ln_f.weight": one(H), "transformer.ln_f.bias": r(H)}
    for i in range(cfg.n_layer):
        p = "transformer.h.%d." % i
        sd.update({p + "ln_1.weight": one(H), p + "ln_1.bias": r(H), p + "attn.c_attn.weight": r(H, 3 * H),
                   p + "attn.c_attn.bias": r(3 * H), p + "attn.c_proj.weight": r(H, H), p + "attn.c_proj.bias": r(H),
                   p + "ln_2.weight": one(H), p + "ln_2.bias": r(H), p + "mlp.c_fc.weight": r(H, 4 * H),
                   p + "mlp.c_fc.bias": r(4 * H), p + "mlp.c_proj.weight": r(4 * H, H), p + "mlp.c_proj.bias": r(H)})
    return sd


def write_gpt2_checkpoint(out_dir, cfg, seed=0):
    import os

    from ..runtime.safetensors_io import save_file
    from ..utils.synthetic import train_small_bpe

    os.makedirs(out_dir, exist_ok=True)
    with open(os.path.join(out_dir, "config.json"), "w") as f:
        json.dump(cfg.to_hf_dict(), f, indent=2)
    with open(os.path.join(out_dir, "generation_config.json"), "w") as f:
        json.dump({"bos_token_id": cfg.bos_token_id, "eos_token_id": cfg.eos_token_id, "do_sample": True}, f)
    save_file(gpt2_state_dict(cfg, seed), os.path.join(out_dir, "model.safetensors"), metadata={"format": "pt"})
    if not os.path.exists(os.path.join(out_dir, "tokenizer.json")):
        train_small_bpe(out_dir, cfg.vocab_size)
