"""Sentence-embedding encoders: BERT family (all-MiniLM-L6-v2, bge-large-en) and XLM-RoBERTa
(BAAI/bge-m3, the reference embedder).

Reference: SentenceTransformer('BAAI/bge-m3').encode([text], normalize_embeddings=True)
(/root/reference/llm/rag.py:33,55) = XLMRobertaModel -> Pooling(CLS) -> Normalize.
Post-LN transformer ([dep] modeling_xlm_roberta.py:329-400), exact-erf GELU.

MI355X-first: sequences are PACKED (varlen, no padding FLOPs), qkv is one GEMM with a bias
epilogue, attention-output and FFN-output GEMMs fuse bias + residual, FFN-up fuses bias +
GELU, LayerNorm is one pass, and CLS/mean pooling + L2 normalise is one kernel.
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass

import torch

from ..ops.backend import get_backend


@dataclass
class EncoderConfig:
    model_type: str = "bert"  # bert | xlm-roberta
    vocab_size: int = 30522
    hidden_size: int = 384
    num_hidden_layers: int = 6
    num_attention_heads: int = 12
    intermediate_size: int = 1536
    max_position_embeddings: int = 512
    type_vocab_size: int = 2
    layer_norm_eps: float = 1e-12
    pad_token_id: int = 0
    pooling: str = "mean"  # cls | mean
    normalize: bool = True
    max_seq_length: int = 256

    @property
    def head_dim(self):
        return self.hidden_size // self.num_attention_heads

    @classmethod
    def from_dict(cls, d, pooling=None, max_seq_length=None):
        c = cls()
        for k in ("model_type", "vocab_size", "hidden_size", "num_hidden_layers", "num_attention_heads",
                  "intermediate_size", "max_position_embeddings", "type_vocab_size", "layer_norm_eps",
                  "pad_token_id"):
            if k in d and d[k] is not None:
                setattr(c, k, d[k])
        if pooling:
            c.pooling = pooling
        if max_seq_length:
            c.max_seq_length = max_seq_length
        return c

    @classmethod
    def from_dir(cls, path):
        with open(os.path.join(path, "config.json")) as f:
            d = json.load(f)
        pooling, msl = None, None
        pcfg = os.path.join(path, "1_Pooling", "config.json")
        if os.path.exists(pcfg):
            with open(pcfg) as f:
                p = json.load(f)
            pooling = "cls" if p.get("pooling_mode_cls_token") else ("mean" if p.get("pooling_mode_mean_tokens")
                                                                    else None)
        sbc = os.path.join(path, "sentence_bert_config.json")
        if os.path.exists(sbc):
            with open(sbc) as f:
                msl = json.load(f).get("max_seq_length")
        if pooling is None:
            pooling = "cls" if d.get("model_type") == "xlm-roberta" else "mean"
        return cls.from_dict(d, pooling=pooling, max_seq_length=msl or min(512, d.get("max_position_embeddings", 512)))

    def to_hf_dict(self):
        d = dict(model_type=self.model_type, vocab_size=self.vocab_size, hidden_size=self.hidden_size,
                 num_hidden_layers=self.num_hidden_layers, num_attention_heads=self.num_attention_heads,
                 intermediate_size=self.intermediate_size, max_position_embeddings=self.max_position_embeddings,
                 type_vocab_size=self.type_vocab_size, layer_norm_eps=self.layer_norm_eps,
                 pad_token_id=self.pad_token_id, hidden_act="gelu", torch_dtype="bfloat16")
        d["architectures"] = ["XLMRobertaModel" if self.model_type == "xlm-roberta" else "BertModel"]
        return d


def minilm_l6():
    return EncoderConfig()


def bge_large_en():
    return EncoderConfig(hidden_size=1024, num_hidden_layers=24, num_attention_heads=16, intermediate_size=4096,
                         pooling="cls", max_seq_length=512)


def bge_m3():
    return EncoderConfig(model_type="xlm-roberta", vocab_size=250002, hidden_size=1024, num_hidden_layers=24,
                         num_attention_heads=16, intermediate_size=4096, max_position_embeddings=8194,
                         type_vocab_size=1, layer_norm_eps=1e-5, pad_token_id=1, pooling="cls", max_seq_length=8192)


class EncoderWeights:
    @classmethod
    def from_hf(cls, cfg: EncoderConfig, get, has, device, dtype=torch.bfloat16):
        w = cls()
        prefix = ""
        for p in ("", "bert.", "roberta.", "model.", "0.auto_model."):
            if has(p + "embeddings.word_embeddings.weight"):
                prefix = p
                break

        def g(n):
            return get(prefix + n).to(device=device, dtype=dtype).contiguous()

        w.word = g("embeddings.word_embeddings.weight")
        w.pos = g("embeddings.position_embeddings.weight")
        w.type_row = g("embeddings.token_type_embeddings.weight")[0].contiguous()
        w.ln_g, w.ln_b = g("embeddings.LayerNorm.weight"), g("embeddings.LayerNorm.bias")
        w.layers = []
        for i in range(cfg.num_hidden_layers):
            p = "encoder.layer.%d." % i
            wq, wk, wv = (g(p + "attention.self.%s.weight" % n) for n in ("query", "key", "value"))
            bq, bk, bv = (g(p + "attention.self.%s.bias" % n) for n in ("query", "key", "value"))
            w.layers.append(dict(
                wqkv=torch.cat([wq, wk, wv], 0).contiguous(), bqkv=torch.cat([bq, bk, bv], 0).contiguous(),
                wo=g(p + "attention.output.dense.weight"), bo=g(p + "attention.output.dense.bias"),
                ln1_g=g(p + "attention.output.LayerNorm.weight"), ln1_b=g(p + "attention.output.LayerNorm.bias"),
                wi=g(p + "intermediate.dense.weight"), bi=g(p + "intermediate.dense.bias"),
                wo2=g(p + "output.dense.weight"), bo2=g(p + "output.dense.bias"),
                ln2_g=g(p + "output.LayerNorm.weight"), ln2_b=g(p + "output.LayerNorm.bias")))
        return w

    @classmethod
    def from_dir(cls, cfg, path, device):
        from ..runtime.safetensors_io import CheckpointReader

        rd = CheckpointReader(path)
        try:
            return cls.from_hf(cfg, lambda n: rd.get(n), rd.has, device)
        finally:
            rd.close()

    @classmethod
    def from_state_dict(cls, cfg, sd, device):
        return cls.from_hf(cfg, lambda n: sd[n], lambda n: n in sd, device)

    @classmethod
    def random(cls, cfg: EncoderConfig, device, seed=0, dtype=torch.bfloat16):
        gen = torch.Generator(device=device).manual_seed(seed)
        H, I = cfg.hidden_size, cfg.intermediate_size

        def r(*s, std=0.02):
            return (torch.randn(*s, device=device, generator=gen) * std).to(dtype)

        def one(n):
            return (1 + 0.05 * torch.randn(n, device=device, generator=gen)).to(dtype)

        w = cls()
        w.word, w.pos, w.type_row = r(cfg.vocab_size, H), r(cfg.max_position_embeddings, H), r(H)
        w.ln_g, w.ln_b = one(H), r(H)
        w.layers = [dict(wqkv=r(3 * H, H), bqkv=r(3 * H), wo=r(H, H), bo=r(H), ln1_g=one(H), ln1_b=r(H),
                         wi=r(I, H), bi=r(I), wo2=r(H, I), bo2=r(H), ln2_g=one(H), ln2_b=r(H))
                    for _ in range(cfg.num_hidden_layers)]
        return w


class EncoderModel:
    def __init__(self, cfg: EncoderConfig, weights: EncoderWeights, device):
        self.cfg, self.w, self.device = cfg, weights, torch.device(device)
        self.be = get_backend(self.device)

    def position_ids(self, lens):
        """BERT: 0..L-1.  XLM-R: cumsum(mask) + padding_idx -> starts at padding_idx + 1."""
        off = self.cfg.pad_token_id + 1 if self.cfg.model_type == "xlm-roberta" else 0
        return torch.cat([torch.arange(off, off + L, dtype=torch.int32) for L in lens])

    def forward_packed(self, ids: torch.Tensor, lens):
        """ids: int32 [T] packed token ids (on device), lens: python list of sequence lengths.
        Returns fp32 [B, H] pooled (+ normalised) sentence embeddings."""
        from ..ops.native import build_prefill_tiles

        be, w, c = self.be, self.w, self.cfg
        H, nh, D = c.hidden_size, c.num_attention_heads, c.head_dim
        dev = self.device
        cu_host = [0]
        for L in lens:
            cu_host.append(cu_host[-1] + L)
        cu = torch.tensor(cu_host, dtype=torch.int32).to(dev)
        pos = self.position_ids(lens).to(dev)
        tiles = build_prefill_tiles(lens, nh, nh).to(dev) if dev.type == "cuda" else None
        h = be.embed_ln(ids, pos, w.word, w.pos, w.type_row, w.ln_g, w.ln_b, c.layer_norm_eps)
        T = h.shape[0]
        attn = torch.empty((T, H), dtype=h.dtype, device=dev)
        for L in w.layers:
            qkv = be.gemm(h, L["wqkv"], bias=L["bqkv"], epi="bias")
            be.attn_encoder(qkv, cu, lens, tiles, attn, nh, D)
            a = be.gemm(attn, L["wo"], bias=L["bo"], resid=h, epi="bias_resid")
            h = be.layernorm(a, L["ln1_g"], L["ln1_b"], c.layer_norm_eps)
            f = be.gemm(h, L["wi"], bias=L["bi"], epi="bias_gelu")
            a = be.gemm(f, L["wo2"], bias=L["bo2"], resid=h, epi="bias_resid")
            h = be.layernorm(a, L["ln2_g"], L["ln2_b"], c.layer_norm_eps)
        return be.pool_l2norm(h, cu, mode=c.pooling, normalize=c.normalize)
