"""Offline synthetic assets (no network on the build/GPU boxes).

* a Zipf-distributed pseudo-English word corpus;
* tokenizers trained on it with HF `tokenizers`: Llama-3-style byte-level BPE (128,000
  regular + 256 special tokens, <|begin_of_text|> auto-prepended), GPT-2-style BPE, and
  BERT WordPiece (for MiniLM / bge-large shaped encoders);
* random-init checkpoints written in the reference's /models layout
  (/root/reference/llm/download_model.py:14-25): config.json, generation_config.json,
  model-0000i-of-0000N.safetensors + index, tokenizer.json, tokenizer_config.json,
  special_tokens_map.json; and sentence-transformers layout for encoders;
* synthetic PDFs through ingest/pdf.write_pdf.
"""
from __future__ import annotations

import json
import os

import numpy as np
import torch

_CONS = list("bcdfghjklmnprstvwz") + ["ch", "sh", "th", "tr", "st", "pl", "gr", "br", "qu"]
_VOW = list("aeiou") + ["ai", "ea", "ou", "io", "ee"]


class WordModel:
    """Zipfian generator over a fixed pseudo-word vocabulary (deterministic per seed)."""

    def __init__(self, n_words=400000, seed=0, zipf_a=1.0):
        r = np.random.default_rng(seed)
        words = []
        seen = set()
        while len(words) < n_words:
            n = int(r.integers(1, 5))
            w = "".join(_CONS[r.integers(len(_CONS))] + _VOW[r.integers(len(_VOW))] for _ in range(n))
            if r.random() < 0.5:
                w += _CONS[r.integers(len(_CONS))]
            if w not in seen:
                seen.add(w)
                words.append(w)
        self.words = np.array(words, dtype=object)
        p = 1.0 / np.arange(1, n_words + 1) ** zipf_a
        self.p = p / p.sum()
        self.cdf = np.cumsum(self.p)
        self.rng = np.random.default_rng(seed + 1)

    def sample(self, n, rng=None):
        rng = rng or self.rng
        idx = np.searchsorted(self.cdf, rng.random(n), side="right")
        idx = np.minimum(idx, len(self.words) - 1)
        return self.words[idx]

    def text(self, n_words, rng=None, sentence=14):
        w = list(self.sample(n_words, rng))
        out = []
        for i, x in enumerate(w):
            if i % sentence == 0:
                x = x.capitalize()
            if i % sentence == sentence - 1:
                x += "."
            out.append(x)
        return " ".join(out)

    def corpus_lines(self, n_words, line_words=200):
        w = list(self.sample(n_words))
        return [" ".join(w[i:i + line_words]) + "." for i in range(0, len(w), line_words)]


LLAMA3_SPECIAL = {128000: "<|begin_of_text|>", 128001: "<|end_of_text|>", 128006: "<|start_header_id|>",
                  128007: "<|end_header_id|>", 128008: "<|eom_id|>", 128009: "<|eot_id|>", 128010: "<|python_tag|>"}


def train_llama3_tokenizer(out_dir, wm: WordModel = None, corpus_words=3_000_000, base_vocab=128000, n_special=256):
    """Byte-level BPE with exactly base_vocab regular tokens + n_special specials (ids base_vocab..)."""
    from tokenizers import AddedToken, Tokenizer, decoders, models, pre_tokenizers, processors, trainers

    wm = wm or WordModel()
    tok = Tokenizer(models.BPE())
    tok.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False, use_regex=True)
    tok.decoder = decoders.ByteLevel()
    tr = trainers.BpeTrainer(vocab_size=base_vocab, min_frequency=2, show_progress=False,
                             initial_alphabet=pre_tokenizers.ByteLevel.alphabet())
    tok.train_from_iterator(wm.corpus_lines(corpus_words), trainer=tr)
    n = tok.get_vocab_size()
    if n < base_vocab:  # pad so the specials land on their Llama-3 ids
        tok.add_tokens(["<|filler_%d|>" % i for i in range(base_vocab - n)])
    specials = []
    for i in range(n_special):
        tid = base_vocab + i
        name = LLAMA3_SPECIAL.get(tid, "<|reserved_special_token_%d|>" % i)
        specials.append(AddedToken(name, special=True, normalized=False))
    tok.add_special_tokens(specials)
    bos = "<|begin_of_text|>"
    tok.post_processor = processors.TemplateProcessing(single=bos + " $A", pair=bos + " $A " + bos + " $B",
                                                       special_tokens=[(bos, tok.token_to_id(bos))])
    os.makedirs(out_dir, exist_ok=True)
    tok.save(os.path.join(out_dir, "tokenizer.json"))
    with open(os.path.join(out_dir, "tokenizer_config.json"), "w") as f:
        json.dump({"bos_token": bos, "eos_token": "<|eot_id|>", "model_max_length": 131072,
                   "tokenizer_class": "PreTrainedTokenizerFast", "clean_up_tokenization_spaces": True}, f, indent=2)
    with open(os.path.join(out_dir, "special_tokens_map.json"), "w") as f:
        json.dump({"bos_token": bos, "eos_token": "<|eot_id|>"}, f, indent=2)
    return tok


def train_gpt2_tokenizer(out_dir, wm: WordModel = None, corpus_words=1_000_000, vocab=50257):
    from tokenizers import AddedToken, Tokenizer, decoders, models, pre_tokenizers, trainers

    wm = wm or WordModel(seed=5)
    tok = Tokenizer(models.BPE())
    tok.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False)
    tok.decoder = decoders.ByteLevel()
    tr = trainers.BpeTrainer(vocab_size=vocab - 1, min_frequency=2, show_progress=False,
                             initial_alphabet=pre_tokenizers.ByteLevel.alphabet())
    tok.train_from_iterator(wm.corpus_lines(corpus_words), trainer=tr)
    n = tok.get_vocab_size()
    if n < vocab - 1:
        tok.add_tokens(["<|filler_%d|>" % i for i in range(vocab - 1 - n)])
    tok.add_special_tokens([AddedToken("<|endoftext|>", special=True)])
    os.makedirs(out_dir, exist_ok=True)
    tok.save(os.path.join(out_dir, "tokenizer.json"))
    with open(os.path.join(out_dir, "tokenizer_config.json"), "w") as f:
        json.dump({"bos_token": "<|endoftext|>", "eos_token": "<|endoftext|>", "model_max_length": 1024}, f)
    return tok


def train_wordpiece_tokenizer(out_dir, wm: WordModel = None, corpus_words=1_000_000, vocab=30522, lowercase=True):
    from tokenizers import Tokenizer, decoders, models, normalizers, pre_tokenizers, processors, trainers

    wm = wm or WordModel(seed=7)
    tok = Tokenizer(models.WordPiece(unk_token="[UNK]", max_input_chars_per_word=100))
    tok.normalizer = normalizers.BertNormalizer(clean_text=True, handle_chinese_chars=True, strip_accents=None,
                                                lowercase=lowercase)
    tok.pre_tokenizer = pre_tokenizers.BertPreTokenizer()
    tok.decoder = decoders.WordPiece(prefix="##")
    specials = ["[PAD]", "[UNK]", "[CLS]", "[SEP]", "[MASK]"]
    tr = trainers.WordPieceTrainer(vocab_size=vocab, special_tokens=specials, show_progress=False)
    tok.train_from_iterator(wm.corpus_lines(corpus_words), trainer=tr)
    n = tok.get_vocab_size()
    if n < vocab:
        tok.add_tokens(["[unused%d]" % i for i in range(vocab - n)])
    tok.post_processor = processors.TemplateProcessing(
        single="[CLS] $A [SEP]", pair="[CLS] $A [SEP] $B:1 [SEP]:1",
        special_tokens=[("[CLS]", tok.token_to_id("[CLS]")), ("[SEP]", tok.token_to_id("[SEP]"))])
    os.makedirs(out_dir, exist_ok=True)
    tok.save(os.path.join(out_dir, "tokenizer.json"))
    with open(os.path.join(out_dir, "tokenizer_config.json"), "w") as f:
        json.dump({"cls_token": "[CLS]", "sep_token": "[SEP]", "pad_token": "[PAD]", "unk_token": "[UNK]",
                   "do_lower_case": lowercase, "model_max_length": 512}, f)
    return tok


def train_xlmr_unigram_tokenizer(out_dir, wm: WordModel = None, corpus_words=600_000, vocab=16000):
    """XLM-R / bge-m3 style tokenizer.json: SentencePiece Unigram (nmt_nfkc Precompiled charsmap,
    Metaspace, <s> $A </s>) with XLM-R's special ids <s>=0 <pad>=1 </s>=2 <unk>=3 -- the layout
    transformers' SpmConverter writes for xlm-roberta. The piece inventory is trained on the synthetic
    corpus (a real 250k-piece vocabulary needs a real corpus); ids stay < the model's vocab_size."""
    import tempfile

    import sentencepiece as spm
    from sentencepiece import sentencepiece_model_pb2 as pb
    from tokenizers import AddedToken, Regex, Tokenizer, decoders, models, normalizers, pre_tokenizers, processors

    wm = wm or WordModel(seed=11)
    with tempfile.TemporaryDirectory() as td:
        corpus = os.path.join(td, "c.txt")
        with open(corpus, "w", encoding="utf-8") as f:
            f.write("\n".join(wm.corpus_lines(corpus_words)))
        spm.SentencePieceTrainer.train(input=corpus, model_prefix=os.path.join(td, "m"), vocab_size=vocab,
                                       model_type="unigram", normalization_rule_name="nmt_nfkc",
                                       character_coverage=1.0, bos_id=0, pad_id=1, eos_id=2, unk_id=3,
                                       hard_vocab_limit=False, minloglevel=2)
        proto = pb.ModelProto()
        with open(os.path.join(td, "m.model"), "rb") as f:
            proto.ParseFromString(f.read())
    pieces = [(p.piece, p.score) for p in proto.pieces]
    tok = Tokenizer(models.Unigram(pieces, unk_id=3))
    tok.normalizer = normalizers.Sequence([normalizers.Precompiled(proto.normalizer_spec.precompiled_charsmap),
                                           normalizers.Replace(Regex(" {2,}"), " ")])
    tok.pre_tokenizer = pre_tokenizers.Metaspace()
    tok.decoder = decoders.Metaspace()
    tok.add_special_tokens([AddedToken(t, special=True) for t in ("<s>", "<pad>", "</s>", "<unk>")])
    tok.post_processor = processors.TemplateProcessing(
        single="<s> $A </s>", pair="<s> $A </s> </s> $B </s>", special_tokens=[("<s>", 0), ("</s>", 2)])
    os.makedirs(out_dir, exist_ok=True)
    tok.save(os.path.join(out_dir, "tokenizer.json"))
    with open(os.path.join(out_dir, "tokenizer_config.json"), "w") as f:
        json.dump({"bos_token": "<s>", "eos_token": "</s>", "pad_token": "<pad>", "unk_token": "<unk>",
                   "cls_token": "<s>", "sep_token": "</s>", "model_max_length": 8192,
                   "tokenizer_class": "XLMRobertaTokenizer"}, f)
    return tok


# --------------------------------------------------------------------------- checkpoints
def llama_state_dict(cfg, seed=0, std=0.02):
    g = torch.Generator().manual_seed(seed)
    H, I, D = cfg.hidden_size, cfg.intermediate_size, cfg.head_dim
    Hq, Hkv = cfg.num_attention_heads, cfg.num_key_value_heads

    def r(*s):
        return (torch.randn(*s, generator=g) * std).bfloat16()

    def one(n):
        return (1 + 0.1 * torch.randn(n, generator=g)).bfloat16()

    sd = {"model.embed_tokens.weight": r(cfg.vocab_size, H)}
    for i in range(cfg.num_hidden_layers):
        p = "model.layers.%d." % i
        sd[p + "input_layernorm.weight"] = one(H)
        sd[p + "post_attention_layernorm.weight"] = one(H)
        sd[p + "self_attn.q_proj.weight"] = r(Hq * D, H)
        sd[p + "self_attn.k_proj.weight"] = r(Hkv * D, H)
        sd[p + "self_attn.v_proj.weight"] = r(Hkv * D, H)
        sd[p + "self_attn.o_proj.weight"] = r(H, Hq * D)
        sd[p + "mlp.gate_proj.weight"] = r(I, H)
        sd[p + "mlp.up_proj.weight"] = r(I, H)
        sd[p + "mlp.down_proj.weight"] = r(H, I)
    sd["model.norm.weight"] = one(H)
    if not cfg.tie_word_embeddings:
        sd["lm_head.weight"] = r(cfg.vocab_size, H)
    return sd


def write_llama_checkpoint(out_dir, cfg, seed=0, n_shards=4, tokenizer=True, wm=None, gen_overrides=None):
    """The download_model.py file set, random-init (offline stand-in for the HF download)."""
    from ..runtime.safetensors_io import save_sharded

    os.makedirs(out_dir, exist_ok=True)
    with open(os.path.join(out_dir, "config.json"), "w") as f:
        json.dump(cfg.to_hf_dict(), f, indent=2)
    gen = {"bos_token_id": cfg.bos_token_id, "eos_token_id": cfg.eos_token_id, "do_sample": True,
           "temperature": 0.6, "top_p": 0.9}
    gen.update(gen_overrides or {})
    with open(os.path.join(out_dir, "generation_config.json"), "w") as f:
        json.dump(gen, f, indent=2)
    save_sharded(llama_state_dict(cfg, seed), out_dir, n_shards)
    if tokenizer and not os.path.exists(os.path.join(out_dir, "tokenizer.json")):
        if cfg.vocab_size >= 128256:
            train_llama3_tokenizer(out_dir, wm)
        else:
            train_small_bpe(out_dir, cfg.vocab_size, wm)


def train_small_bpe(out_dir, vocab, wm=None):
    """Small byte-level BPE for tiny test models (vocab includes 2 specials: <s>=1? no --
    specials are the LAST two ids: bos = vocab-2, eos = vocab-1)."""
    from tokenizers import AddedToken, Tokenizer, decoders, models, pre_tokenizers, processors, trainers

    wm = wm or WordModel(n_words=20000, seed=11)
    tok = Tokenizer(models.BPE())
    tok.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False)
    tok.decoder = decoders.ByteLevel()
    tr = trainers.BpeTrainer(vocab_size=vocab - 2, show_progress=False,
                             initial_alphabet=pre_tokenizers.ByteLevel.alphabet())
    tok.train_from_iterator(wm.corpus_lines(200000), trainer=tr)
    n = tok.get_vocab_size()
    if n < vocab - 2:
        tok.add_tokens(["<|f%d|>" % i for i in range(vocab - 2 - n)])
    tok.add_special_tokens([AddedToken("<s>", special=True), AddedToken("</s>", special=True)])
    tok.post_processor = processors.TemplateProcessing(single="<s> $A", special_tokens=[("<s>", tok.token_to_id("<s>"))])
    os.makedirs(out_dir, exist_ok=True)
    tok.save(os.path.join(out_dir, "tokenizer.json"))
    with open(os.path.join(out_dir, "tokenizer_config.json"), "w") as f:
        json.dump({"bos_token": "<s>", "eos_token": "</s>"}, f)
    return tok


def encoder_state_dict(cfg, seed=0, std=0.02):
    g = torch.Generator().manual_seed(seed)
    H, I = cfg.hidden_size, cfg.intermediate_size

    def r(*s):
        return (torch.randn(*s, generator=g) * std).bfloat16()

    def one(n):
        return (1 + 0.05 * torch.randn(n, generator=g)).bfloat16()

    sd = {"embeddings.word_embeddings.weight": r(cfg.vocab_size, H),
          "embeddings.position_embeddings.weight": r(cfg.max_position_embeddings, H),
          "embeddings.token_type_embeddings.weight": r(cfg.type_vocab_size, H),
          "embeddings.LayerNorm.weight": one(H), "embeddings.LayerNorm.bias": r(H)}
    for i in range(cfg.num_hidden_layers):
        p = "encoder.layer.%d." % i
        for n in ("query", "key", "value"):
            sd[p + "attention.self.%s.weight" % n] = r(H, H)
            sd[p + "attention.self.%s.bias" % n] = r(H)
        sd[p + "attention.output.dense.weight"] = r(H, H)
        sd[p + "attention.output.dense.bias"] = r(H)
        sd[p + "attention.output.LayerNorm.weight"] = one(H)
        sd[p + "attention.output.LayerNorm.bias"] = r(H)
        sd[p + "intermediate.dense.weight"] = r(I, H)
        sd[p + "intermediate.dense.bias"] = r(I)
        sd[p + "output.dense.weight"] = r(H, I)
        sd[p + "output.dense.bias"] = r(H)
        sd[p + "output.LayerNorm.weight"] = one(H)
        sd[p + "output.LayerNorm.bias"] = r(H)
    return sd


def write_encoder_checkpoint(out_dir, cfg, seed=0, wm=None):
    """sentence-transformers directory layout (Transformer -> Pooling -> Normalize)."""
    from ..runtime.safetensors_io import save_file

    os.makedirs(os.path.join(out_dir, "1_Pooling"), exist_ok=True)
    os.makedirs(os.path.join(out_dir, "2_Normalize"), exist_ok=True)
    with open(os.path.join(out_dir, "config.json"), "w") as f:
        json.dump(cfg.to_hf_dict(), f, indent=2)
    with open(os.path.join(out_dir, "1_Pooling", "config.json"), "w") as f:
        json.dump({"word_embedding_dimension": cfg.hidden_size, "pooling_mode_cls_token": cfg.pooling == "cls",
                   "pooling_mode_mean_tokens": cfg.pooling == "mean"}, f, indent=2)
    with open(os.path.join(out_dir, "sentence_bert_config.json"), "w") as f:
        json.dump({"max_seq_length": cfg.max_seq_length, "do_lower_case": False}, f)
    with open(os.path.join(out_dir, "modules.json"), "w") as f:
        json.dump([{"idx": 0, "name": "0", "path": "", "type": "sentence_transformers.models.Transformer"},
                   {"idx": 1, "name": "1", "path": "1_Pooling", "type": "sentence_transformers.models.Pooling"},
                   {"idx": 2, "name": "2", "path": "2_Normalize",
                    "type": "sentence_transformers.models.Normalize"}], f, indent=2)
    save_file(encoder_state_dict(cfg, seed), os.path.join(out_dir, "model.safetensors"), metadata={"format": "pt"})
    if not os.path.exists(os.path.join(out_dir, "tokenizer.json")):
        if cfg.model_type == "xlm-roberta":
            train_xlmr_unigram_tokenizer(out_dir, wm, vocab=min(16000, cfg.vocab_size))
        else:
            train_wordpiece_tokenizer(out_dir, wm, vocab=cfg.vocab_size)


def write_pdf_corpus(out_dir, n_docs, pages=4, words_per_page=600, wm=None, seed=0):
    from ..ingest.pdf import write_pdf

    wm = wm or WordModel(n_words=50000, seed=seed)
    rng = np.random.default_rng(seed)
    os.makedirs(out_dir, exist_ok=True)
    paths = []
    for d in range(n_docs):
        pg = []
        for _ in range(pages):
            words = wm.text(words_per_page, rng).split()
            pg.append([" ".join(words[i:i + 12]) for i in range(0, len(words), 12)])
        p = os.path.join(out_dir, "doc_%05d.pdf" % d)
        with open(p, "wb") as f:
            f.write(write_pdf(pg, compress=bool(d % 2 == 0), object_streams=bool(d % 3 == 0)))
        paths.append(p)
    return paths
