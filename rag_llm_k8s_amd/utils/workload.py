"""Synthetic RAG serving workload (shared by bench.py, smoke() and the GPU e2e tests).

Builds, fully offline and on the target device:
  * a Llama-3-style 128,256-token BPE tokenizer and a BERT WordPiece tokenizer trained on a
    Zipfian pseudo-English corpus (same word model as the documents);
  * random-init Llama weights of the requested architecture generated directly in HBM;
  * a random-init sentence encoder (MiniLM-L6 / bge-large / bge-m3 shaped);
  * a corpus of N chunks of `chunk_words` words (the reference chunker's 1000-word windows),
    embedded by the encoder into the HBM-resident index;
  * a RagService wired exactly like the server (retrieve_k / context_k / prompt template).
"""
from __future__ import annotations

import hashlib
import json
import os
import time

import numpy as np
import torch

from ..config import RagConfig
from .synthetic import (WordModel, train_llama3_tokenizer, train_small_bpe, train_wordpiece_tokenizer,
                        train_xlmr_unigram_tokenizer)


def asset_dir(tag):
    d = os.path.join(os.environ.get("RAGK_ASSET_DIR", "/tmp/ragk_assets"), tag)
    os.makedirs(d, exist_ok=True)
    return d


def _once(path, build, ctx=None):
    """Build an asset once per node: rank 0 builds, others wait on the file."""
    from ..parallel.dist import barrier

    done = path + ".done"
    is_builder = ctx is None or ctx.local_rank == 0
    if is_builder and not os.path.exists(done):
        build()
        with open(done, "w") as f:
            f.write("ok")
    if ctx is not None and ctx.initialized:
        barrier(ctx)
    t0 = time.time()
    while not os.path.exists(done):
        time.sleep(0.2)
        if time.time() - t0 > 600:
            raise TimeoutError("asset %s never appeared" % path)


def make_tokenizers(wm, llm_vocab, enc_vocab, ctx=None, enc_kind="wordpiece"):
    """LLM BPE + encoder tokenizer: BERT WordPiece (MiniLM / bge-large) or XLM-R SentencePiece
    Unigram (bge-m3)."""
    from ..runtime.tokenizer import Tokenizer

    tag = "tok_%d_%d" % (llm_vocab, enc_vocab) + ("" if enc_kind == "wordpiece" else "_" + enc_kind)
    d = asset_dir(tag)
    llm_d, enc_d = os.path.join(d, "llm"), os.path.join(d, "enc")

    def build():
        if llm_vocab >= 128256:
            train_llama3_tokenizer(llm_d, wm)
        else:
            train_small_bpe(llm_d, llm_vocab, wm)
        if enc_kind == "unigram":
            train_xlmr_unigram_tokenizer(enc_d, wm, corpus_words=600_000, vocab=enc_vocab)
        else:
            train_wordpiece_tokenizer(enc_d, wm, corpus_words=600_000, vocab=enc_vocab)

    _once(os.path.join(d, "tok"), build, ctx)
    return Tokenizer(llm_d), Tokenizer(enc_d)


def make_chunks(wm, n_chunks, chunk_words, seed=0):
    rng = np.random.default_rng(seed + 123)
    idx = np.searchsorted(wm.cdf, rng.random(n_chunks * chunk_words), side="right")
    idx = np.minimum(idx, len(wm.words) - 1)
    words = wm.words[idx]
    out = []
    for i in range(n_chunks):
        w = words[i * chunk_words:(i + 1) * chunk_words]
        out.append(" ".join(w))
    return out


class TopicCorpus:
    """Chunks with topical structure, as a real corpus has (documents cluster by subject, which is what
    makes an IVF index's coarse quantizer useful): topic t owns `topic_words` mid-frequency words; a chunk
    of topic t draws a `mix` share of its words from them and the rest from the global Zipf law. Queries
    are drawn the same way from a topic, so their true neighbours are that topic's chunks."""

    def __init__(self, wm, n_topics=2000, topic_words=400, mix=0.5, seed=0):
        rng = np.random.default_rng(seed + 99)
        lo, hi = 500, min(len(wm.words), 200000)
        self.wm, self.mix = wm, mix
        self.vocab = rng.integers(lo, hi, size=(n_topics, topic_words))

    def _words(self, n, words, rng):
        topics = rng.integers(0, len(self.vocab), n)
        glob = np.minimum(np.searchsorted(self.wm.cdf, rng.random((n, words)), side="right"), len(self.wm.words) - 1)
        top = self.vocab[topics[:, None], rng.integers(0, self.vocab.shape[1], (n, words))]
        idx = np.where(rng.random((n, words)) < self.mix, top, glob)
        w = self.wm.words[idx]
        return [" ".join(r) for r in w], topics

    def chunks(self, n, words, seed):
        return self._words(n, words, np.random.default_rng(seed))[0]

    def paragraph_chunks(self, n, words, seed, para_words=100, paras_per_topic=64):
        """Fast path for index-scale corpora (1M x 1000 words): each topic owns a pool of
        `paras_per_topic` topical paragraphs and a chunk is `words // para_words` of its topic's
        paragraphs in random order, so chunks of one topic share vocabulary but (almost) never text."""
        rng = np.random.default_rng(seed)
        if getattr(self, "_paras", None) is None:
            prng = np.random.default_rng(4242)
            self._paras = self._words(len(self.vocab) * paras_per_topic, para_words, prng)[0]
        per = max(1, words // para_words)
        topics = rng.integers(0, len(self.vocab), n)
        pick = topics[:, None] * paras_per_topic + rng.integers(0, paras_per_topic, (n, per))
        P = self._paras
        return [" ".join([P[j] for j in row]) for row in pick.tolist()]

    def queries(self, n, words, seed):
        return [q.capitalize() + "?" for q in self._words(n, words, np.random.default_rng(seed + 7))[0]]


def make_queries(wm, n, seed, words=12):
    rng = np.random.default_rng(seed)
    qs = []
    for _ in range(n):
        w = list(wm.sample(words, rng))
        qs.append(" ".join(w).capitalize() + "?")
    return qs


class Workload:
    def __init__(self, svc, wm, llm_tok, timings, n_chunks):
        self.svc, self.wm, self.llm_tok, self.timings, self.n_chunks = svc, wm, llm_tok, timings, n_chunks


def build_workload(model="8b", embedder="minilm", n_chunks=10000, chunk_words=1000, retrieve_k=4, context_k=4,
                   max_new_tokens=150, max_batch=32, max_model_len=8192, max_prefill_tokens=32768, device="cuda",
                   ctx=None, tp_comm=None, seed=0, use_graphs=True, index_type="flat", kv_blocks=None,
                   word_vocab=400000, dtype="bf16", index_vectors=0, start_threads=False, ignore_eos=False,
                   mixed_prefill_tokens=0, progress=None):
    """`progress(msg)`: called after each setup stage (bench.py prints it: a 70B / 1M-vector setup runs
    for minutes)."""
    from ..engine.encoder_engine import EmbeddingEngine
    from ..engine.llm_engine import LLMEngine
    from ..index.store import DocumentStore
    from ..models import encoder as E
    from ..models import llama as L
    from ..server.rag_service import RagService

    t = {}
    t0 = time.time()
    wm = WordModel(n_words=word_vocab, seed=seed)
    lcfg = {"8b": L.llama31_8b, "70b": L.llama31_70b,
            "tiny": lambda: L.llama_tiny(vocab=1024, layers=2, hidden=512, heads=4, kv_heads=2, inter=512),
            # TP=4/8 layouts: 8 KV heads (1 per rank at TP=8, as Llama-3.1 8B/70B), vocab % 8 != 0
            "tiny8": lambda: L.llama_tiny(vocab=1001, layers=2, hidden=512, heads=16, kv_heads=8, inter=1024)}[model]()
    ecfg = {"minilm": E.minilm_l6, "bge-large": E.bge_large_en, "bge-m3": E.bge_m3,
            "tiny": lambda: E.EncoderConfig(vocab_size=2048, hidden_size=128, num_hidden_layers=2,
                                            num_attention_heads=4, intermediate_size=256, max_seq_length=128)}[embedder]()
    xlmr = ecfg.model_type == "xlm-roberta"  # bge-m3: XLM-R embeddings (position offset) + Unigram ids
    enc_vocab = min(16000, ecfg.vocab_size) if xlmr else ecfg.vocab_size
    llm_tok, enc_tok = make_tokenizers(wm, lcfg.vocab_size, enc_vocab, ctx, "unigram" if xlmr else "wordpiece")
    t["tokenizers_s"] = time.time() - t0
    say = progress or (lambda msg: None)
    say("tokenizers %.1f s" % t["tokenizers_s"])

    t0 = time.time()
    tp_rank = ctx.tp_rank if ctx is not None else 0
    tp_size = ctx.tp if ctx is not None else 1
    w = L.LlamaWeights.random(lcfg, device, tp_rank, tp_size, seed=seed)
    if dtype == "fp8":  # BASELINE config 5: e4m3fn linear weights (bf16 embeddings / norms / lm_head)
        w.quantize_fp8()
        if device.startswith("cuda"):
            torch.cuda.empty_cache()
    m = L.LlamaModel(lcfg, w, device, comm=tp_comm, max_positions=max_model_len)
    blocks = kv_blocks or (max_batch * (-(-max_model_len // 64)) + 16)
    engine = LLMEngine(m, num_blocks=blocks, max_batch=max_batch, max_prefill_tokens=max_prefill_tokens,
                       max_model_len=max_model_len, eos_ids=lcfg.eos_token_id, use_graphs=use_graphs,
                       tp_group=ctx.tp_group if (ctx is not None and tp_size > 1) else None,
                       mixed_prefill_tokens=mixed_prefill_tokens)
    ew = E.EncoderWeights.random(ecfg, device, seed=seed + 1)
    emb = EmbeddingEngine(E.EncoderModel(ecfg, ew, device), enc_tok)
    t["weights_s"] = time.time() - t0
    say("weights %.1f s" % t["weights_s"])

    t0 = time.time()
    chunks = make_chunks(wm, n_chunks, chunk_words, seed)
    t["corpus_s"] = time.time() - t0
    t0 = time.time()
    cfg = RagConfig(device=device, retrieve_k=retrieve_k, context_k=context_k, max_new_tokens=max_new_tokens,
                    max_batch=max_batch, max_model_len=max_model_len, index_path="/tmp/ragk_bench_index",
                    index_type=index_type, seed=seed, max_prefill_tokens=max_prefill_tokens, ignore_eos=ignore_eos,
                    mixed_prefill_tokens=mixed_prefill_tokens)
    n_index = max(n_chunks, index_vectors)
    store = DocumentStore(cfg.index_path, emb.dim, device=device, index_type=index_type,
                          ivf_nlist=4096 if n_index >= 500_000 else 1024)
    vecs = emb.embed(chunks)
    if device.startswith("cuda"):
        torch.cuda.synchronize()
    t["embed_s"] = time.time() - t0  # tokenize + encode of the n_chunks corpus (ingest throughput)
    say("corpus %.1f s, embed %.1f s" % (t["corpus_s"], t["embed_s"]))
    meta = [{"filename": "synthetic_%05d.pdf" % (i // 20), "chunk_id": i % 20, "text": c}
            for i, c in enumerate(chunks)]
    # BASELINE config 4 scale (1M-chunk index): the rest of the index is a second corpus of
    # `chunk_words`-word chunks with topical structure, EMBEDDED by the same encoder (a real corpus, not
    # random vectors; ~1 min for 1M chunks with MiniLM, ~7 GB of host text). Their text is real, so
    # retrieval picks them and the prompts keep the reference chunker's size.
    pads = []
    if index_vectors > len(meta):
        tc = TopicCorpus(wm, n_topics=2000, topic_words=40, mix=0.5, seed=seed)
        bs, done = 65536, len(meta)
        while done < index_vectors:
            nb = min(bs, index_vectors - done)
            texts = tc.paragraph_chunks(nb, chunk_words, seed=seed + 17 + done // bs)
            pads.append((emb.embed(texts), [{"filename": "synthetic_pad_%04d.pdf" % ((done + i) // 1000),
                                             "chunk_id": (done + i) % 1000, "text": x}
                                            for i, x in enumerate(texts)]))
            done += nb
            say("index corpus %d / %d chunks embedded" % (done, index_vectors))
    if index_type == "ivf":  # train the coarse quantizer on the whole corpus (faiss subsample rule)
        store.index.train(torch.cat([vecs] + [v for v, _ in pads]))
    store.add(vecs, meta, dedupe=False, persist=False)
    for v, m in pads:
        store.add(v, m, dedupe=False, persist=False)
    if device.startswith("cuda"):
        torch.cuda.synchronize()
    t["ingest_s"] = time.time() - t0
    say("ingest %.1f s" % t["ingest_s"])
    svc = RagService(cfg, engine, llm_tok, emb, store, gen_config={"do_sample": True,
                                                                   "eos_token_id": lcfg.eos_token_id},
                     start_threads=start_threads)
    svc.ready = True
    return Workload(svc, wm, llm_tok, t, n_chunks)


def config_hash(d):
    return hashlib.sha1(json.dumps(d, sort_keys=True).encode()).hexdigest()[:8]
