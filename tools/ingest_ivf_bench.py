"""Ingest throughput and a real 1M-chunk IVF-Flat build on one MI355X.

1. Ingest: N x 1000-word chunks (the reference chunker's windows, /root/reference/llm/rag.py:63-75)
   through the embedding engine (C++ tokenizer threads + packed varlen encoder) for each embedder:
   chunks/s and tokens/s, tokenize and encode split.
2. IVF (BASELINE config 4): a corpus of M chunks of W words, EMBEDDED by the MiniLM-shaped encoder
   (no random padding), indexed twice: FlatL2 (ground truth) and IVF-Flat (GPU k-means training with
   the MFMA assign kernel + list appends); reports build time, search latency and recall@4 vs flat for
   a set of held-out queries (themselves embedded query texts).

  python tools/ingest_ivf_bench.py --embedders minilm,bge-large --chunks 10000 \
      --ivf-chunks 1000000 --ivf-words 100 --nlist 4096 --nprobe 32 --json gpurun_out/ingest_ivf.json
Random-init weights (no checkpoints offline); synthetic Zipfian pseudo-English corpus.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def log(*a):
    print(*a, flush=True)


def sync():
    torch.cuda.synchronize()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--embedders", default="minilm,bge-large")
    ap.add_argument("--chunks", type=int, default=10000)
    ap.add_argument("--ivf-chunks", type=int, default=1_000_000)
    ap.add_argument("--ivf-words", type=int, default=100)
    ap.add_argument("--nlist", type=int, default=4096)
    ap.add_argument("--nprobe", type=int, default=32)
    ap.add_argument("--queries", type=int, default=1000)
    ap.add_argument("--topics", type=int, default=2000,
                    help="topical structure of the IVF corpus (0: plain Zipf words, no clusters)")
    ap.add_argument("--topic-mix", type=float, default=0.5, help="share of a chunk's words drawn from its topic")
    ap.add_argument("--topic-words", type=int, default=400, help="vocabulary size of one topic")
    ap.add_argument("--json", default=None)
    a = ap.parse_args()

    from rag_llm_k8s_amd import _build
    from rag_llm_k8s_amd.engine.encoder_engine import EmbeddingEngine
    from rag_llm_k8s_amd.index.flat import FlatL2Index
    from rag_llm_k8s_amd.index.ivf import IVFFlatIndex
    from rag_llm_k8s_amd.models import encoder as E
    from rag_llm_k8s_amd.runtime.tokenizer import Tokenizer
    from rag_llm_k8s_amd.utils.synthetic import WordModel, train_wordpiece_tokenizer
    from rag_llm_k8s_amd.utils.workload import TopicCorpus, asset_dir, make_chunks, make_queries

    _build.build_all()
    dev = "cuda:0"
    res = {"device": torch.cuda.get_device_name(0), "ingest": {}, "ivf": {}}
    wm = WordModel(n_words=400000, seed=0)
    tdir = os.path.join(asset_dir("enc_wp_30522"), "enc")
    if not os.path.exists(os.path.join(tdir, "tokenizer.json")):
        train_wordpiece_tokenizer(tdir, wm, corpus_words=600_000, vocab=30522)
    tok = Tokenizer(tdir)
    log("tokenizer backend:", tok.backend)

    # ------------------------------------------------------------------ 1. ingest throughput
    t0 = time.time()
    chunks = make_chunks(wm, a.chunks, 1000, seed=0)
    log("corpus: %d x 1000-word chunks in %.1fs" % (len(chunks), time.time() - t0))
    engines = {}
    for name in [e for e in a.embedders.split(",") if e]:
        cfg = {"minilm": E.minilm_l6, "bge-large": E.bge_large_en}[name]()
        emb = EmbeddingEngine(E.EncoderModel(cfg, E.EncoderWeights.random(cfg, dev, seed=1), dev), tok)
        emb.embed(chunks[:512])  # warm-up (kernel first launches, allocator)
        sync()
        t0 = time.time()
        ids, lens = emb.tokenize_flat(chunks)
        t_tok = time.time() - t0
        t1 = time.time()
        v = emb.embed_flat(ids, lens)
        sync()
        t_enc = time.time() - t1
        t2 = time.time()
        v2 = emb.embed(chunks)  # the ingest path: tokenisation of group g+1 overlaps encoding of group g
        sync()
        t_pipe = time.time() - t2
        assert torch.allclose(v, v2)
        ntok = int(lens.sum())
        r = {"chunks": len(chunks), "max_seq_length": cfg.max_seq_length, "tokens": ntok,
             "tokenize_s": round(t_tok, 3), "encode_s": round(t_enc, 3), "pipelined_s": round(t_pipe, 3),
             "chunks_per_s": round(len(chunks) / t_pipe, 1),
             "encode_tokens_per_s": round(ntok / t_enc, 0), "dim": int(v.shape[1])}
        res["ingest"][name] = r
        log("ingest %s: %s" % (name, r))
        engines[name] = emb

    # ------------------------------------------------------------------ 2. 1M-chunk IVF build
    if a.ivf_chunks > 0:
        emb = engines.get("minilm")
        if emb is None:
            cfg = E.minilm_l6()
            emb = EmbeddingEngine(E.EncoderModel(cfg, E.EncoderWeights.random(cfg, dev, seed=1), dev), tok)
        M, d = a.ivf_chunks, emb.dim
        tc = TopicCorpus(wm, n_topics=a.topics, topic_words=a.topic_words, mix=a.topic_mix) if a.topics else None
        xb = torch.empty((M, d), dtype=torch.float32, device=dev)
        t0 = time.time()
        bs = 50000
        for lo in range(0, M, bs):
            n = min(bs, M - lo)
            texts = (tc.chunks(n, a.ivf_words, seed=1000 + lo // bs) if tc else
                     make_chunks(wm, n, a.ivf_words, seed=1000 + lo // bs))
            xb[lo:lo + n] = emb.embed(texts)
            if (lo // bs) % 4 == 0:
                log("  embedded %d / %d (%.0fs)" % (lo + n, M, time.time() - t0))
        sync()
        t_emb = time.time() - t0
        qtexts = tc.queries(a.queries, 12, seed=31337) if tc else make_queries(wm, a.queries, seed=31337, words=12)
        q = emb.embed(qtexts)
        sync()
        log("embedded %d chunks in %.1fs (%.0f chunks/s)" % (M, t_emb, M / t_emb))

        t0 = time.time()
        flat = FlatL2Index(d, device=dev, capacity=M)
        flat.add(xb)
        sync()
        t_flat = time.time() - t0
        Df, If = flat.search(q, 4)
        # relative contrast (mean distance to a random base vector / distance to the 4th neighbour): ~1
        # means the neighbourhoods are barely distinguishable and any partitioned index loses recall
        ridx = torch.randint(0, M, (256,), device=dev)
        dmean = torch.cdist(q, xb[ridx]).pow(2).mean(1).cpu()
        contrast = float((dmean / Df[:, 3].clamp_min(1e-12)).mean())
        log("relative contrast (mean dist / 4-NN dist): %.3f" % contrast)

        t0 = time.time()
        ivf = IVFFlatIndex(d, device=dev, nlist=a.nlist, nprobe=a.nprobe)
        ivf.train(xb)
        sync()
        t_train = time.time() - t0
        log("IVF train (k-means %d lists on %d points): %.1fs" % (ivf.nlist, min(M, 256 * a.nlist), t_train))
        t1 = time.time()
        for lo in range(0, M, 250000):  # appended in batches, as uploads would
            ivf.add(xb[lo:lo + 250000])
        sync()
        t_add = time.time() - t1
        log("IVF add: %.1fs (%d store regrows)" % (t_add, ivf.regrows))

        def timed(idx, qq, reps=20):
            idx.search(qq, 4)
            sync()
            t = time.time()
            for _ in range(reps):
                out = idx.search(qq, 4)
            sync()
            return (time.time() - t) / reps * 1e3, out

        ivf_rows = {}
        for npb in sorted({1, 8, a.nprobe, 4 * a.nprobe, ivf.nlist}):
            ivf.nprobe = npb
            _, (Di, Ii) = timed(ivf, q, reps=3)
            rec = float(np.mean([len(set(x.tolist()) & set(y.tolist())) / 4 for x, y in zip(Ii, If)]))
            ms1, _ = timed(ivf, q[:1])
            ms32, _ = timed(ivf, q[:32])
            ivf_rows[npb] = {"recall_at_4": round(rec, 4), "search_ms_b1": round(ms1, 3), "search_ms_b32": round(ms32, 3)}
            log("nprobe %d: %s" % (npb, ivf_rows[npb]))
        fms1, _ = timed(flat, q[:1])
        fms32, _ = timed(flat, q[:32])
        sizes = ivf._size
        res["ivf"] = {"chunks": M, "words_per_chunk": a.ivf_words, "topics": a.topics, "topic_mix": a.topic_mix, "topic_words": a.topic_words,
                      "relative_contrast": round(contrast, 3), "embedder": "all-MiniLM-L6-v2 (random init)",
                      "dim": d, "nlist": ivf.nlist, "queries": a.queries,
                      "embed_s": round(t_emb, 1), "flat_build_s": round(t_flat, 2), "ivf_train_s": round(t_train, 2),
                      "ivf_add_s": round(t_add, 2), "ivf_build_s": round(t_train + t_add, 2),
                      "regrows": ivf.regrows, "list_size_min_med_max": [int(sizes.min()), int(np.median(sizes)),
                                                                        int(sizes.max())],
                      "by_nprobe": ivf_rows, "flat_search_ms_b1": round(fms1, 3), "flat_search_ms_b32": round(fms32, 3)}
        log("ivf:", json.dumps(res["ivf"]))
    line = json.dumps(res)
    print(line, flush=True)
    if a.json:
        os.makedirs(os.path.dirname(a.json) or ".", exist_ok=True)
        with open(a.json, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
