"""Batched sentence-embedding engine (replaces SentenceTransformer.encode, D3).

Reference: one chunk at a time, batch size 1 (/root/reference/llm/rag.py:54-55,100-101).
Here: tokenise (C++ worker threads, truncated encode, flat int32 output), sort by length, pack
into varlen batches of up to `max_batch_tokens` tokens (no padding FLOPs), run the encoder,
restore the input order. Large inputs are pipelined: the next group of texts is tokenised on the
CPU (GIL released) while the GPU encodes the current one, so ingest costs max(tokenise, encode)
rather than their sum. Optional data parallelism: each rank embeds a strided shard and the
results are all-gathered over RCCL (parallel/dp.py).
"""
from __future__ import annotations

from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch

PIPELINE_GROUP = 2048  # texts per tokenise/encode pipeline stage


class EmbeddingEngine:
    def __init__(self, model, tokenizer, max_batch_tokens: int = 65536):
        self.model = model
        self.tok = tokenizer
        self.max_batch_tokens = max_batch_tokens
        self.device = model.device
        self._pool = None

    @property
    def dim(self):
        return self.model.cfg.hidden_size

    def tokenize(self, texts):
        return self.tok.encode_batch(texts, add_special_tokens=True, max_length=self.model.cfg.max_seq_length)

    def tokenize_flat(self, texts):
        """(ids int32 [sum lens], lens int32 [n]) numpy."""
        if hasattr(self.tok, "encode_batch_flat"):
            return self.tok.encode_batch_flat(texts, add_special_tokens=True, max_length=self.model.cfg.max_seq_length)
        out = self.tokenize(texts)
        lens = np.array([len(x) for x in out], dtype=np.int32)
        ids = np.array([t for x in out for t in x], dtype=np.int32)
        return ids, lens

    @torch.no_grad()
    def embed_ids(self, id_lists):
        lens = np.array([len(x) for x in id_lists], dtype=np.int32)
        ids = np.array([t for x in id_lists for t in x], dtype=np.int32)
        return self.embed_flat(ids, lens)

    @torch.no_grad()
    def embed_flat(self, ids, lens, out=None, row0=0):
        """Embeddings of the sequences given as flat ids + lens; written to out[row0 + i] (allocated
        when None). Returns out."""
        n = len(lens)
        if out is None:
            out = torch.empty((n, self.dim), dtype=torch.float32, device=self.device)
        if n == 0:
            return out
        starts = np.zeros(n + 1, dtype=np.int64)
        np.cumsum(lens, out=starts[1:])
        order = np.argsort(-lens.astype(np.int64), kind="stable")
        slens = lens[order].astype(np.int64)
        i = 0
        while i < n:
            # greedy packing in descending length order: as many sequences as fit in max_batch_tokens
            csum = np.cumsum(slens[i:])
            j = i + max(1, int(np.searchsorted(csum, self.max_batch_tokens, side="right")))
            rows = order[i:j]
            flat = np.concatenate([ids[starts[r]:starts[r + 1]] for r in rows])
            t = torch.from_numpy(flat).to(self.device)  # pageable source: a synchronous copy, safe to reuse
            emb = self.model.forward_packed(t, [int(x) for x in slens[i:j]])
            out[torch.from_numpy(rows + row0).to(self.device)] = emb
            i = j
        return out

    def embed(self, texts):
        """fp32 [n, d] unit-norm embeddings on the engine device."""
        texts = list(texts)
        n = len(texts)
        if n <= PIPELINE_GROUP:
            return self.embed_flat(*self.tokenize_flat(texts))
        out = torch.empty((n, self.dim), dtype=torch.float32, device=self.device)
        if self._pool is None:
            self._pool = ThreadPoolExecutor(max_workers=1, thread_name_prefix="ragk-tokenize")
        groups = [(lo, texts[lo:lo + PIPELINE_GROUP]) for lo in range(0, n, PIPELINE_GROUP)]
        fut = self._pool.submit(self.tokenize_flat, groups[0][1])
        for g, (lo, _) in enumerate(groups):
            ids, lens = fut.result()
            if g + 1 < len(groups):  # tokenise the next group while this one encodes
                fut = self._pool.submit(self.tokenize_flat, groups[g + 1][1])
            self.embed_flat(ids, lens, out, lo)
        return out
