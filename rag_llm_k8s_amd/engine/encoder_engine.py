"""Batched sentence-embedding engine (replaces SentenceTransformer.encode, D3).

Reference: one chunk at a time, batch size 1 (/root/reference/llm/rag.py:54-55,100-101).
Here: tokenise all texts, sort by length, pack into varlen batches of up to
`max_batch_tokens` tokens (no padding FLOPs), run the encoder, restore the input order.
Optional data parallelism: each rank embeds a strided shard and the results are
all-gathered over RCCL (parallel/dp.py).
"""
from __future__ import annotations

import torch


class EmbeddingEngine:
    def __init__(self, model, tokenizer, max_batch_tokens: int = 65536):
        self.model = model
        self.tok = tokenizer
        self.max_batch_tokens = max_batch_tokens
        self.device = model.device

    @property
    def dim(self):
        return self.model.cfg.hidden_size

    def tokenize(self, texts):
        return self.tok.encode_batch(texts, add_special_tokens=True, max_length=self.model.cfg.max_seq_length)

    @torch.no_grad()
    def embed_ids(self, id_lists):
        n = len(id_lists)
        out = torch.empty((n, self.dim), dtype=torch.float32, device=self.device)
        if n == 0:
            return out
        order = sorted(range(n), key=lambda i: -len(id_lists[i]))
        i = 0
        while i < n:
            batch, toks = [], 0
            while i < n and (not batch or toks + len(id_lists[order[i]]) <= self.max_batch_tokens):
                batch.append(order[i])
                toks += len(id_lists[order[i]])
                i += 1
            lens = [len(id_lists[j]) for j in batch]
            flat = [t for j in batch for t in id_lists[j]]
            ids = torch.tensor(flat, dtype=torch.int32).to(self.device)
            emb = self.model.forward_packed(ids, lens)
            out[torch.tensor(batch, device=self.device)] = emb
        return out

    def embed(self, texts):
        """fp32 [n, d] unit-norm embeddings on the engine device."""
        return self.embed_ids(self.tokenize(texts))
