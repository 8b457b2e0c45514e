"""Tokenizer front-end (replaces the reference's AutoTokenizer, D5).

Reference use: tokenizer.encode(full_prompt) -> ids with BOS, no chat template
(/root/reference/llm/rag.py:170) and tokenizer.decode(output[0], skip_special_tokens=True)
(:173); the embedder tokenises with truncation at max_seq_length (sentence-transformers).

Backends, in order of preference:
  1. the native C++ tokenizer in ``_ragk_rt`` (byte-level BPE for Llama-3 / GPT-2,
     WordPiece for BERT, Unigram for XLM-R) reading the same ``tokenizer.json``;
  2. HF ``tokenizers`` (Rust), which the reference itself uses -- also the parity oracle.
Set RAGK_TOKENIZER=hf|native to force one.
"""
from __future__ import annotations

import json
import os

import numpy as np

def _default_threads():
    try:
        n = len(os.sched_getaffinity(0))
    except Exception:
        n = os.cpu_count() or 8
    return max(1, min(16, n))


ENCODE_THREADS = int(os.environ.get("RAGK_TOKENIZER_THREADS", "0")) or _default_threads()


class Tokenizer:
    def __init__(self, path_or_dir, backend=None):
        p = path_or_dir
        if os.path.isdir(p):
            p = os.path.join(p, "tokenizer.json")
        self.path = p
        with open(p, encoding="utf-8") as f:
            self.spec = json.load(f)
        self.cfg = {}
        tc = os.path.join(os.path.dirname(p), "tokenizer_config.json")
        if os.path.exists(tc):
            with open(tc) as f:
                self.cfg = json.load(f)
        backend = backend or os.environ.get("RAGK_TOKENIZER", "auto")
        self.impl = None
        self.backend = None
        if backend in ("auto", "native"):
            try:
                from . import native_rt

                rt = native_rt()
                if rt is not None and hasattr(rt, "Tokenizer"):
                    self.impl = rt.Tokenizer(p)
                    self.backend = "native"
            except Exception:
                if backend == "native":
                    raise
                self.impl = None
        if self.impl is None:
            from tokenizers import Tokenizer as HFTok

            self.impl = HFTok.from_file(p)
            self.impl.no_truncation()
            self.impl.no_padding()
            self.backend = "hf"
        self.special_ids = set()
        for t in self.spec.get("added_tokens", []):
            if t.get("special"):
                self.special_ids.add(t["id"])
        self.vocab_size = self._vocab_size()
        self.bos_id = self._tok_id(self.cfg.get("bos_token"))
        self.eos_id = self._tok_id(self.cfg.get("eos_token"))

    def _tok_id(self, t):
        if isinstance(t, dict):
            t = t.get("content")
        if not t:
            return None
        return self.token_to_id(t)

    def _vocab_size(self):
        if self.backend == "hf":
            return self.impl.get_vocab_size(with_added_tokens=True)
        return self.impl.vocab_size()

    def token_to_id(self, t):
        return self.impl.token_to_id(t)

    # Long single texts (a ~20 KB RAG prompt: 5 ms on one thread) are cut into pieces at pre-tokenizer
    # boundaries and encoded on the C++ worker threads. Exact for byte-level BPE without a normalizer:
    # a cut sits before a space that follows a non-space and precedes a letter, where the Llama-3 /
    # GPT-2 split regexes always end a pre-token (" word" starts one), and BPE merges never cross
    # pre-tokens. Only for tokenizers whose special tokens are a pure prefix (Llama-3: BOS).
    SPLIT_MIN_CHARS = int(os.environ.get("RAGK_TOKENIZER_SPLIT_CHARS", "4096"))

    def _split_ok(self):
        ok = getattr(self, "_split_ok_v", None)
        if ok is None:
            m = self.spec.get("model") or {}
            ok = (self.backend == "native" and hasattr(self.impl, "encode_batch") and m.get("type") == "BPE"
                  and not self.spec.get("normalizer"))
            if ok:
                probe = "Context: alpha beta, gamma 12 delta. Question: why?"
                pre = list(self.impl.encode("", True, -1))
                ok = list(self.impl.encode(probe, True, -1)) == pre + list(self.impl.encode(probe, False, -1))
                self._special_prefix = pre
            self._split_ok_v = ok
        return ok

    @staticmethod
    def _pieces(text, n):
        """`text` cut into about n pieces at split-safe boundaries (see SPLIT_MIN_CHARS)."""
        step = len(text) // n
        cuts, pos = [0], 0
        for _ in range(n - 1):
            i = max(pos + 1, cuts[-1] + step)
            while i < len(text) - 1 and not (text[i] == " " and not text[i - 1].isspace() and text[i + 1].isalpha()):
                i += 1
            if i >= len(text) - 1:
                break
            cuts.append(i)
            pos = i
        cuts.append(len(text))
        return [text[a:b] for a, b in zip(cuts[:-1], cuts[1:])]

    def _encode_split(self, text, add_special_tokens):
        pieces = self._pieces(text, max(2, min(ENCODE_THREADS, len(text) // 2048)))
        out = self.impl.encode_batch(pieces, False, ENCODE_THREADS, -1)
        ids = list(self._special_prefix) if add_special_tokens else []
        for x in out:
            ids.extend(x)
        return ids

    def _encode_batch_split(self, texts, add_special_tokens):
        """encode_batch of fewer texts than worker threads (C=1: one ~20 KB RAG prompt, ~6 ms on a single
        worker): every long text is cut as in encode() and all pieces go to the workers in one call, then
        each text is reassembled (special prefix + its pieces' ids in order) -- ~2 ms."""
        per = max(2, ENCODE_THREADS // len(texts))
        pieces, owner = [], []
        for ti, t in enumerate(texts):
            n = min(per, len(t) // 2048) if len(t) >= self.SPLIT_MIN_CHARS else 1
            ps = self._pieces(t, n) if n > 1 else [t]
            pieces.extend(ps)
            owner.extend([ti] * len(ps))
        enc = self.impl.encode_batch(pieces, False, ENCODE_THREADS, -1)
        out = [list(self._special_prefix) if add_special_tokens else [] for _ in texts]
        for ti, x in zip(owner, enc):
            out[ti].extend(x)
        return out

    def encode(self, text, add_special_tokens=True, max_length=None):
        if max_length is None and len(text) >= self.SPLIT_MIN_CHARS and self._split_ok():
            return self._encode_split(text, add_special_tokens)
        if self.backend == "hf":
            ids = self.impl.encode(text, add_special_tokens=add_special_tokens).ids
        else:  # native: stops tokenizing once max_length body tokens exist (same prefix, less work)
            ids = self.impl.encode(text, add_special_tokens, -1 if max_length is None else int(max_length))
        if max_length is not None and len(ids) > max_length:
            ids = self._truncate(ids, max_length, add_special_tokens)
        return list(ids)

    def _truncate(self, ids, max_length, add_special):
        """Right truncation that keeps the trailing special token (e.g. [SEP] / </s>)."""
        if add_special and ids and ids[-1] in self.special_ids:
            return ids[:max_length - 1] + [ids[-1]]
        return ids[:max_length]

    def encode_batch(self, texts, add_special_tokens=True, max_length=None):
        if self.backend == "hf":
            encs = self.impl.encode_batch(list(texts), add_special_tokens=add_special_tokens)
            out = [e.ids for e in encs]
        elif hasattr(self.impl, "encode_batch"):  # C++ worker threads, GIL released
            texts = list(texts)
            if (max_length is None and len(texts) < ENCODE_THREADS and self._split_ok()
                    and any(len(t) >= self.SPLIT_MIN_CHARS for t in texts)):
                return self._encode_batch_split(texts, add_special_tokens)
            out = self.impl.encode_batch(texts, add_special_tokens, ENCODE_THREADS,
                                         -1 if max_length is None else int(max_length))
        else:
            out = [self.impl.encode(t, add_special_tokens) for t in texts]
        if max_length is not None:
            out = [self._truncate(list(x), max_length, add_special_tokens) if len(x) > max_length else list(x)
                   for x in out]
        return out

    def encode_batch_flat(self, texts, add_special_tokens=True, max_length=None):
        """(ids int32 [sum of lengths], lens int32 [n]) numpy arrays: encode_batch + truncation, built in
        C++ on the native backend (the embedding engine's ingest path)."""
        if self.backend == "native" and hasattr(self.impl, "encode_batch_flat"):
            return self.impl.encode_batch_flat(list(texts), add_special_tokens, ENCODE_THREADS,
                                               -1 if max_length is None else int(max_length))
        out = self.encode_batch(texts, add_special_tokens, max_length)
        lens = np.fromiter((len(x) for x in out), dtype=np.int32, count=len(out))
        ids = np.fromiter((t for x in out for t in x), dtype=np.int32, count=int(lens.sum()))
        return ids, lens

    def decode(self, ids, skip_special_tokens=True):
        ids = [int(i) for i in ids if 0 <= int(i) < self.vocab_size]
        if self.backend == "hf":
            return self.impl.decode(ids, skip_special_tokens=skip_special_tokens)
        return self.impl.decode(ids, skip_special_tokens)
