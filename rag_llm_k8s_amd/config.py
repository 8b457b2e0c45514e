"""Runtime configuration: one dataclass, reference values as defaults, env overrides.

Reference knobs (all hard-coded there except MODEL_PATH):
  MODEL_PATH env (default /models)          /root/reference/llm/rag.py:18, llm/dockerfile_rag:25
  INDEX_PATH "/models/faiss_index"          /root/reference/llm/rag.py:19 (ignores MODEL_PATH)
  PDF_DIR "/pdfs"                           /root/reference/llm/rag.py:20
  chunk 1000 words / 200 overlap            /root/reference/llm/rag.py:39
  retrieve k=5, top-3 into the prompt       /root/reference/llm/rag.py:114,164
  max_new_tokens=150, T=0.7, top_p=0.9      /root/reference/llm/rag.py:172 (top_k=50 GenerationConfig default)
  port 5001                                 /root/reference/llm/rag.py:204
"""
from __future__ import annotations

import dataclasses
import os
from dataclasses import dataclass, field
from typing import Optional


def _env(name, default, cast=str):
    v = os.environ.get(name)
    if v is None or v == "":
        return default
    if cast is bool:
        return v.strip().lower() in ("1", "true", "yes", "on")
    return cast(v)


@dataclass
class RagConfig:
    model_path: str = "/models"
    index_path: str = "/models/faiss_index"
    pdf_dir: str = "/pdfs"
    embed_model: str = "/models/bge-m3"
    host: str = "0.0.0.0"
    port: int = 5001
    retrieve_k: int = 5
    context_k: int = 3
    chunk_words: int = 1000
    chunk_overlap: int = 200
    max_new_tokens: int = 150
    temperature: float = 0.7
    top_p: float = 0.9
    top_k: int = 50
    do_sample: Optional[bool] = None  # None -> generation_config.json (reference: model.generate defaults)
    seed: int = 0
    tp_size: int = 1
    dtype: str = "bf16"
    device: str = "auto"  # auto | cuda | cpu
    index_type: str = "flat"  # flat | ivf
    ivf_nlist: int = 1024
    ivf_nprobe: int = 32
    reingest_append: bool = False  # True reproduces the reference's duplicate-on-restart ingest
    max_batch: int = 64  # concurrent sequences in one decode step
    max_model_len: int = 16384
    max_prefill_tokens: int = 32768  # tokens per prefill step (chunked prefill budget)
    # prompt tokens per step while sequences are decoding (decode-aware cap; 0 = off). Off by default:
    # at Poisson 8 req/s caps of 2048 / 1024 / 512 made TPOT p50 15-27 ms and TTFT p50 0.2-10 s against
    # 10.6 ms / 82 ms uncapped -- every small chunk re-reads the weights (profiles/serve_r5b.json)
    mixed_prefill_tokens: int = 0
    kv_cache_fraction: float = 0.80  # of free HBM after weights
    kv_cache_blocks: int = 0  # explicit override (64-token blocks)
    embed_batch_tokens: int = 65536
    max_embed_len: int = 8192
    use_cuda_graphs: bool = True
    log_level: str = "INFO"
    truncate_prompt: str = "left"  # left | none (GPT-2 has 1024 positions; the reference prompt is ~4.3k tokens)
    request_timeout_s: float = 600.0  # /generate waits at most this long, then aborts the sequence -> 500
    step_timeout_s: float = 300.0  # watchdog: an engine step (incl. its collectives) longer than this = hung
    watchdog_exit: bool = True  # hung engine -> dump stacks and exit so k8s restarts the pod
    index_recovery: str = "rebuild"  # rebuild (quarantine unreadable index, re-ingest PDF_DIR) | fail
    ignore_eos: bool = False  # benchmarks only: every request generates exactly max_new_tokens
    index_sharded: bool = False  # TP server: each rank keeps a row shard of the index, search is collective
    extra: dict = field(default_factory=dict)

    @classmethod
    def from_env(cls, **overrides) -> "RagConfig":
        c = cls()
        m = {
            "MODEL_PATH": ("model_path", str), "INDEX_PATH": ("index_path", str), "PDF_DIR": ("pdf_dir", str),
            "EMBED_MODEL": ("embed_model", str), "HOST": ("host", str), "PORT": ("port", int),
            "RETRIEVE_K": ("retrieve_k", int), "CONTEXT_K": ("context_k", int), "CHUNK_WORDS": ("chunk_words", int),
            "CHUNK_OVERLAP": ("chunk_overlap", int), "MAX_NEW_TOKENS": ("max_new_tokens", int),
            "TEMPERATURE": ("temperature", float), "TOP_P": ("top_p", float), "TOP_K": ("top_k", int),
            "SEED": ("seed", int), "TP_SIZE": ("tp_size", int), "DTYPE": ("dtype", str), "DEVICE": ("device", str),
            "INDEX_TYPE": ("index_type", str), "IVF_NLIST": ("ivf_nlist", int), "IVF_NPROBE": ("ivf_nprobe", int),
            "REINGEST_APPEND": ("reingest_append", bool), "MAX_BATCH": ("max_batch", int),
            "MAX_MODEL_LEN": ("max_model_len", int), "MAX_PREFILL_TOKENS": ("max_prefill_tokens", int),
            "MIXED_PREFILL_TOKENS": ("mixed_prefill_tokens", int),
            "KV_CACHE_FRACTION": ("kv_cache_fraction", float), "KV_CACHE_BLOCKS": ("kv_cache_blocks", int),
            "USE_CUDA_GRAPHS": ("use_cuda_graphs", bool), "LOG_LEVEL": ("log_level", str),
            "TRUNCATE_PROMPT": ("truncate_prompt", str), "REQUEST_TIMEOUT_S": ("request_timeout_s", float),
            "STEP_TIMEOUT_S": ("step_timeout_s", float), "WATCHDOG_EXIT": ("watchdog_exit", bool),
            "INDEX_RECOVERY": ("index_recovery", str), "IGNORE_EOS": ("ignore_eos", bool),
            "INDEX_SHARDED": ("index_sharded", bool),
        }
        for env, (attr, cast) in m.items():
            setattr(c, attr, _env(env, getattr(c, attr), cast))
        ds = os.environ.get("DO_SAMPLE")
        if ds:
            c.do_sample = ds.strip().lower() in ("1", "true", "yes")
        for k, v in overrides.items():
            if not hasattr(c, k):
                raise AttributeError("unknown config key %s" % k)
            setattr(c, k, v)
        return c

    def resolved_device(self) -> str:
        if self.device != "auto":
            return self.device
        import torch

        return "cuda" if torch.cuda.is_available() else "cpu"

    def replace(self, **kw) -> "RagConfig":
        return dataclasses.replace(self, **kw)
