"""Assemble a RagService from a RagConfig (the reference's module-scope init, rag.py:13-33,199-204).

Model directory = the reference's /models PVC layout (download_model.py file list). The
generator architecture is read from config.json (llama or gpt2); the embedder from
EMBED_MODEL (a local sentence-transformers directory: the reference fetched BAAI/bge-m3
from the network at startup, /root/reference/llm/rag.py:33, which is dropped here).
"""
from __future__ import annotations

import json
import logging
import os

import torch

log = logging.getLogger(__name__)


def _load_json(p, default=None):
    if os.path.exists(p):
        with open(p) as f:
            return json.load(f)
    return default


def kv_blocks_for(model, cfg, device):
    if cfg.kv_cache_blocks > 0:
        return cfg.kv_cache_blocks
    per = model.kv_bytes_per_block()
    if torch.device(device).type == "cuda":
        free, _ = torch.cuda.mem_get_info(torch.device(device))
        budget = int(free * cfg.kv_cache_fraction)
    else:
        budget = 2 << 30
    need = cfg.max_batch * (-(-cfg.max_model_len // 64)) + 8
    return max(16, min(need, budget // per))


def build_generator(cfg, device, tp_rank=0, tp_size=1, comm=None, tp_group=None):
    from ..engine.llm_engine import LLMEngine
    from ..runtime.tokenizer import Tokenizer

    mcfg = _load_json(os.path.join(cfg.model_path, "config.json"))
    if mcfg is None:
        raise FileNotFoundError("no config.json under MODEL_PATH=%s" % cfg.model_path)
    gen = _load_json(os.path.join(cfg.model_path, "generation_config.json"), {})
    tok = Tokenizer(cfg.model_path)
    mt = mcfg.get("model_type", "llama")
    if mt == "gpt2":
        from ..models.gpt2 import GPT2Config, GPT2Model, GPT2Weights

        c = GPT2Config.from_dict(mcfg)
        w = GPT2Weights.from_checkpoint(cfg.model_path, c, device)
        model = GPT2Model(c, w, device)
        max_len = min(cfg.max_model_len, c.n_positions)
        eos = [c.eos_token_id]
    else:
        from ..models.llama import LlamaConfig, LlamaModel, LlamaWeights

        c = LlamaConfig.from_dict(mcfg)
        w = LlamaWeights.from_checkpoint(cfg.model_path, c, device, tp_rank, tp_size)
        if cfg.dtype == "fp8":  # DTYPE=fp8: e4m3fn linear weights, per-row scales (BASELINE config 5)
            w.quantize_fp8()
        max_len = min(cfg.max_model_len, c.max_position_embeddings)
        model = LlamaModel(c, w, device, comm=comm, max_positions=max_len)
        eos = c.eos_token_id
    geos = gen.get("eos_token_id", eos)
    eos = geos if isinstance(geos, list) else [geos]
    cfg.max_model_len = max_len
    blocks = kv_blocks_for(model, cfg, device)
    engine = LLMEngine(model, num_blocks=blocks, max_batch=cfg.max_batch, max_prefill_tokens=cfg.max_prefill_tokens,
                       max_model_len=max_len, eos_ids=eos, use_graphs=cfg.use_cuda_graphs, tp_group=tp_group,
                       mixed_prefill_tokens=cfg.mixed_prefill_tokens)
    return engine, tok, gen


def build_embedder(cfg, device):
    from ..engine.encoder_engine import EmbeddingEngine
    from ..models.encoder import EncoderConfig, EncoderModel, EncoderWeights
    from ..runtime.tokenizer import Tokenizer

    path = cfg.embed_model
    if not os.path.isdir(path):
        raise FileNotFoundError("EMBED_MODEL=%s is not a local sentence-transformers directory (the framework "
                                "never downloads at startup; see llm/download_model.py --embedder)" % path)
    ec = EncoderConfig.from_dir(path)
    ec.max_seq_length = min(ec.max_seq_length, cfg.max_embed_len)
    w = EncoderWeights.from_dir(ec, path, device)
    return EmbeddingEngine(EncoderModel(ec, w, device), Tokenizer(path), max_batch_tokens=cfg.embed_batch_tokens)


def build_service(cfg, start_threads=True, tp_rank=0, tp_size=1, comm=None, tp_group=None, control=None):
    from ..index.store import DocumentStore
    from .rag_service import RagService

    device = cfg.resolved_device()
    if device.startswith("cuda"):
        device = "cuda:%d" % torch.cuda.current_device() if device == "cuda" else device
    log.info("Loading model from: %s (device %s, tp %d/%d)", cfg.model_path, device, tp_rank, tp_size)
    engine, tok, gen = build_generator(cfg, device, tp_rank, tp_size, comm, tp_group)
    log.info("Model and tokenizer loaded successfully")
    embedder = build_embedder(cfg, device)
    shard = None
    if cfg.index_sharded and tp_size > 1:
        shard = (tp_group, tp_rank, tp_size)  # INDEX_SHARDED=1: row shard per TP rank (parallel/dp.py)
    store = DocumentStore(cfg.index_path, embedder.dim, device=device, index_type=cfg.index_type,
                          ivf_nlist=cfg.ivf_nlist, ivf_nprobe=cfg.ivf_nprobe, recovery=cfg.index_recovery,
                          shard=shard)
    svc = RagService(cfg, engine, tok, embedder, store, gen_config=gen, start_threads=start_threads, control=control,
                     tp_group=tp_group if tp_size > 1 else None)
    return svc
