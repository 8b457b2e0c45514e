"""Failure detection / recovery / fault injection, CPU plumbing config.

Each test switches on one hook of rag_llm_k8s_amd/utils/faults.py (or damages files directly) and
checks the recovery path: torn/corrupt index -> quarantined and rebuilt from PDF_DIR; missing
checkpoint shard -> fail fast naming the shard; engine failure -> 500 + liveness 503; slow engine
-> request timeout that aborts the sequence and frees its KV blocks; hung step -> watchdog.
"""
import os
import time

import pytest
import torch

from rag_llm_k8s_amd.config import RagConfig
from rag_llm_k8s_amd.models import encoder as E
from rag_llm_k8s_amd.models import gpt2 as G2
from rag_llm_k8s_amd.utils import faults
from rag_llm_k8s_amd.utils import synthetic as S


@pytest.fixture(scope="module")
def assets(tmp_path_factory):
    root = tmp_path_factory.mktemp("models")
    G2.write_gpt2_checkpoint(str(root), G2.gpt2_tiny(1024), seed=0)
    ecfg = E.EncoderConfig(vocab_size=1024, hidden_size=128, num_hidden_layers=2, num_attention_heads=4,
                           intermediate_size=256, max_seq_length=128)
    S.write_encoder_checkpoint(str(root / "minilm"), ecfg, seed=0)
    pdfs = tmp_path_factory.mktemp("pdfs")
    S.write_pdf_corpus(str(pdfs), 2, pages=1, words_per_page=900)
    return root, pdfs


@pytest.fixture(autouse=True)
def _clear_faults():
    faults.set_faults("")
    yield
    faults.set_faults(None)


def cfg_for(assets, idx_dir, **kw):
    root, pdfs = assets
    base = dict(model_path=str(root), index_path=str(idx_dir / "faiss_index"), pdf_dir=str(pdfs),
                embed_model=str(root / "minilm"), device="cpu", max_new_tokens=6, max_model_len=1024, max_batch=4,
                use_cuda_graphs=False, kv_cache_blocks=64, seed=1, watchdog_exit=False)
    base.update(kw)
    return RagConfig(**base)


def service(cfg, start_threads=True):
    from rag_llm_k8s_amd.server.builder import build_service

    svc = build_service(cfg, start_threads=start_threads)
    svc.store.ensure_exists()
    return svc


def test_corrupt_index_is_quarantined_and_rebuilt(assets, tmp_path):
    svc = service(cfg_for(assets, tmp_path), start_threads=False)
    svc.ingest_directory()
    n = svc.store.index.ntotal
    assert n > 0
    p = str(tmp_path / "faiss_index")
    with open(p, "r+b") as f:  # torn write: the reference would crash-loop on this file
        f.truncate(60)
    svc2 = service(cfg_for(assets, tmp_path), start_threads=False)
    assert svc2.store.recovered and svc2.store.index.ntotal == 0
    assert any(x.startswith("faiss_index.corrupt-") for x in os.listdir(tmp_path))
    svc2.ingest_directory()  # startup ingest rebuilds it
    assert svc2.store.index.ntotal == n
    svc3 = service(cfg_for(assets, tmp_path), start_threads=False)
    assert svc3.store.recovered is None and svc3.store.index.ntotal == n


def test_index_metadata_mismatch_and_fail_policy(assets, tmp_path):
    from rag_llm_k8s_amd.index.faiss_io import load_metadata, save_metadata

    svc = service(cfg_for(assets, tmp_path), start_threads=False)
    svc.ingest_directory()
    meta = load_metadata(str(tmp_path / "faiss_index.metadata"))
    save_metadata(str(tmp_path / "faiss_index.metadata"), meta[:-1])
    with pytest.raises(ValueError, match="metadata"):
        service(cfg_for(assets, tmp_path, index_recovery="fail"), start_threads=False)
    faults.set_faults("index_read_error")
    with pytest.raises(faults.FaultInjected):
        service(cfg_for(assets, tmp_path, index_recovery="fail"), start_threads=False)
    s = service(cfg_for(assets, tmp_path), start_threads=False)
    assert s.store.recovered


def test_unreadable_snapshot_keeps_resident_index(assets, tmp_path):
    svc = service(cfg_for(assets, tmp_path), start_threads=False)
    svc.ingest_directory()
    n = svc.store.index.ntotal
    p = str(tmp_path / "faiss_index")
    time.sleep(0.02)
    with open(p, "wb") as f:
        f.write(b"IxF2garbage")
    os.utime(p, (time.time() + 5, time.time() + 5))
    svc.store.maybe_reload()
    assert svc.store.index.ntotal == n
    q = svc.embedder.embed(["hello"])
    assert len(svc.store.search(q, 3)[0]) == 3


def test_missing_shard_fails_fast(tmp_path):
    from rag_llm_k8s_amd.runtime.safetensors_io import CheckpointReader, save_sharded

    t = {"a.weight": torch.randn(4, 4), "b.weight": torch.randn(4, 4), "c.weight": torch.randn(2)}
    save_sharded(t, str(tmp_path), 3)
    CheckpointReader(str(tmp_path)).close()
    faults.set_faults("missing_shard=2")
    with pytest.raises(FileNotFoundError, match="model-00002-of-00003"):
        CheckpointReader(str(tmp_path))
    faults.set_faults("")
    os.remove(str(tmp_path / "model-00003-of-00003.safetensors"))
    with pytest.raises(FileNotFoundError, match="missing shard"):
        CheckpointReader(str(tmp_path))


def test_engine_failure_surfaces_as_500_and_liveness_503(assets, tmp_path):
    from rag_llm_k8s_amd.server.app import create_app

    svc = service(cfg_for(assets, tmp_path))
    svc.ingest_directory()
    svc.ready = True
    c = create_app(svc).test_client()
    try:
        assert c.get("/healthz").status_code == 200
        faults.set_faults("engine_crash_at_step=1")
        r = c.post("/generate", json={"prompt": "hello"})
        assert r.status_code == 500 and "engine" in r.get_json()["error"]
        assert c.get("/healthz").status_code == 503
        assert c.get("/readyz").status_code == 503
    finally:
        svc.shutdown()


def test_request_timeout_aborts_and_frees_blocks(assets, tmp_path):
    from rag_llm_k8s_amd.server.app import create_app

    svc = service(cfg_for(assets, tmp_path, max_new_tokens=200, request_timeout_s=0.3))
    svc.ingest_directory()
    c = create_app(svc).test_client()
    free0 = svc.engine.bm.free_blocks()
    try:
        faults.set_faults("step_delay_ms=100")
        r = c.post("/generate", json={"prompt": "hello"})
        assert r.status_code == 500 and "timed out" in r.get_json()["error"]
        faults.set_faults("")
        deadline = time.time() + 10
        while time.time() < deadline and (svc.engine.has_work() or svc.engine.bm.free_blocks() != free0):
            time.sleep(0.05)
        assert not svc.engine.has_work() and svc.engine.bm.free_blocks() == free0
        assert c.get("/healthz").status_code == 200  # a timeout is not an engine failure
    finally:
        svc.shutdown()


def test_embed_error_is_500(assets, tmp_path):
    from rag_llm_k8s_amd.server.app import create_app

    svc = service(cfg_for(assets, tmp_path))
    c = create_app(svc).test_client()
    try:
        faults.set_faults("embed_error")
        r = c.post("/generate", json={"prompt": "hello"})
        assert r.status_code == 500 and "embed_error" in r.get_json()["error"]
        faults.set_faults("")
        assert c.get("/healthz").status_code == 200
    finally:
        svc.shutdown()


def test_watchdog_declares_hung_step(assets, tmp_path):
    from rag_llm_k8s_amd.server.rag_service import Watchdog

    class Loop:
        step_started = None

    lp = Loop()
    wd = Watchdog(lp, step_timeout_s=5.0, exit_on_hang=False)
    assert not wd.check()
    lp.step_started = time.monotonic() - 2
    assert not wd.check()
    lp.step_started = time.monotonic() - 6
    assert wd.check()


def test_fault_spec_parsing(monkeypatch):
    faults.set_faults(None)
    monkeypatch.setenv("RAGK_FAULTS", "step_delay_ms=5, embed_error ,missing_shard=3")
    assert faults.faults() == {"step_delay_ms": "5", "embed_error": "1", "missing_shard": "3"}
    assert faults.active("embed_error") and faults.value("missing_shard") == "3"
    monkeypatch.setenv("RAGK_FAULTS", "")
    assert faults.faults() == {}


def test_peer_wait_error_record_decodes():
    """The comm watchdog's error word (csrc/comm/allreduce.hip ar_record) names the collective, the peer
    that never arrived, the block / row slot and the call index; CommError carries the decoded text."""
    from rag_llm_k8s_amd.parallel.ipc_allreduce import describe_error

    rec = 1 | 4 << 1 | 6 << 4 | 3 << 7 | 1234 << 15
    assert describe_error(rec) == ("fused reduce+norm row (start barrier), block/row 3, call 1234 (mod 65536): "
                                   "peer rank 6 never arrived")
    assert describe_error(1 | 1 << 1 | 1 << 4 | 1 << 15).startswith("all-reduce (start barrier), block/row 0, call 1")
    assert describe_error(0) == "no error"
    assert rec < 2 ** 31  # ragk_ar_error returns it as a non-negative int
