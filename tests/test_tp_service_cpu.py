"""Tensor-parallel SERVICE on CPU (2 gloo ranks): the whole TP server path of parallel/tp.py --
rank 0 runs Flask + the engine loop + the control channel, rank 1 follows -- with data-parallel
ingest (every rank embeds a share of an upload's chunks, all-gathered) and, with INDEX_SHARDED, a
row-sharded index searched collectively. Reference surface: /upload_pdf, /index_info, /generate
(/root/reference/llm/rag.py:122-197)."""
import io
import os
import socket
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

WORLD = 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.fixture(scope="module")
def assets(tmp_path_factory):
    from rag_llm_k8s_amd.models import encoder as E
    from rag_llm_k8s_amd.models.llama import llama_tiny
    from rag_llm_k8s_amd.utils import synthetic as S

    root = tmp_path_factory.mktemp("models_tp")
    S.write_llama_checkpoint(str(root), llama_tiny(vocab=1024, layers=2, hidden=256, heads=4, kv_heads=2, inter=512),
                             seed=0, n_shards=2)
    ecfg = E.EncoderConfig(vocab_size=1024, hidden_size=128, num_hidden_layers=2, num_attention_heads=4,
                           intermediate_size=256, max_seq_length=128)
    S.write_encoder_checkpoint(str(root / "minilm"), ecfg, seed=0)
    pdfs = tmp_path_factory.mktemp("pdfs_tp")
    S.write_pdf_corpus(str(pdfs), 2, pages=2, words_per_page=700)
    return str(root), str(pdfs)


def _worker(rank, port, d, root, pdfs, sharded):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(WORLD),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(2)
    from rag_llm_k8s_amd.config import RagConfig
    from rag_llm_k8s_amd.ingest.pdf import write_pdf
    from rag_llm_k8s_amd.parallel.comm import TPComm
    from rag_llm_k8s_amd.parallel.dist import init_distributed
    from rag_llm_k8s_amd.parallel.tp import TPControl, follow, make_channel
    from rag_llm_k8s_amd.server.app import create_app
    from rag_llm_k8s_amd.server.builder import build_service

    ctx = init_distributed(tp=WORLD, backend="gloo")
    res = {}
    try:
        cfg = RagConfig(model_path=root, index_path=os.path.join(d, "faiss_index"), pdf_dir=pdfs,
                        embed_model=os.path.join(root, "minilm"), device="cpu", max_new_tokens=4, max_model_len=1024,
                        max_batch=4, use_cuda_graphs=False, kv_cache_blocks=64, seed=1, index_sharded=sharded,
                        retrieve_k=3, context_k=2)
        comm = TPComm(ctx.tp_group, ctx.tp, ctx.tp_rank, "cpu", ctx.tp_cpu_group)
        chan = make_channel(ctx.tp_cpu_group, ctx.tp_rank, ctx.tp)
        control = TPControl(ctx.tp_cpu_group, channel=chan) if rank == 0 else None
        svc = build_service(cfg, start_threads=(rank == 0), tp_rank=ctx.tp_rank, tp_size=ctx.tp, comm=comm,
                            tp_group=ctx.tp_group, control=control)
        if rank != 0:
            if svc.store.sharded:
                svc.store.ensure_exists()
            follow(svc.engine, ctx.tp_cpu_group, channel=chan, jobs=svc.job_fns())
        else:
            svc.store.ensure_exists()
            res["dir_files"] = svc.ingest_directory()
            svc.ready = True
            c = create_app(svc).test_client()
            words = " ".join("w%d" % i for i in range(1700))
            r = c.post("/upload_pdf", data={"file": (io.BytesIO(write_pdf([[words]])), "up.pdf")},
                       content_type="multipart/form-data")
            res["upload"] = (r.status_code, r.get_json())
            res["info"] = c.get("/index_info").get_json()
            g = c.post("/generate", json={"prompt": "what do the documents say about w17"})
            res["gen_status"] = g.status_code
            res["context"] = g.get_json().get("context")
            res["health"] = c.get("/healthz").status_code
            svc.shutdown()
            svc.loop.join(30)
        svc.store.flush()
        idx = svc.store.index
        local = idx.local if svc.store.sharded else idx
        res["local_rows"] = local.reconstruct_all()
        res["ntotal"] = int(idx.ntotal)
        res["meta"] = [(m["filename"], m["chunk_id"]) for m in svc.store.metadata]
        res["chunks"] = {(m["filename"], m["chunk_id"]): m["text"] for m in svc.store.metadata}
    finally:
        torch.save(res, os.path.join(d, "r%d.pt" % rank))
        dist.destroy_process_group()


def _run(root, pdfs, sharded):
    port = _free_port()
    d = tempfile.mkdtemp()
    mp.spawn(_worker, args=(port, d, root, pdfs, sharded), nprocs=WORLD, join=True)
    return [torch.load(os.path.join(d, "r%d.pt" % r), weights_only=False) for r in range(WORLD)], d


def _reference_embeddings(root, texts):
    from rag_llm_k8s_amd.server.builder import build_embedder
    from rag_llm_k8s_amd.config import RagConfig

    emb = build_embedder(RagConfig(embed_model=os.path.join(root, "minilm"), device="cpu"), "cpu")
    return emb.embed(texts).cpu()


@pytest.mark.parametrize("sharded", [False, True])
def test_tp_service_dp_ingest_and_sharded_index(assets, sharded):
    root, pdfs = assets
    out, d = _run(root, pdfs, sharded)
    r0, r1 = out
    assert r0["dir_files"] == 2
    assert r0["upload"][0] == 200 and "3 chunks created" in r0["upload"][1]["message"]
    assert r0["gen_status"] == 200 and r0["health"] == 200
    assert r0["context"].startswith("Document '")
    n = r0["ntotal"]
    assert r0["info"]["total_vectors"] == n == len(r0["meta"])
    # the data-parallel ingest produced exactly the single-process embeddings, in metadata order
    ref = _reference_embeddings(root, [r0["chunks"][k] for k in r0["meta"]])
    if not sharded:
        assert torch.allclose(torch.as_tensor(r0["local_rows"]), ref, atol=1e-5)
        assert len(r1["local_rows"]) == 0  # replicated mode: only rank 0 retrieves, so only rank 0 indexes
    else:
        assert r1["ntotal"] == n and r1["meta"] == r0["meta"]
        got = torch.empty_like(ref)
        got[0::2] = torch.as_tensor(r0["local_rows"])
        got[1::2] = torch.as_tensor(r1["local_rows"])
        assert torch.allclose(got, ref, atol=1e-5)
        for r in range(WORLD):  # each rank persisted its shard as a faiss file
            assert os.path.exists(os.path.join(d, "faiss_index.shard%dof2" % r))
    test_tp_service_dp_ingest_and_sharded_index.contexts[sharded] = r0["context"]
    if len(test_tp_service_dp_ingest_and_sharded_index.contexts) == 2:  # same retrieval either way
        c = test_tp_service_dp_ingest_and_sharded_index.contexts
        assert c[True] == c[False]


test_tp_service_dp_ingest_and_sharded_index.contexts = {}


def _abort_worker(rank, port, d, root, pdfs):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(WORLD),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(2)
    import time

    from rag_llm_k8s_amd.config import RagConfig
    from rag_llm_k8s_amd.parallel.comm import TPComm
    from rag_llm_k8s_amd.parallel.dist import init_distributed
    from rag_llm_k8s_amd.parallel.tp import TPControl, follow, make_channel
    from rag_llm_k8s_amd.server.app import create_app
    from rag_llm_k8s_amd.server.builder import build_service
    from rag_llm_k8s_amd.utils import faults

    ctx = init_distributed(tp=WORLD, backend="gloo")
    res = {}
    try:
        cfg = RagConfig(model_path=root, index_path=os.path.join(d, "faiss_index"), pdf_dir=pdfs,
                        embed_model=os.path.join(root, "minilm"), device="cpu", max_new_tokens=300, max_model_len=1024,
                        max_batch=4, use_cuda_graphs=False, kv_cache_blocks=64, seed=1, retrieve_k=3, context_k=2,
                        request_timeout_s=0.5, ignore_eos=True)
        comm = TPComm(ctx.tp_group, ctx.tp, ctx.tp_rank, "cpu", ctx.tp_cpu_group)
        chan = make_channel(ctx.tp_cpu_group, ctx.tp_rank, ctx.tp)
        control = TPControl(ctx.tp_cpu_group, channel=chan) if rank == 0 else None
        svc = build_service(cfg, start_threads=(rank == 0), tp_rank=ctx.tp_rank, tp_size=ctx.tp, comm=comm,
                            tp_group=ctx.tp_group, control=control)
        free0 = svc.engine.bm.free_blocks()
        if rank != 0:
            follow(svc.engine, ctx.tp_cpu_group, channel=chan, jobs=svc.job_fns())
        else:
            svc.store.ensure_exists()
            svc.ingest_directory()
            svc.ready = True
            c = create_app(svc).test_client()
            faults.set_faults("step_delay_ms=50")
            r = c.post("/generate", json={"prompt": "what do the documents say about w17"})
            res["status"], res["body"] = r.status_code, r.get_json()
            # steps stay slow: running the sequence out (300 x 50 ms) would miss this deadline
            deadline = time.time() + 8
            while time.time() < deadline and (svc.engine.has_work() or svc.engine.bm.free_blocks() != free0):
                time.sleep(0.05)
            faults.set_faults("")
            res["health"] = c.get("/healthz").status_code
            from rag_llm_k8s_amd.engine.llm_engine import SamplingParams

            # the server still serves after the abort
            out = svc.generate("w3", params=SamplingParams(max_new_tokens=2, ignore_eos=True))
            res["after"] = 200 if "generated_text" in out else 500
            svc.shutdown()
            svc.loop.join(30)
        res["free"] = (svc.engine.bm.free_blocks(), free0)
        res["has_work"] = svc.engine.has_work()
        res["decode_tokens"] = svc.engine.stats["decode_tokens"]
    finally:
        torch.save(res, os.path.join(d, "a%d.pt" % rank))
        dist.destroy_process_group()


def test_tp_request_timeout_aborts_on_every_rank(assets):
    """A timed-out TP request is aborted on every rank at the same step boundary (control-channel
    abort record) and both ranks' KV block managers return to full."""
    root, pdfs = assets
    port = _free_port()
    d = tempfile.mkdtemp()
    mp.spawn(_abort_worker, args=(port, d, root, pdfs), nprocs=WORLD, join=True)
    r0, r1 = [torch.load(os.path.join(d, "a%d.pt" % r), weights_only=False) for r in range(WORLD)]
    assert r0["status"] == 500 and "timed out" in r0["body"]["error"]
    assert r0["health"] == 200 and r0["after"] == 200
    for r in (r0, r1):
        assert r["free"][0] == r["free"][1] and not r["has_work"]
        assert r["decode_tokens"] < 150  # aborted, not run out to max_new_tokens
