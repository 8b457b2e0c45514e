"""T3' distributed tier on CPU: 2-process gloo groups exercising the same code paths the GPUs
use over RCCL (TP sharded Llama, TP request broadcast, DP embedding all-gather, sharded index)."""
import os
import socket
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from rag_llm_k8s_amd.models.llama import llama_tiny
from rag_llm_k8s_amd.utils.synthetic import llama_state_dict

WORLD = 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(fn, *args):
    port = _free_port()
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_entry, args=(fn, port, d, args), nprocs=WORLD, join=True)
        out = {}
        for r in range(WORLD):
            p = os.path.join(d, "r%d.pt" % r)
            if os.path.exists(p):
                out[r] = torch.load(p, weights_only=False)
        return out


def _entry(rank, fn, port, d, args):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(WORLD),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(2)
    from rag_llm_k8s_amd.parallel.dist import init_distributed

    ctx = init_distributed(tp=args[0] if args else 1, backend="gloo")
    try:
        res = fn(ctx, *args[1:])
        torch.save(res, os.path.join(d, "r%d.pt" % rank))
    finally:
        dist.destroy_process_group()


CFG = llama_tiny(vocab=320, layers=2, hidden=256, heads=4, kv_heads=2, inter=512)


def _prefill_logits(model, ids):
    from rag_llm_k8s_amd.models.llama import StepInput
    from rag_llm_k8s_amd.ops.backend import AttnMeta

    n = len(ids)
    model.allocate_kv_cache(8)
    slots = torch.arange(64, 64 + n, dtype=torch.int32)
    bt = torch.tensor([[1, 2, 3, 4]], dtype=torch.int32)
    meta = AttnMeta("prefill", torch.tensor([n], dtype=torch.int32), bt, cu_q=torch.tensor([0, n], dtype=torch.int32),
                    host_kv_lens=[n])
    return model.forward(StepInput(torch.tensor(ids, dtype=torch.int32), torch.arange(n, dtype=torch.int32), slots,
                                   meta, torch.tensor([n - 1], dtype=torch.int32)))


def _tp_worker(ctx, sd, ids):
    from rag_llm_k8s_amd.models.llama import LlamaModel, LlamaWeights
    from rag_llm_k8s_amd.parallel.comm import TPComm

    w = LlamaWeights.from_state_dict(CFG, sd, "cpu", ctx.tp_rank, ctx.tp)
    comm = TPComm(ctx.tp_group, ctx.tp, ctx.tp_rank, "cpu")
    m = LlamaModel(CFG, w, "cpu", comm=comm, max_positions=512)
    local = _prefill_logits(m, ids)  # vocab shard
    parts = [torch.empty_like(local) for _ in range(ctx.tp)]
    dist.all_gather(parts, local, group=ctx.tp_group)
    return torch.cat(parts, 1)[:, :CFG.vocab_size]


def test_tp2_logits_match_tp1():
    from rag_llm_k8s_amd.models.llama import LlamaModel, LlamaWeights

    sd = llama_state_dict(CFG, seed=4, std=0.05)
    ids = torch.randint(3, CFG.vocab_size, (40,), generator=torch.Generator().manual_seed(40)).tolist()
    ref = _prefill_logits(LlamaModel(CFG, LlamaWeights.from_state_dict(CFG, sd, "cpu"), "cpu", max_positions=512), ids)
    out = _run(_tp_worker, 2, sd, ids)
    for r in range(WORLD):
        rel = ((out[r] - ref).norm() / ref.norm()).item()
        assert rel < 2e-2, rel
    assert torch.equal(out[0], out[1])


def _tp_sp_worker(ctx, sd, ids):
    """TP=2 prefill logits with Megatron sequence parallelism vs the all-reduce path."""
    from rag_llm_k8s_amd.models.llama import LlamaModel, LlamaWeights
    from rag_llm_k8s_amd.parallel.comm import TPComm

    w = LlamaWeights.from_state_dict(CFG, sd, "cpu", ctx.tp_rank, ctx.tp)
    m = LlamaModel(CFG, w, "cpu", comm=TPComm(ctx.tp_group, ctx.tp, ctx.tp_rank, "cpu"), max_positions=512)
    out = {}
    for sp in (False, True):
        m.seq_parallel, m.sp_min_tokens = sp, 1
        local = _prefill_logits(m, ids)
        parts = [torch.empty_like(local) for _ in range(ctx.tp)]
        dist.all_gather(parts, local, group=ctx.tp_group)
        out[sp] = torch.cat(parts, 1)[:, :CFG.vocab_size]
    return out


@pytest.mark.parametrize("n", [40, 41])  # 41: token count not divisible by TP (padded rows)
def test_tp2_sequence_parallel_matches_allreduce_path(n):
    from rag_llm_k8s_amd.models.llama import LlamaModel, LlamaWeights

    sd = llama_state_dict(CFG, seed=8, std=0.05)
    ids = torch.randint(3, CFG.vocab_size, (n,), generator=torch.Generator().manual_seed(n)).tolist()
    ref = _prefill_logits(LlamaModel(CFG, LlamaWeights.from_state_dict(CFG, sd, "cpu"), "cpu", max_positions=512), ids)
    out = _run(_tp_sp_worker, 2, sd, ids)
    for r in range(WORLD):
        for sp in (False, True):
            rel = ((out[r][sp] - ref).norm() / ref.norm()).item()
            assert rel < 2e-2, (sp, rel)
        # bf16 activations, different reduction order (reduce-scatter + all-gather vs all-reduce).
        # Measured with these seeded ids: 7.9e-3 (n=40) and 9.1e-3 (n=41); bound ~1.5x that.
        rel = ((out[r][True] - out[r][False]).norm() / out[r][False].norm()).item()
        assert rel < 1.4e-2, rel
    assert torch.equal(out[0][True], out[1][True])


def _tp_control_worker(ctx, sd, prompts):
    import threading

    from rag_llm_k8s_amd.engine.llm_engine import LLMEngine, SamplingParams
    from rag_llm_k8s_amd.models.llama import LlamaModel, LlamaWeights
    from rag_llm_k8s_amd.parallel.comm import TPComm
    from rag_llm_k8s_amd.parallel.tp import TPControl, follow
    from rag_llm_k8s_amd.server.rag_service import EngineLoop

    w = LlamaWeights.from_state_dict(CFG, sd, "cpu", ctx.tp_rank, ctx.tp)
    m = LlamaModel(CFG, w, "cpu", comm=TPComm(ctx.tp_group, ctx.tp, ctx.tp_rank, "cpu"), max_positions=512)
    eng = LLMEngine(m, num_blocks=32, max_batch=4, max_model_len=512, use_graphs=False, tp_group=ctx.tp_group)
    p = SamplingParams(max_new_tokens=5, temperature=0.8, top_p=0.9, top_k=20, ignore_eos=True)
    if ctx.rank == 0:
        loop = EngineLoop(eng, control=TPControl(ctx.tp_cpu_group))
        loop.start()
        seqs = [loop.submit(pr, p, seed=i + 7) for i, pr in enumerate(prompts)]
        for s in seqs:
            s.done.wait(60)
        loop.stop()
        loop.join(30)
        return [s.out for s in seqs]
    follow(eng, ctx.tp_cpu_group)
    return "followed"


def test_tp_control_broadcast_keeps_ranks_in_lockstep():
    sd = llama_state_dict(CFG, seed=5, std=0.05)
    prompts = [[5, 6, 7, 8, 9], list(range(10, 60)), [100, 101]]
    out = _run(_tp_control_worker, 2, sd, prompts)
    assert out[1] == "followed"
    assert [len(o) for o in out[0]] == [5, 5, 5]


def _tp_overlap_worker(ctx, sd, prompts):
    """TP=2 engine: prefill as 2 micro-batches with async all-reduces vs the synchronous path."""
    from rag_llm_k8s_amd.engine.llm_engine import LLMEngine, SamplingParams
    from rag_llm_k8s_amd.models.llama import LlamaModel, LlamaWeights
    from rag_llm_k8s_amd.parallel.comm import TPComm

    outs = {}
    for thr in (10 ** 9, 8, "sp"):  # never / always micro-batch (8 tokens min) / sequence parallel
        w = LlamaWeights.from_state_dict(CFG, sd, "cpu", ctx.tp_rank, ctx.tp)
        m = LlamaModel(CFG, w, "cpu", comm=TPComm(ctx.tp_group, ctx.tp, ctx.tp_rank, "cpu"), max_positions=512)
        m.seq_parallel, m.sp_min_tokens = thr == "sp", 8
        eng = LLMEngine(m, num_blocks=32, max_batch=4, max_prefill_tokens=96, max_model_len=512, use_graphs=False,
                        tp_group=ctx.tp_group)
        eng.tp_overlap_min_tokens = 8 if thr == "sp" else thr
        # a mixed step computes decode rows through the prefill path, whose SP reduce-scatter sums in
        # another order than the decode all-reduce: a near-tie may flip; off so the test compares the
        # prefill schedules alone (mixed steps: tests/test_llama_cpu.py)
        eng.mixed_steps = False
        p = SamplingParams(max_new_tokens=4, do_sample=False, ignore_eos=True)
        outs[thr] = eng.generate(prompts, p)
    return outs


def test_tp_prefill_microbatch_overlap_matches_sync():
    sd = llama_state_dict(CFG, seed=6, std=0.05)
    # 3 prompts, 96-token prefill budget: chunks get cut across micro-batches and steps
    prompts = [list(range(3, 73)), list(range(100, 141)), [7, 8, 9, 10, 11]]
    out = _run(_tp_overlap_worker, 2, sd, prompts)
    for r in range(WORLD):
        assert out[r][8] == out[r][10 ** 9], out[r]
        assert out[r]["sp"] == out[r][10 ** 9], out[r]
    assert out[0] == out[1]


def test_split_chunks_cuts_token_stream_evenly():
    from rag_llm_k8s_amd.engine.llm_engine import LLMEngine

    a, b, c = object(), object(), object()
    parts = LLMEngine._split_chunks([(a, 0, 70), (b, 10, 41), (c, 0, 5)], 2)
    assert [sum(n for _, _, n in g) for g in parts] == [58, 58]
    assert parts[0] == [(a, 0, 58)] and parts[1] == [(a, 58, 12), (b, 10, 41), (c, 0, 5)]


def _dp_worker(ctx, texts):
    from rag_llm_k8s_amd.engine.encoder_engine import EmbeddingEngine
    from rag_llm_k8s_amd.models import encoder as E
    from rag_llm_k8s_amd.parallel.dp import ShardedFlatIndex, embed_distributed
    from rag_llm_k8s_amd.utils.synthetic import encoder_state_dict

    class Tok:  # deterministic toy tokenizer
        def encode_batch(self, ts, add_special_tokens=True, max_length=None):
            return [[(ord(c) * 7 + i) % 500 for i, c in enumerate(t[:60])] or [1] for t in ts]

    cfg = E.EncoderConfig(vocab_size=500, hidden_size=128, num_hidden_layers=1, num_attention_heads=4,
                          intermediate_size=256, max_seq_length=64)
    weights = E.EncoderWeights.from_state_dict(cfg, encoder_state_dict(cfg, seed=1), "cpu")
    enc = EmbeddingEngine(E.EncoderModel(cfg, weights, "cpu"), Tok())
    full = embed_distributed(enc, texts, group=None)
    idx = ShardedFlatIndex(128, device="cpu")
    idx.add(full)
    q = full[ctx.rank::2] + 0.01
    D, I = idx.search(q, 4)
    return dict(full=full, D=D, I=I, q=q)


def test_dp_embedding_and_sharded_search():
    from rag_llm_k8s_amd.index.flat import FlatL2Index

    texts = ["doc %d %s" % (i, "abc" * (i % 7)) for i in range(23)]
    out = _run(_dp_worker, 1, texts)
    assert torch.allclose(out[0]["full"], out[1]["full"])
    ref = FlatL2Index(128)
    ref.add(out[0]["full"])
    for r in range(WORLD):
        D, I = ref.search(out[r]["q"], 4)
        assert torch.equal(out[r]["I"], I)
        assert torch.allclose(out[r]["D"], D, atol=1e-5)


def _tp_batch_worker(ctx, n_queries):
    """TP=2 generate_batch with more prompts than one prefill step holds: both ranks must queue the
    same prompts at the same steps (the leader broadcasts the token ids) and sample the same tokens."""
    from rag_llm_k8s_amd.engine.llm_engine import SamplingParams
    from rag_llm_k8s_amd.parallel.comm import TPComm
    from rag_llm_k8s_amd.utils.workload import build_workload, make_queries

    comm = TPComm(ctx.tp_group, ctx.tp, ctx.tp_rank, "cpu")
    wl = build_workload(model="tiny", embedder="tiny", n_chunks=48, chunk_words=60, retrieve_k=2, context_k=2,
                        max_new_tokens=4, max_batch=8, max_model_len=1024, max_prefill_tokens=256, device="cpu",
                        ctx=ctx, tp_comm=comm, use_graphs=False, word_vocab=5000)
    qs = make_queries(wl.wm, n_queries, seed=3)
    p = SamplingParams(max_new_tokens=4, temperature=0.8, top_p=0.9, top_k=20, ignore_eos=True)
    outs = wl.svc.generate_batch(qs, params=p, seeds=list(range(100, 100 + n_queries)))
    return [(o.get("_gen_tokens"), o.get("_prompt_tokens"), o["generated_text"]) for o in outs]


def test_tp_generate_batch_same_schedule_on_every_rank():
    out = _run(_tp_batch_worker, 2, 10)
    assert len(out[0]) == 10
    assert all(o[0] == 4 for o in out[0])
    assert out[0] == out[1]


def _tp_channel_worker(ctx, mode):
    import os as _os

    _os.environ["RAGK_TP_CONTROL"] = mode
    from rag_llm_k8s_amd.parallel.tp import K_SHUTDOWN, K_STEP, GlooChannel, ShmChannel, make_channel

    ch = make_channel(ctx.tp_cpu_group, ctx.rank, ctx.world)
    kind = type(ch).__name__
    msgs = [b"", b"abc", bytes(range(256)) * 50, b"", bytes(3 << 20)]  # last one exceeds the shm mailbox
    got = []
    if ctx.rank == 0:
        for m in msgs:
            ch.send(K_STEP, m)
        ch.send(K_SHUTDOWN)
    else:
        while True:
            k, p = ch.recv()
            if k == K_SHUTDOWN:
                break
            got.append(p)
    ch.close()
    return dict(kind=kind, got=got, ok=(got == msgs) if ctx.rank else True)


@pytest.mark.parametrize("mode", ["auto", "gloo"])
def test_tp_control_channel_transports(mode):
    out = _run(_tp_channel_worker, 2, mode)
    assert out[1]["ok"]
    assert out[0]["kind"] == ("ShmChannel" if mode == "auto" else "GlooChannel")
