"""TP=4 / TP=8 layouts on CPU (gloo, one process per rank): the shard geometry Llama-3.1 has at
TP=8 -- one KV head per rank, 2 (here) / 4 (8B) / 8 (70B) query heads, 8-way vocab shards with a
vocabulary not divisible by 8 (last shard padded), 8-way FFN slices -- through every TP code path:
prefill logits with and without sequence parallelism, the split-K decode path with the row-parallel
reduction fused into its RMSNorm consumer (TPComm.add_partials_rmsnorm), generate_batch lockstep,
the control channel, DP ingest and the row-sharded index. Reference: one CPU model, no parallelism
(/root/reference/llm/rag.py:24, /root/reference/llm/ragdeploy.yaml:6); SURVEY §2.5, §4.2 T3."""
import os
import socket
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from rag_llm_k8s_amd.models.llama import llama_tiny
from rag_llm_k8s_amd.utils.synthetic import llama_state_dict

CFG = llama_tiny(vocab=1001, layers=2, hidden=256, heads=16, kv_heads=8, inter=512)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _entry(rank, world, fn, port, d, args):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from rag_llm_k8s_amd.parallel.dist import init_distributed

    ctx = init_distributed(tp=args[0], backend="gloo")
    try:
        res = fn(ctx, *args[1:])
        torch.save(res, os.path.join(d, "r%d.pt" % rank))
    finally:
        dist.destroy_process_group()


def _run(world, fn, *args):
    port = _free_port()
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_entry, args=(world, fn, port, d, args), nprocs=world, join=True)
        return {r: torch.load(os.path.join(d, "r%d.pt" % r), weights_only=False) for r in range(world)}


def _meta_prefill(lens, bts):
    from rag_llm_k8s_amd.ops.backend import AttnMeta

    cu = [0]
    for n in lens:
        cu.append(cu[-1] + n)
    return AttnMeta("prefill", torch.tensor(lens, dtype=torch.int32), torch.tensor(bts, dtype=torch.int32),
                    cu_q=torch.tensor(cu, dtype=torch.int32), host_kv_lens=list(lens))


def _logits_two_steps(model, prompts):
    """Prefill every prompt (one packed step), then ONE decode step for all of them; returns
    (prefill last-token logits, decode logits), each over this rank's vocab shard."""
    from rag_llm_k8s_amd.models.llama import StepInput
    from rag_llm_k8s_amd.ops.backend import AttnMeta

    model.allocate_kv_cache(4 * len(prompts) + 1)
    bts = [[1 + 4 * i + j for j in range(4)] for i in range(len(prompts))]
    ids, pos, slots, last = [], [], [], []
    for i, p in enumerate(prompts):
        ids += p
        pos += list(range(len(p)))
        slots += [bts[i][t // 64] * 64 + t % 64 for t in range(len(p))]
        last.append(len(ids) - 1)
    inp = StepInput(torch.tensor(ids, dtype=torch.int32), torch.tensor(pos, dtype=torch.int32),
                    torch.tensor(slots, dtype=torch.int32), _meta_prefill([len(p) for p in prompts], bts),
                    torch.tensor(last, dtype=torch.int32))
    lp = model.forward(inp)
    nxt = [int(x) % 997 + 3 for x in range(len(prompts))]
    dpos = [len(p) for p in prompts]
    dslots = [bts[i][t // 64] * 64 + t % 64 for i, t in enumerate(dpos)]
    kvl = torch.tensor([t + 1 for t in dpos], dtype=torch.int32)
    meta = AttnMeta("decode", kvl, torch.tensor(bts, dtype=torch.int32), host_kv_lens=kvl.tolist())
    ld = model.forward(StepInput(torch.tensor(nxt, dtype=torch.int32), torch.tensor(dpos, dtype=torch.int32),
                                 torch.tensor(dslots, dtype=torch.int32), meta, None))
    return lp, ld


def _gather_vocab(ctx, local):
    parts = [torch.empty_like(local) for _ in range(ctx.tp)]
    dist.all_gather(parts, local.contiguous(), group=ctx.tp_group)
    return torch.cat(parts, 1)[:, :CFG.vocab_size]


def _layout_worker(ctx, sd, prompts):
    from rag_llm_k8s_amd.models.llama import LlamaModel, LlamaWeights
    from rag_llm_k8s_amd.parallel.comm import TPComm

    w = LlamaWeights.from_state_dict(CFG, sd, "cpu", ctx.tp_rank, ctx.tp)
    g = w.geom()
    m = LlamaModel(CFG, w, "cpu", comm=TPComm(ctx.tp_group, ctx.tp, ctx.tp_rank, "cpu"), max_positions=512)
    out = dict(geom=(g["Hq"], g["Hkv"], g["I"], g["V"], w.vocab_valid))
    for sp in (False, True):
        for part in (False, True):  # decode: plain path + all-reduce | split-K path + fused reduction
            m.seq_parallel, m.sp_min_tokens = sp, 1
            m.be.enable_part = part
            lp, ld = _logits_two_steps(m, prompts)
            out[(sp, part)] = (_gather_vocab(ctx, lp), _gather_vocab(ctx, ld))
    return out


@pytest.mark.parametrize("world", [4, 8])
def test_tp_layouts_logits_match_tp1(world):
    from rag_llm_k8s_amd.models.llama import LlamaModel, LlamaWeights

    sd = llama_state_dict(CFG, seed=11, std=0.05)
    g = torch.Generator().manual_seed(world)
    prompts = [torch.randint(3, CFG.vocab_size, (n,), generator=g).tolist() for n in (37, 5, 66)]
    ref_m = LlamaModel(CFG, LlamaWeights.from_state_dict(CFG, sd, "cpu"), "cpu", max_positions=512)
    ref = {}
    for part in (False, True):
        ref_m.be.enable_part = part
        ref[part] = _logits_two_steps(ref_m, prompts)
    # TP=1: the split-K decode path computes the same rounding points as the plain one
    assert ((ref[True][1] - ref[False][1]).norm() / ref[False][1].norm()).item() < 1e-2
    out = _run(world, _layout_worker, world, sd, prompts)
    Vl = -(-CFG.vocab_size // world)
    assert out[0]["geom"] == (16 // world, 8 // world, 512 // world, Vl, Vl)
    assert out[world - 1]["geom"][4] == CFG.vocab_size - (world - 1) * Vl  # padded last shard
    for r in range(world):
        for key, val in out[r].items():
            if key == "geom":
                continue
            lp, ld = val
            for got, want in ((lp, ref[False][0]), (ld, ref[False][1])):
                rel = ((got - want).norm() / want.norm()).item()
                assert rel < 2e-2, (world, r, key, rel)
    for key in out[0]:  # every rank holds the same gathered logits, bit for bit
        if key != "geom":
            assert all(torch.equal(out[0][key][0], out[r][key][0]) and torch.equal(out[0][key][1], out[r][key][1])
                       for r in range(world))


def _batch_worker(ctx, n_queries):
    from rag_llm_k8s_amd.engine.llm_engine import SamplingParams
    from rag_llm_k8s_amd.parallel.comm import TPComm
    from rag_llm_k8s_amd.utils.workload import build_workload, make_queries

    comm = TPComm(ctx.tp_group, ctx.tp, ctx.tp_rank, "cpu")
    wl = build_workload(model="tiny8", embedder="tiny", n_chunks=40, chunk_words=50, retrieve_k=2, context_k=2,
                        max_new_tokens=3, max_batch=8, max_model_len=1024, max_prefill_tokens=256, device="cpu",
                        ctx=ctx, tp_comm=comm, use_graphs=False, word_vocab=3000)
    wl.svc.engine.model.be.enable_part = True  # decode on the split-K path with the fused reduction
    qs = make_queries(wl.wm, n_queries, seed=5)
    p = SamplingParams(max_new_tokens=3, temperature=0.8, top_p=0.9, top_k=20, ignore_eos=True)
    outs = wl.svc.generate_batch(qs, params=p, seeds=list(range(200, 200 + n_queries)))
    return [(o.get("_gen_tokens"), o.get("_prompt_tokens"), o["generated_text"]) for o in outs]


@pytest.mark.parametrize("world", [4, 8])
def test_tp_layouts_generate_batch_lockstep(world):
    out = _run(world, _batch_worker, world, 9)
    assert len(out[0]) == 9 and all(o[0] == 3 for o in out[0])
    assert all(out[r] == out[0] for r in range(world))


def _control_worker(ctx, sd, prompts):
    from rag_llm_k8s_amd.engine.llm_engine import LLMEngine, SamplingParams
    from rag_llm_k8s_amd.models.llama import LlamaModel, LlamaWeights
    from rag_llm_k8s_amd.parallel.comm import TPComm
    from rag_llm_k8s_amd.parallel.tp import TPControl, follow
    from rag_llm_k8s_amd.server.rag_service import EngineLoop

    w = LlamaWeights.from_state_dict(CFG, sd, "cpu", ctx.tp_rank, ctx.tp)
    m = LlamaModel(CFG, w, "cpu", comm=TPComm(ctx.tp_group, ctx.tp, ctx.tp_rank, "cpu"), max_positions=512)
    m.be.enable_part = True
    eng = LLMEngine(m, num_blocks=32, max_batch=4, max_model_len=512, use_graphs=False, tp_group=ctx.tp_group)
    p = SamplingParams(max_new_tokens=4, temperature=0.8, top_p=0.9, top_k=0, ignore_eos=True)  # top_k 0: exact path
    if ctx.rank == 0:
        loop = EngineLoop(eng, control=TPControl(ctx.tp_cpu_group))
        loop.start()
        seqs = [loop.submit(pr, p, seed=i + 3) for i, pr in enumerate(prompts)]
        for s in seqs:
            s.done.wait(120)
        loop.stop()
        loop.join(60)
        return [s.out for s in seqs]
    follow(eng, ctx.tp_cpu_group)
    return "followed"


def test_tp8_control_channel_and_full_vocab_sampler():
    """8 ranks in lockstep through the control channel; top_k = 0 takes the exact full-vocabulary
    sampler, whose all-gather pads the narrower last vocab shard (1001 % 8 != 0)."""
    sd = llama_state_dict(CFG, seed=12, std=0.05)
    prompts = [[5, 6, 7, 8, 9], list(range(10, 70)), [100, 101]]
    out = _run(8, _control_worker, 8, sd, prompts)
    assert all(out[r] == "followed" for r in range(1, 8))
    assert [len(o) for o in out[0]] == [4, 4, 4]
    assert all(0 <= t < CFG.vocab_size for o in out[0] for t in o)


def _dp_worker(ctx, texts):
    from rag_llm_k8s_amd.engine.encoder_engine import EmbeddingEngine
    from rag_llm_k8s_amd.models import encoder as E
    from rag_llm_k8s_amd.parallel.dp import ShardedFlatIndex, embed_distributed
    from rag_llm_k8s_amd.utils.synthetic import encoder_state_dict

    class Tok:
        def encode_batch(self, ts, add_special_tokens=True, max_length=None):
            return [[(ord(c) * 7 + i) % 500 for i, c in enumerate(t[:60])] or [1] for t in ts]

    cfg = E.EncoderConfig(vocab_size=500, hidden_size=64, num_hidden_layers=1, num_attention_heads=4,
                          intermediate_size=128, max_seq_length=64)
    enc = EmbeddingEngine(E.EncoderModel(cfg, E.EncoderWeights.from_state_dict(cfg, encoder_state_dict(cfg, seed=2),
                                                                                "cpu"), "cpu"), Tok())
    full = embed_distributed(enc, texts, group=None)
    idx = ShardedFlatIndex(64, device="cpu")
    idx.add(full)
    q = full[ctx.rank::ctx.world] + 0.01
    D, I = idx.search(q, 5)
    return dict(full=full, D=D, I=I, q=q)


@pytest.mark.parametrize("world", [4, 8])
def test_dp_ingest_and_sharded_search_layouts(world):
    from rag_llm_k8s_amd.index.flat import FlatL2Index

    texts = ["doc %d %s" % (i, "xyz" * (i % 5)) for i in range(29)]  # 29 % world != 0
    out = _run(world, _dp_worker, 1, texts)
    ref = FlatL2Index(64)
    ref.add(out[0]["full"])
    for r in range(world):
        assert torch.allclose(out[r]["full"], out[0]["full"])
        D, I = ref.search(out[r]["q"], 5)
        assert torch.equal(out[r]["I"], I)
        assert torch.allclose(out[r]["D"], D, atol=1e-5)


def test_tp8_skewed_ranks_same_results(monkeypatch):
    """The 8-rank TP collective sequence (prefill, split-K decode with the fused row-parallel reduction,
    vocab-parallel sampling, control channel) with every rank reaching every collective late by a
    different 0..20 ms (RAGK_FAULTS comm_skew_ms): the same tokens and texts as without skew. A rank
    that is merely late is never an error; only a bounded wait that expires is (tests/test_faults_cpu.py)."""
    ref = _run(8, _batch_worker, 8, 5)
    monkeypatch.setenv("RAGK_FAULTS", "comm_skew_ms=20")
    out = _run(8, _batch_worker, 8, 5)
    assert all(out[r] == ref[0] for r in range(8))
