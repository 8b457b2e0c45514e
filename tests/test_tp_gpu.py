"""Tensor parallelism on the GPU, as far as one MI355X allows: 2, 4 and 8 ranks on cuda:0.

Every rank runs the real TP code path -- Megatron-sharded Llama weights at Llama-3.1-8B widths
(hidden 4096, 32/8 heads, FFN 14336, 128,256-token vocabulary; 2 layers), the peer-mapped
all-reduce / all-gather kernels (csrc/comm/allreduce.hip, hipIpc handles exchanged over gloo),
the vocab-parallel sampler with its candidate all-gather, graph-captured and asynchronous decode --
only the xGMI hop is replaced by local HBM. RCCL itself cannot run two ranks on one device, so
bulk messages are kept under the peer-mapped size limit here.

Oracles: the TP=1 model on the same weights (prefill logits), the eager synchronous engine (graph
+ async decode must produce the same tokens), and the other rank (identical samples).
"""
import os
import socket
import tempfile
import time

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
WORLD = 2  # the fault test; the engine test is parametrized over 2 / 4 / 8 ranks


def _log(rank, world, msg):
    """Progress on stderr (captured by pytest) and, on the GPU box, appended to gpurun_out/ (pytest's
    capture hides stderr until the test ends: a multi-minute 8-rank run must not look silent)."""
    import sys

    line = "[tp%d r%d %.0fs] %s" % (world, rank, time.monotonic() % 100000, msg)
    print(line, file=sys.stderr, flush=True)
    root = os.environ.get("GRAFT_REPO_ROOT")
    if root:
        try:
            os.makedirs(os.path.join(root, "gpurun_out"), exist_ok=True)
            with open(os.path.join(root, "gpurun_out", "tp_test_progress.log"), "a") as f:
                f.write(line + "\n")
        except OSError:
            pass


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _cfg(layers=2):
    from rag_llm_k8s_amd.models.llama import llama31_8b

    c = llama31_8b()
    c.num_hidden_layers = layers
    return c


def _state_dict(cfg, seed=1234):
    """HF-named full weights generated on the GPU (same values in every process)."""
    g = torch.Generator(device="cuda").manual_seed(seed)
    H, D, I, V = cfg.hidden_size, cfg.head_dim, cfg.intermediate_size, cfg.vocab_size
    Hq, Hkv = cfg.num_attention_heads, cfg.num_key_value_heads

    def rnd(*shape, std=0.02):
        return (torch.randn(*shape, generator=g, device="cuda") * std).bfloat16()

    def ones(n):
        return (1.0 + 0.1 * torch.randn(n, generator=g, device="cuda")).bfloat16()

    sd = {"model.embed_tokens.weight": rnd(V, H, std=0.5)}
    for i in range(cfg.num_hidden_layers):
        p = "model.layers.%d." % i
        sd[p + "input_layernorm.weight"] = ones(H)
        sd[p + "post_attention_layernorm.weight"] = ones(H)
        sd[p + "self_attn.q_proj.weight"] = rnd(Hq * D, H)
        sd[p + "self_attn.k_proj.weight"] = rnd(Hkv * D, H)
        sd[p + "self_attn.v_proj.weight"] = rnd(Hkv * D, H)
        sd[p + "self_attn.o_proj.weight"] = rnd(H, Hq * D)
        sd[p + "mlp.gate_proj.weight"] = rnd(I, H)
        sd[p + "mlp.up_proj.weight"] = rnd(I, H)
        sd[p + "mlp.down_proj.weight"] = rnd(H, I)
    sd["model.norm.weight"] = ones(H)
    sd["lm_head.weight"] = rnd(V, H)
    return sd


def _prefill_logits(model, ids):
    """Full-prompt prefill through the native kernels; logits of the last position (vocab shard)."""
    from rag_llm_k8s_amd.models.llama import StepInput
    from rag_llm_k8s_amd.ops.backend import AttnMeta
    from rag_llm_k8s_amd.ops.native import build_prefill_tiles

    n = len(ids)
    nb = -(-n // 64)
    model.allocate_kv_cache(nb + 1)
    dev = model.device
    i32 = dict(dtype=torch.int32, device=dev)
    bt = torch.zeros((1, nb + 1), **i32)
    bt[0, :nb] = torch.arange(1, nb + 1, **i32)
    meta = AttnMeta("prefill", torch.tensor([n], **i32), bt, cu_q=torch.tensor([0, n], **i32),
                    tiles=build_prefill_tiles([n], model.Hq, model.Hkv).to(dev), host_kv_lens=[n], host_q_lens=[n])
    inp = StepInput(torch.tensor(ids, **i32), torch.arange(n, **i32), torch.arange(64, 64 + n, **i32), meta,
                    torch.tensor([n - 1], **i32))
    return model.forward(inp)


def _prefill_decode_logits(model, ids, nxt):
    """Prefill `ids`, then one decode step of token `nxt` through the model's decode path (the split-K
    GEMMs with the row-parallel reduction fused into the RMSNorm under TP): its logits (vocab shard)."""
    from rag_llm_k8s_amd.models.llama import StepInput
    from rag_llm_k8s_amd.ops.backend import AttnMeta
    from rag_llm_k8s_amd.ops.native import build_prefill_tiles, decode_partitions

    n = len(ids)
    nb = -(-(n + 1) // 64)
    model.allocate_kv_cache(nb + 2)
    dev = model.device
    i32 = dict(dtype=torch.int32, device=dev)
    bt = torch.zeros((1, nb + 1), **i32)
    bt[0, :nb] = torch.arange(1, nb + 1, **i32)
    meta = AttnMeta("prefill", torch.tensor([n], **i32), bt, cu_q=torch.tensor([0, n], **i32),
                    tiles=build_prefill_tiles([n], model.Hq, model.Hkv).to(dev), host_kv_lens=[n], host_q_lens=[n])
    model.forward(StepInput(torch.tensor(ids, **i32), torch.arange(n, **i32), torch.arange(64, 64 + n, **i32), meta,
                            torch.tensor([n - 1], **i32)))
    pt, mp = decode_partitions(8192, 1, model.Hkv)
    ws_o = torch.empty((1, model.Hq, mp, model.D), dtype=torch.float32, device=dev) if mp > 1 else None
    ws_ml = torch.empty((1, model.Hq, mp, 2), dtype=torch.float32, device=dev) if mp > 1 else None
    dm = AttnMeta("decode", torch.tensor([n + 1], **i32), bt, part_tiles=pt, max_parts=mp, ws_o=ws_o, ws_ml=ws_ml)
    h = torch.empty((1, model.cfg.hidden_size), dtype=torch.bfloat16, device=dev)
    inp = StepInput(torch.tensor([nxt], **i32), torch.tensor([n], **i32), torch.tensor([64 + n], **i32), dm, None)
    assert model._decode_part_ok(inp, h)
    return model.forward(inp)


def _init(rank, port, world=WORLD):
    # every rank on cuda:0 on purpose: the distinctness self-test must be told so. Eight processes with
    # HIP's default 4 hardware queues each over-subscribe the device's mapped queues (a rank's collective
    # kernel started ~43 s after its peers', profiles/tp8_trace_report_r5.txt); 2 queues per process still
    # stalled a round-6 suite run (215 s to the first logits, then a timed-out collective). One queue per
    # process (set before HIP init): 8 queues, every one mapped, no peer-waiting kernel on an unmapped queue.
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0", RAGK_TP_CONTROL="gloo", RAGK_ALLOW_SHARED_DEVICE="1")
    if world >= 8:
        os.environ["GPU_MAX_HW_QUEUES"] = "1"
    from rag_llm_k8s_amd.parallel.dist import init_distributed

    return init_distributed(tp=world, backend="gloo")


def _tp_worker(rank, port, d, world):
    WORLD = world
    ctx = _init(rank, port, world)  # 8 ranks: 1 hardware queue per process (see _init)
    _log(rank, world, "process group up")
    from rag_llm_k8s_amd.engine.llm_engine import LLMEngine, SamplingParams
    from rag_llm_k8s_amd.models.llama import LlamaModel, LlamaWeights
    from rag_llm_k8s_amd.parallel.comm import TPComm

    res = {}
    comm = None
    try:
        cfg = _cfg()
        sd = _state_dict(cfg)
        # 8 processes time-slicing one GPU (and 16 host CPUs): a rank can trail the others by a long time.
        # On a FRESH box the first 8-rank run stalled 29 s and then > 60 s inside its first two prefills
        # (call 5-10 peer waits) while a second run in the same pytest process, and the 2 / 4-rank runs before
        # it, finished in seconds: per-process cold start (first launches of each kernel while the image's
        # pages come in), not the protocol. The rehearsal's peer waits get a 240 s bound instead of the
        # serving default (5 s); the 2 / 4-rank cases keep the default. (Until round 6 the kernels held the
        # bound as 32-bit 100 MHz ticks, capped at 43 s: the "60 s" asked for here was 43 s.)
        comm = TPComm(ctx.tp_group, ctx.tp, ctx.tp_rank, ctx.device, ctx.tp_cpu_group, ipc_max_bytes=16 << 20,
                      ipc_spin_limit=240_000_000 if world >= 8 else None)
        res["ipc"] = comm.ipc is not None
        _log(rank, world, "comm up (peer-mapped: %s)" % res["ipc"])
        w = LlamaWeights.from_state_dict(cfg, sd, ctx.device, ctx.tp_rank, ctx.tp)
        m = LlamaModel(cfg, w, ctx.device, comm=comm, max_positions=4096)
        _log(rank, world, "model up")
        gen = torch.Generator().manual_seed(7)
        ids = torch.randint(3, cfg.vocab_size, (300,), generator=gen).tolist()
        local = _prefill_logits(m, ids)  # [1, V/2] this rank's vocab shard
        torch.cuda.synchronize()
        _log(rank, world, "prefill logits")
        full = comm.ipc.all_gather(local.contiguous()).view(WORLD, 1, -1)
        res["tp_logits"] = torch.cat([full[r] for r in range(WORLD)], 1)[:, :cfg.vocab_size].cpu()
        _log(rank, world, "prefill logits gathered")
        local = _prefill_decode_logits(m, ids, 77)  # decode: fused row-parallel reduction
        full = comm.ipc.all_gather(local.contiguous()).view(WORLD, 1, -1)
        res["tp_dec_logits"] = torch.cat([full[r] for r in range(WORLD)], 1)[:, :cfg.vocab_size].cpu()
        _log(rank, world, "prefill + decode logits")
        if rank == 0:
            ref = LlamaModel(cfg, LlamaWeights.from_state_dict(cfg, sd, ctx.device), ctx.device, max_positions=4096)
            res["ref_logits"] = _prefill_logits(ref, ids).cpu()
            res["ref_dec_logits"] = _prefill_decode_logits(ref, ids, 77).cpu()
            del ref
            _log(rank, world, "TP=1 reference done")
        # the other ranks must not enter the engine's collectives while rank 0 computes the TP=1
        # reference: their bounded peer waits (5 s) spin on the shared GPU and starve rank 0 -- the
        # cause of the 8-rank timeouts of round 4 (rank 0 alone took longer than the bound)
        dist.barrier(group=ctx.tp_cpu_group)
        del sd
        torch.cuda.empty_cache()

        # engine: graph-captured + asynchronous decode vs eager synchronous, sampled and greedy
        # the 1100-token prompt makes the first prefill step >= RAGK_TP_OVERLAP_MIN (1024): two
        # micro-batches with the peer-mapped all-reduce on the side stream overlapping the next one
        prompts = [torch.randint(3, cfg.vocab_size, (n,), generator=gen).tolist() for n in (100, 1100, 37)]
        sampled = SamplingParams(max_new_tokens=12, temperature=0.7, top_p=0.9, top_k=50, ignore_eos=True)
        greedy = SamplingParams(max_new_tokens=12, do_sample=False, ignore_eos=True)
        # 8 ranks: graph-captured decode only. The eager (host-launched, synchronous) engine at 8 processes
        # on ONE GPU timed out in a peer wait even with a 60 s bound (round 4, 1 of 2 runs): 8 time-sliced
        # GPU contexts plus the parent's, each collective needing all 8 mapped at once. One rank per GPU
        # (the deployment) has no such sharing; eager == graph is checked at 2 / 4 ranks.
        for graphs in ((True, False) if world < 8 else (True,)):
            eng = LLMEngine(m, num_blocks=64, max_batch=4, max_model_len=2048, use_graphs=graphs,
                            tp_group=ctx.tp_group, graph_buckets=[1, 2, 4])
            assert eng.tp_overlap_min_tokens <= 1237
            if graphs:
                eng.warmup_graphs()
                _log(rank, world, "graphs captured")
            res[("sampled", graphs)] = eng.generate(prompts, sampled, seeds=[11, 12, 13])
            _log(rank, world, "sampled generate done (graphs=%s)" % graphs)
            res[("greedy", graphs)] = eng.generate(prompts, greedy)
            res[("async", graphs)] = eng.async_decode
            _log(rank, world, "engine graphs=%s" % graphs)
            del eng
            torch.cuda.empty_cache()
        res["error"] = comm.ipc.error()
    finally:
        torch.cuda.synchronize()
        dist.barrier(group=ctx.tp_cpu_group)
        if comm is not None and comm.ipc is not None:
            comm.ipc.close()
        torch.save(res, os.path.join(d, "r%d.pt" % rank))
        dist.destroy_process_group()


def _spawn(target, timeout=600, world=WORLD):
    port = _free_port()
    d = tempfile.mkdtemp()
    ctx = mp.get_context("spawn")
    extra = (world,) if target is _tp_worker else ()
    procs = [ctx.Process(target=target, args=(r, port, d) + extra) for r in range(world)]
    for p in procs:
        p.start()
    deadline = time.monotonic() + timeout
    while time.monotonic() < deadline and any(p.is_alive() for p in procs):
        procs[[p.is_alive() for p in procs].index(True)].join(timeout=30)
        alive = [r for r, p in enumerate(procs) if p.is_alive()]
        if alive:  # the parent's view every 30 s: which ranks are still running
            _log(-1, world, "ranks still running: %s" % alive)
    for p in procs:
        if p.is_alive():
            p.kill()
            p.join()
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    return [torch.load(os.path.join(d, "r%d.pt" % r), weights_only=False) for r in range(world)]


# 8 ranks as 8 processes on ONE GPU: with HIP's default 4 hardware queues per process (32 queues) a rank's
# collective kernel could start tens of seconds after its peers' (queue co-scheduling; kernel trace in
# profiles/tp8_trace_report_r5.txt), so the workers run one queue each (_tp_worker).
TP_WORLDS = [int(w) for w in os.environ.get("RAGK_TP_WORLDS", "2,4,8").split(",")]


@pytest.mark.timeout(900)
@pytest.mark.parametrize("world", TP_WORLDS)
def test_tp_llama8b_widths_on_one_gpu(native, world):
    """TP=2/4/8 shards of Llama-3.1-8B widths (TP=8: 4 query heads, 1 KV head, 1792 FFN rows, a 16k-row
    vocab shard per rank), 2 layers, every rank a process on cuda:0: prefill logits and fused-decode
    logits vs TP=1, graph + async decode == eager (2 / 4 ranks), the same samples on every rank, and the
    micro-batched overlap prefill (the 1100-token prompt)."""
    WORLD = world
    out = _spawn(_tp_worker, world=world, timeout=840 if world >= 8 else 600)
    assert all(o["ipc"] for o in out), "peer-mapped collectives must pass their self-test"
    ref = out[0]["ref_logits"]
    for r in range(WORLD):
        got = out[r]["tp_logits"]
        rel = ((got - ref).norm() / ref.norm()).item()
        assert rel < 2e-2, (r, rel)
        assert out[r]["error"] is False
    for r in range(1, WORLD):
        assert torch.equal(out[0]["tp_logits"], out[r]["tp_logits"])
    dref = out[0]["ref_dec_logits"]
    for r in range(WORLD):
        rel = ((out[r]["tp_dec_logits"] - dref).norm() / dref.norm()).item()
        assert rel < 2e-2, ("decode", r, rel)
    for r in range(1, WORLD):
        assert torch.equal(out[0]["tp_dec_logits"], out[r]["tp_dec_logits"])
    for r in range(WORLD):
        assert out[r][("async", True)] is True
        for kind in ("sampled", "greedy"):
            g = out[r][(kind, True)]
            assert [len(x) for x in g] == [12, 12, 12]
            if (kind, False) in out[r]:
                assert g == out[r][(kind, False)], (r, kind)  # graph-captured async TP decode == eager synchronous
    for kind in ("sampled", "greedy"):
        for r in range(1, WORLD):
            assert out[0][(kind, True)] == out[r][(kind, True)]  # every rank sampled the same tokens


def _fault_worker(rank, port, d):
    """Rank 1 stops taking part after set-up; rank 0's engine loop must fail its step with
    CommError within the bounded wait, and the service must report unhealthy."""
    ctx = _init(rank, port)
    from types import SimpleNamespace

    from rag_llm_k8s_amd.config import RagConfig
    from rag_llm_k8s_amd.engine.llm_engine import LLMEngine, SamplingParams
    from rag_llm_k8s_amd.models.llama import LlamaModel, LlamaWeights, llama_tiny
    from rag_llm_k8s_amd.parallel.comm import TPComm
    from rag_llm_k8s_amd.server.rag_service import RagService

    res = {}
    comm = None
    try:
        cfg = llama_tiny(vocab=1024, layers=2, hidden=512, heads=8, kv_heads=2, inter=1024)
        comm = TPComm(ctx.tp_group, ctx.tp, ctx.tp_rank, ctx.device, ctx.tp_cpu_group, ipc_spin_limit=20000)  # 20 ms
        res["ipc"] = comm.ipc is not None
        w = LlamaWeights.random(cfg, ctx.device, ctx.tp_rank, ctx.tp, seed=3)
        m = LlamaModel(cfg, w, ctx.device, comm=comm, max_positions=1024)
        eng = LLMEngine(m, num_blocks=16, max_batch=2, max_model_len=512, use_graphs=False, tp_group=ctx.tp_group)
        if rank == 0:
            store = SimpleNamespace(index=SimpleNamespace(ntotal=0), flush=lambda: None)
            svc = RagService(RagConfig(device=ctx.device), eng, None, None, store, start_threads=True)
            before = svc.health()
            t0 = time.monotonic()
            s = svc.loop.submit(list(range(3, 40)), SamplingParams(max_new_tokens=4, do_sample=False), seed=1)
            s.done.wait(60)
            res["elapsed"] = time.monotonic() - t0
            res["finish"] = s.finish_reason
            res["before"] = before["engine_alive"]
            h = svc.health()
            res["after"] = h["engine_alive"]
            res["comm_ok"] = h["comm_ok"]
            res["error"] = h["engine_error"]
            svc.shutdown()
    finally:
        torch.cuda.synchronize()
        dist.barrier(group=ctx.tp_cpu_group)  # rank 1 keeps its mapped region alive until rank 0 is done
        if comm is not None and comm.ipc is not None:
            comm.ipc.close()
        torch.save(res, os.path.join(d, "r%d.pt" % rank))
        dist.destroy_process_group()


def test_tp_comm_fault_fails_step_and_health(native):
    out = _spawn(_fault_worker, timeout=300)
    r0 = out[0]
    assert r0["ipc"]
    assert r0["before"] is True
    assert r0["finish"] == "error", r0
    assert "CommError" in (r0["error"] or ""), r0
    assert r0["after"] is False and r0["comm_ok"] is False
    assert r0["elapsed"] < 30, r0["elapsed"]
