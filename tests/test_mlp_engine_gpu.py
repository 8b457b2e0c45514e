"""Persistent batch-1 decode MLP (csrc/kernels/mlp_engine.hip) vs a plain PyTorch fp32 reference and vs
the separate-kernel path it replaces (SiLU*up GEMM + down GEMM with the residual epilogue)."""
import math

import pytest
import torch

from rag_llm_k8s_amd.ops import reference as R

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(autouse=True)
def _engine_on(native):
    old = native.MLP_ENGINE
    native.MLP_ENGINE = True
    yield
    native.MLP_ENGINE = old


def rel_err(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


def _weights(H, I, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    gate = (torch.randn(I, H, device=DEV, generator=g) / math.sqrt(H)).bfloat16()
    up = (torch.randn(I, H, device=DEV, generator=g) / math.sqrt(H)).bfloat16()
    down = (torch.randn(H, I, device=DEV, generator=g) / math.sqrt(I)).bfloat16()
    return gate, up, R.pack_gate_up(gate, up), down


def _ref(x, h, gate, up, down):
    a = (torch.nn.functional.silu(x.float() @ gate.float().t()) * (x.float() @ up.float().t())).bfloat16()
    return (h.float() + a.float() @ down.float().t()).bfloat16()


@pytest.mark.parametrize("H,I", [(4096, 14336), (1024, 2048), (2048, 5632)])
def test_mlp_engine_matches_reference(native, H, I):
    gate, up, wgu, down = _weights(H, I, 5)
    assert native.mlp_engine_ok(1, wgu, down)
    torch.manual_seed(6)
    x = torch.randn(1, H, device=DEV).bfloat16()
    h0 = torch.randn(1, H, device=DEV).bfloat16()
    h = h0.clone()
    native.mlp_engine(x, wgu, down, h)
    torch.cuda.synchronize()
    native.mlp_engine_check()
    ref = _ref(x, h0, gate, up, down)
    assert rel_err(h - h0, ref - h0) < 2e-2
    # the separate kernels of the same step (bf16 activations, fused residual)
    a = native.gemm(x, wgu, epi="silu_mul")
    h2 = h0.clone()
    native.gemm(a, down, resid=h2, epi="resid", out=h2)
    assert rel_err(h - h0, h2 - h0) < 1e-2


def test_mlp_engine_repeated_and_graph(native):
    """Many launches in a row (monotonic arrival counters: every launch is its own generation), different
    weights per launch, and the same launches captured in a hipGraph and replayed: identical results."""
    H, I = 4096, 14336
    layers = [_weights(H, I, 10 + i) for i in range(3)]
    torch.manual_seed(7)
    x = torch.randn(1, H, device=DEV).bfloat16()
    h0 = torch.randn(1, H, device=DEV).bfloat16()

    def run(h):
        for _, _, wgu, down in layers:
            native.mlp_engine(x, wgu, down, h)
        return h

    outs = [run(h0.clone()) for _ in range(4)]
    torch.cuda.synchronize()
    native.mlp_engine_check()
    for o in outs[1:]:
        assert torch.equal(o, outs[0])
    hr = h0.clone()
    for gate, up, _, down in layers:
        hr = _ref(x, hr, gate, up, down)
    assert rel_err(outs[0] - h0, hr - h0) < 2e-2

    hg = h0.clone()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        run(hg.clone())  # warm (workspace allocation outside the capture)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):  # the warm-up stream: its engine workspace exists
        run(hg)
    for _ in range(5):
        hg.copy_(h0)
        g.replay()
        torch.cuda.synchronize()
        native.mlp_engine_check()
        assert torch.equal(hg, outs[0])


@pytest.mark.parametrize("S", [8, 4, 11])
def test_mlp_engine_tail_matches_separate_kernels(native, S):
    """The fused post-attention tail (o_proj slabs + residual + RMSNorm inside the launch) vs
    add_partials_rmsnorm followed by the separate SiLU*up / down kernels."""
    H, I = 4096, 14336
    gate, up, wgu, down = _weights(H, I, 21)
    torch.manual_seed(22)
    P = torch.randn(S, 1, H, device=DEV) * 0.3
    gamma = (1 + 0.1 * torch.randn(H, device=DEV)).bfloat16()
    h0 = torch.randn(1, H, device=DEV).bfloat16()
    h = h0.clone()
    native.mlp_engine_tail(P, h, gamma, 1e-5, wgu, down)
    torch.cuda.synchronize()
    native.mlp_engine_check()
    h2 = h0.clone()
    xn = native.add_partials_rmsnorm(P, h2, gamma, 1e-5)
    hmid = h2.clone()
    a = native.gemm(xn, wgu, epi="silu_mul")
    native.gemm(a, down, resid=h2, epi="resid", out=h2)
    assert rel_err(h - hmid, h2 - hmid) < 1e-2
    assert rel_err(h, h2) < 1e-2
    # the residual rows themselves (h + bf16(sum P)) are the same arithmetic: the MLP delta is what differs
    xr = R.rmsnorm(hmid, gamma, 1e-5)
    assert rel_err(h - hmid, _ref(xr, hmid, gate, up, down) - hmid) < 2e-2


def test_mlp_engine_under_concurrent_load(native):
    """Hand-off under uneven load: a memory-bound kernel on another stream holds CUs while the engine
    launches, so its workgroups are dispatched late and unevenly and stream at uneven rates; every launch
    must still complete (no timeout) and match the unloaded result bit for bit."""
    H, I = 4096, 14336
    _, _, wgu, down = _weights(H, I, 41)
    torch.manual_seed(42)
    P = torch.randn(8, 1, H, device=DEV) * 0.2
    gamma = (1 + 0.1 * torch.randn(H, device=DEV)).bfloat16()
    h0 = torch.randn(1, H, device=DEV).bfloat16()
    ref = h0.clone()
    native.mlp_engine_tail(P, ref, gamma, 1e-5, wgu, down)
    torch.cuda.synchronize()
    big = torch.ones(256 * 1024 * 1024 // 4, device=DEV)  # 1 GiB
    side = torch.cuda.Stream()
    outs = []
    for k in range(6):
        with torch.cuda.stream(side):
            for _ in range(2 + k % 3):
                big.mul_(1.0000001)
        h = h0.clone()
        native.mlp_engine_tail(P, h, gamma, 1e-5, wgu, down)
        outs.append(h)
    torch.cuda.synchronize()
    native.mlp_engine_check()
    for h in outs:
        assert torch.equal(h, ref)


def test_mlp_engine_shape_gate(native):
    """Shapes the engine does not take are refused up front (the model keeps the separate kernels)."""
    _, _, wgu, down = _weights(1024, 2048, 3)
    assert not native.mlp_engine_ok(2, wgu, down)  # batch 1 only
    _, _, wgu70, down70 = _weights(8192, 1024, 4)   # H = 8192: x does not fit next to the ring
    assert native.mlp_engine_ok(1, wgu70, down70) == (2 * 8192 <= 28672)


def _engine_run(native, model, cfg, prompt, fault_at=None, switch_at=None):
    """Greedy batch-1 generation through the engine (hipGraph + async decode). fault_at: the persistent MLP
    launches of that decode step get a one-tick deadline (every wait gives up). switch_at: the engine is
    turned off (as the recovery does) before that decode step, without any fault."""
    from rag_llm_k8s_amd.engine.llm_engine import LLMEngine, SamplingParams
    from rag_llm_k8s_amd.utils import faults

    native.MLP_ENGINE = True
    faults.set_faults("mlp_engine_timeout_at_step=%d" % fault_at if fault_at else "")
    try:
        eng = LLMEngine(model, num_blocks=64, max_batch=1, max_prefill_tokens=4096, max_model_len=1024,
                        eos_ids=cfg.eos_token_id, graph_buckets=[1])
        eng.warmup_graphs([1])
        s = eng.add_request(prompt, SamplingParams(max_new_tokens=16, do_sample=False, ignore_eos=True), seed=1)
        while eng.has_work():
            if switch_at is not None and native.MLP_ENGINE and eng.stats["decode_steps"] == switch_at - 1:
                torch.cuda.synchronize()
                native.MLP_ENGINE = False
                eng.graphs.clear()
            eng.step()
        torch.cuda.synchronize()
        return list(s.out), dict(eng.stats)
    finally:
        faults.set_faults(None)


def test_engine_fault_is_discarded_and_recomputed(native):
    """A persistent MLP launch whose waits give up (forced one-tick deadline at decode step 5, inside the
    captured graph) writes no h rows, the launches behind it in the same step exit at entry, and the engine
    sees the host-mapped error word at that step's collection: the step and the one in flight behind it are
    discarded, the counters re-armed, the engine turned off and the rows recomputed on the separate kernels.
    No token of a failed step is accepted (the output equals a run that switched to the separate kernels at
    the same step without a fault), the loop finishes every request, nothing raises."""
    from rag_llm_k8s_amd.models import llama as L

    cfg = L.llama_tiny(vocab=512, layers=2, hidden=1024, heads=8, kv_heads=2, inter=2048)
    w = L.LlamaWeights.random(cfg, DEV, seed=3)
    model = L.LlamaModel(cfg, w, DEV, max_positions=2048)
    assert native.mlp_engine_ok(1, w.layers[0]["wgu"], w.layers[0]["wdown"])
    prompt = torch.randint(3, cfg.vocab_size, (40,), generator=torch.Generator().manual_seed(4)).tolist()
    n_ws = len(native._me_ws)
    ref, st_ref = _engine_run(native, model, cfg, prompt, switch_at=5)
    assert st_ref.get("engine_faults", 0) == 0 and len(ref) == 16
    assert len(native._me_ws) > n_ws  # the engine ran (a workspace for this engine's capture stream)
    got, st = _engine_run(native, model, cfg, prompt, fault_at=5)
    assert st.get("engine_faults", 0) == 1
    assert native.mlp_engine_fault() == 0  # re-armed
    assert got == ref
    # and the engine itself is healthy again after a re-arm: a clean run reproduces an all-engine run
    on1, st1 = _engine_run(native, model, cfg, prompt)
    on2, st2 = _engine_run(native, model, cfg, prompt)
    assert on1 == on2 and st1.get("engine_faults", 0) == 0 and len(on1) == 16
