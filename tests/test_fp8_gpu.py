"""fp8 weight GEMMs (csrc/kernels/gemm_fp8.hip) vs their fp32 oracle (ops/fp8.reference_linear):
W8A16 decode (M <= 64) and W8A8 prefill (block-scaled fp8 MFMA), every fused epilogue."""
import math

import pytest
import torch

from rag_llm_k8s_amd.ops import fp8 as F8
from rag_llm_k8s_amd.ops import reference as R

pytestmark = pytest.mark.gpu
DEV = "cuda"


def rel_err(a, b):
    a, b = a.float(), b.float()
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


def test_quant_rows_matches_torch(native):
    torch.manual_seed(0)
    x = (torch.randn(37, 4096, device=DEV) * torch.linspace(0.01, 5, 37, device=DEV)[:, None]).bfloat16()
    q, s = native.quant_fp8_rows(x)
    rq, rs = F8.quantize_rows(x)
    assert torch.allclose(s, rs, rtol=1e-6, atol=0)
    same = (q.view(torch.uint8) == rq.view(torch.uint8)).float().mean().item()
    assert same > 0.999, same  # RNE on both sides; ties may differ by the 1/s rounding
    assert rel_err(q.float() * s[:, None], x.float()) < 0.05


@pytest.mark.parametrize("M", [1, 7, 16, 33, 64, 65, 200, 1024])
@pytest.mark.parametrize("N,K", [(768, 1024), (4096, 4096)])
def test_gemm_fp8_epilogues(native, M, N, K):
    torch.manual_seed(M + N)
    x = torch.randn(M, K, device=DEV).bfloat16()
    w = (torch.randn(N, K, device=DEV) / math.sqrt(K)).bfloat16()
    wq = F8.quantize_weight(w)
    assert rel_err(wq.dequant(), w.float()) < 0.05
    bias = torch.randn(N, device=DEV).bfloat16()
    r = torch.randn(M, N, device=DEV).bfloat16()
    for epi, kw in [("none", {}), ("resid", dict(resid=r)), ("bias", dict(bias=bias)),
                    ("bias_gelu", dict(bias=bias))]:
        y = native.gemm_fp8(x, wq, epi=epi, **kw)
        ref = F8.reference_linear(x, wq, epi=epi, **kw)
        assert rel_err(y, ref) < 1e-2, (epi, rel_err(y, ref))
    yf = native.gemm_fp8(x, wq, out_f32=True)
    assert rel_err(yf, F8.reference_linear(x, wq, out_f32=True)) < 2e-3
    # vs the bf16 GEMM: the fp8 error budget (weights ~2-3 %, activations too above M=64)
    assert rel_err(native.gemm_fp8(x, wq), x.float() @ w.float().t()) < 0.08


@pytest.mark.parametrize("M", [1, 32, 64, 300])
def test_gemm_fp8_silu_mul(native, M):
    torch.manual_seed(5)
    K, N = 4096, 1024
    x = torch.randn(M, K, device=DEV).bfloat16()
    g = (torch.randn(N, K, device=DEV) / 64).bfloat16()
    u = (torch.randn(N, K, device=DEV) / 64).bfloat16()
    wq = F8.quantize_weight(R.pack_gate_up(g, u))
    y = native.gemm_fp8(x, wq, epi="silu_mul")
    ref = F8.reference_linear(x, wq, epi="silu_mul")
    assert y.shape == (M, N) and rel_err(y, ref) < 1e-2


def test_fp8_engine_gpu_matches_cpu_reference(native):
    """fp8-weight Llama: GPU engine (fp8 kernels, hipGraph decode) vs the CPU engine running the
    fp32 oracle of the same quantized arithmetic; prefill logits (W8A8) and greedy tokens (W8A16)."""
    from rag_llm_k8s_amd.engine.llm_engine import LLMEngine, SamplingParams
    from rag_llm_k8s_amd.models.llama import LlamaModel, LlamaWeights, StepInput, llama_tiny
    from rag_llm_k8s_amd.ops.backend import AttnMeta
    from rag_llm_k8s_amd.ops.native import build_prefill_tiles
    from rag_llm_k8s_amd.utils.synthetic import llama_state_dict

    cfg = llama_tiny(vocab=1024, layers=2, hidden=512, heads=4, kv_heads=1, inter=512)
    sd = llama_state_dict(cfg, seed=3, std=0.05)

    def engine(dev, graphs):
        w = LlamaWeights.from_state_dict(cfg, sd, dev).quantize_fp8()
        m = LlamaModel(cfg, w, dev, max_positions=2048)
        return LLMEngine(m, num_blocks=64, max_batch=8, max_prefill_tokens=300, max_model_len=2048, use_graphs=graphs)

    outs = {}
    for dev in ("cuda", "cpu"):
        eng = engine(dev, False)
        eng.bm.ensure(7, 150)
        tbl = eng.bm.table(7)
        slots = torch.tensor([tbl[p // 64] * 64 + p % 64 for p in range(150)], dtype=torch.int32)
        bt = torch.tensor([tbl + [0] * (eng.max_blocks - len(tbl))], dtype=torch.int32)
        meta = AttnMeta("prefill", torch.tensor([150], dtype=torch.int32).to(dev), bt.to(dev),
                        cu_q=torch.tensor([0, 150], dtype=torch.int32).to(dev),
                        tiles=build_prefill_tiles([150], 4, 1).to(dev), host_kv_lens=[150])
        ids = torch.arange(150, dtype=torch.int32) * 7 % 1000
        inp = StepInput(ids.to(dev), torch.arange(150, dtype=torch.int32).to(dev), slots.to(dev), meta, None)
        outs[dev] = eng.model.forward(inp).float().cpu()
    # W8A8 re-quantizes every layer input: bf16-level GPU/CPU differences flip fp8 roundings
    assert rel_err(outs["cuda"], outs["cpu"]) < 0.15
    torch.manual_seed(0)
    prompts = [torch.randint(3, 1000, (n,)).tolist() for n in (5, 77, 130, 300)]
    p = SamplingParams(max_new_tokens=6, do_sample=False, ignore_eos=True)
    gpu = engine("cuda", True).generate(prompts, p)
    cpu = engine("cpu", False).generate(prompts, p)
    first = sum(int(g[0] == c[0]) for g, c in zip(gpu, cpu))
    assert first >= 3, (gpu, cpu)


@pytest.mark.parametrize("M", [1, 17, 33, 64])
@pytest.mark.parametrize("N,K", [(768, 1024), (4096, 4096), (1024, 14336)])
def test_gemm_fp8_stream_decode(native, monkeypatch, M, N, K):
    """The glds-ring decode kernel (gemm_stream.hip) on fp8 weights, forced for every shape."""
    monkeypatch.setattr(native, "use_stream", lambda *a, **k: True)
    torch.manual_seed(M + K)
    x = torch.randn(M, K, device=DEV).bfloat16()
    w = (torch.randn(N, K, device=DEV) / math.sqrt(K)).bfloat16()
    wq = F8.quantize_weight(w)
    r = torch.randn(M, N, device=DEV).bfloat16()
    for epi, kw in [("none", {}), ("resid", dict(resid=r))]:
        for _ in range(2):
            y = native.gemm_fp8(x, wq, epi=epi, **kw)
            assert rel_err(y, F8.reference_linear(x, wq, epi=epi, **kw)) < 1e-2
    g = (torch.randn(N, K, device=DEV) / math.sqrt(K)).bfloat16()
    wgu = F8.quantize_weight(R.pack_gate_up(w[: N // 2 // 64 * 64 or 64], g[: N // 2 // 64 * 64 or 64]))
    y = native.gemm_fp8(x, wgu, epi="silu_mul")
    assert rel_err(y, F8.reference_linear(x, wgu, epi="silu_mul")) < 1e-2


@pytest.mark.parametrize("M", [1, 32, 64])
@pytest.mark.parametrize("N,K", [(4096, 4096), (6144, 4096), (4096, 14336), (1000, 1024)])
def test_gemm_part_fp8(native, M, N, K):
    """W8A16 split-K partial GEMM (gemm_part.hip FP8): the slabs (row scale applied) sum to
    x @ dequant(w)^T, for every slice size the planner can pick."""
    torch.manual_seed(M + N)
    x = torch.randn(M, K, device=DEV).bfloat16()
    wq = F8.quantize_weight((torch.randn(N, K, device=DEV) / math.sqrt(K)).bfloat16())
    ref = x.float() @ wq.dequant().t()
    ks0, S0 = native.gemm_part_slabs(M, N, K)
    assert S0 > 0
    for ks in sorted({ks0, 8, 16}):
        if K % (64 * ks):
            continue
        P = native.gemm_part(x, wq, ks=ks)
        assert P.shape == (K // (64 * ks), M, N)
        assert rel_err(P.sum(0), ref) < 2e-3, ks
