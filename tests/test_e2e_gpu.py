"""T2/T5 on the GPU: native engine vs the CPU reference path on identical weights, hipGraph decode
vs eager decode, encoder vs CPU encoder, and a tiny end-to-end RAG workload."""
import pytest
import torch

from rag_llm_k8s_amd.engine.llm_engine import LLMEngine, SamplingParams
from rag_llm_k8s_amd.models import encoder as E
from rag_llm_k8s_amd.models.llama import LlamaModel, LlamaWeights, llama_tiny
from rag_llm_k8s_amd.utils.synthetic import encoder_state_dict, llama_state_dict

pytestmark = pytest.mark.gpu


def _engine(cfg, sd, device, graphs, mb=8):
    w = LlamaWeights.from_state_dict(cfg, sd, device)
    m = LlamaModel(cfg, w, device, max_positions=2048)
    return LLMEngine(m, num_blocks=64, max_batch=mb, max_prefill_tokens=300, max_model_len=2048, use_graphs=graphs)


@pytest.fixture(scope="module")
def tiny_llama():
    cfg = llama_tiny(vocab=1024, layers=2, hidden=512, heads=4, kv_heads=1, inter=512)
    return cfg, llama_state_dict(cfg, seed=3, std=0.05)


def _oracle_logits(cfg, sd, ids):
    """fp32-accumulating CPU oracle: logits [T, V] of every position of `ids` (one prefill)."""
    from rag_llm_k8s_amd.models.llama import StepInput
    from rag_llm_k8s_amd.ops.backend import AttnMeta

    eng = _engine(cfg, sd, "cpu", graphs=False)
    n = len(ids)
    eng.bm.ensure(99, n + 1)
    tbl = eng.bm.table(99)
    slots = torch.tensor([tbl[q // 64] * 64 + q % 64 for q in range(n)], dtype=torch.int32)
    bt = torch.tensor([tbl + [0] * (eng.max_blocks - len(tbl))], dtype=torch.int32)
    meta = AttnMeta("prefill", torch.tensor([n], dtype=torch.int32), bt, cu_q=torch.tensor([0, n], dtype=torch.int32),
                    host_kv_lens=[n])
    inp = StepInput(torch.tensor(ids, dtype=torch.int32), torch.arange(n, dtype=torch.int32), slots, meta, None)
    return eng.model.forward(inp).float()


def _check_greedy(cfg, sd, prompts, outs, rel_tol=0.02):
    """Per-step top-1 margin check (teacher forced on the GPU's own tokens, so one flip does not
    cascade): every greedy token must be the oracle's argmax, or within rel_tol x the row's logit
    spread of it (a near-tie that a bf16 reduction order may legitimately flip). Returns the count of
    exact argmax agreements."""
    exact = 0
    for pr, out in zip(prompts, outs):
        lg = _oracle_logits(cfg, sd, pr + out[:-1])
        for k, tok in enumerate(out):
            row = lg[len(pr) - 1 + k]
            top = float(row.max())
            gap = top - float(row[tok])
            spread = top - float(row.min())
            assert gap <= rel_tol * spread, (k, tok, int(row.argmax()), gap, spread)
            exact += int(gap == 0.0)
    return exact


def test_gpu_engine_matches_cpu_greedy(native, tiny_llama):
    """GPU engine (graphs, async decode, mixed steps) greedy tokens vs the fp32 CPU oracle, per step."""
    cfg, sd = tiny_llama
    torch.manual_seed(0)
    prompts = [torch.randint(3, 1000, (n,)).tolist() for n in (5, 77, 130, 300, 513)]
    p = SamplingParams(max_new_tokens=6, do_sample=False, ignore_eos=True)
    gpu = _engine(cfg, sd, "cuda", graphs=True).generate(prompts, p)
    exact = _check_greedy(cfg, sd, prompts, gpu)
    assert exact >= 0.7 * sum(len(x) for x in gpu), exact


def test_graph_decode_equals_eager(native, tiny_llama):
    cfg, sd = tiny_llama
    torch.manual_seed(1)
    prompts = [torch.randint(3, 1000, (n,)).tolist() for n in (9, 40, 200)]
    p = SamplingParams(max_new_tokens=10, temperature=0.8, top_p=0.9, top_k=40, ignore_eos=True)
    a = _engine(cfg, sd, "cuda", graphs=True).generate(prompts, p, seeds=[1, 2, 3])
    b = _engine(cfg, sd, "cuda", graphs=False).generate(prompts, p, seeds=[1, 2, 3])
    assert a == b


def test_async_decode_equals_sync(native, tiny_llama):
    """Asynchronous decode pipeline (ids fed on the device, tokens accepted one step late, deferred
    KV frees) vs the synchronous graph path: identical tokens with early stops (stop tokens), per-request
    lengths (batch composition changes -> the gather path) and more requests than batch slots
    (prefills drain the pipeline mid-run); sampled, so the per-step seeds must line up too."""
    cfg, sd = tiny_llama
    torch.manual_seed(4)
    prompts = [torch.randint(3, 1000, (n,)).tolist() for n in (9, 40, 200, 5, 77, 130, 31)]
    stop = list(range(3, 1000, 9))  # ~1/9 of the vocabulary ends a sequence
    params = [SamplingParams(max_new_tokens=m, temperature=0.9, top_p=0.95, top_k=50, stop_token_ids=stop)
              for m in (12, 3, 20, 7, 16, 1, 9)]
    outs = {}
    for mode in (True, False):
        eng = _engine(cfg, sd, "cuda", graphs=True, mb=4)
        eng.async_decode = mode
        # mixed prefill+decode steps run a decoding row through the prefill kernels (different bf16
        # reduction order), and WHICH steps are mixed shifts with the one-step-late acceptance: off here,
        # so the comparison isolates the pipeline (mixed steps: test_mixed_steps_gpu_close_to_separate)
        eng.mixed_steps = False
        seqs = [eng.add_request(pr, pa, seed=10 + i) for i, (pr, pa) in enumerate(zip(prompts, params))]
        eng.run_until_done()
        assert eng._inflight is None and not eng.running
        assert eng.bm.free_blocks() == 64 - 1  # every block back (block 0 is the scratch block)
        outs[mode] = [(s.out, s.finish_reason) for s in seqs]
    assert outs[True] == outs[False]
    assert any(r == "stop" for _, r in outs[True]) and any(r == "length" for _, r in outs[True])


def test_gpu_prefill_logits_vs_cpu(native, tiny_llama):
    cfg, sd = tiny_llama
    from rag_llm_k8s_amd.models.llama import StepInput
    from rag_llm_k8s_amd.ops.backend import AttnMeta
    from rag_llm_k8s_amd.ops.native import build_prefill_tiles

    outs = {}
    for dev in ("cuda", "cpu"):
        eng = _engine(cfg, sd, dev, graphs=False)
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
    rel = ((outs["cuda"] - outs["cpu"]).norm() / outs["cpu"].norm()).item()
    assert rel < 3e-2, rel


def test_encoder_gpu_vs_cpu(native):
    cfg = E.EncoderConfig(vocab_size=1000, hidden_size=384, num_hidden_layers=2, num_attention_heads=12,
                          intermediate_size=1536, max_position_embeddings=512)
    sd = encoder_state_dict(cfg, seed=2, std=0.05)
    lens = [7, 64, 200, 1]
    ids = torch.cat([torch.randint(0, 1000, (n,)) for n in lens]).int()
    res = {}
    for dev in ("cuda", "cpu"):
        m = E.EncoderModel(cfg, E.EncoderWeights.from_state_dict(cfg, sd, dev), dev)
        res[dev] = m.forward_packed(ids.to(dev), lens).cpu()
    cos = torch.nn.functional.cosine_similarity(res["cuda"], res["cpu"], dim=-1)
    assert cos.min().item() > 0.995, cos


def test_tiny_rag_workload_end_to_end(native):
    from rag_llm_k8s_amd.utils.smoke import run_smoke

    run_smoke("cuda:0")


def test_mixed_steps_gpu_close_to_separate(native, tiny_llama):
    """Mixed prefill+decode steps on the GPU: decoding rows computed inside prefill steps (prefill
    attention / tile GEMM path) still produce (near-)argmax greedy tokens under the fp32 oracle, for
    staggered arrivals; every KV block comes back."""
    cfg, sd = tiny_llama
    torch.manual_seed(6)
    prompts = [torch.randint(3, 1000, (n,)).tolist() for n in (30, 200, 64, 150)]
    p = SamplingParams(max_new_tokens=6, do_sample=False, ignore_eos=True)
    outs, mixed = {}, {}
    for m in (False, True):
        eng = _engine(cfg, sd, "cuda", graphs=True, mb=4)
        eng.mixed_steps = m
        eng.max_prefill_tokens = 128
        seqs = []
        for pr in prompts:  # staggered: each new prompt is prefilled while the earlier ones decode
            seqs.append(eng.add_request(pr, p, seed=1))
            for _ in range(2):
                eng.step()
        eng.run_until_done()
        assert eng._inflight is None and not eng.running and eng.bm.free_blocks() == 64 - 1
        outs[m] = [s.out for s in seqs]
        mixed[m] = eng.stats.get("mixed_decode_tokens", 0)
    assert mixed[True] > 0 and mixed[False] == 0
    for m in (False, True):  # every token of both runs is a (near-)argmax of the fp32 oracle
        _check_greedy(cfg, sd, prompts, outs[m])
