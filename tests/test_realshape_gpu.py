"""Numerics at the shapes the bench runs (not tiny models), against plain fp32 PyTorch oracles:

* Llama-3.1-8B layer widths (hidden 4096, 32 q / 8 kv heads of 128, MLP 14336, Llama-3 RoPE scaling;
  2 layers, small vocabulary) serving a 5.2k-token RAG prompt through chunked prefill (2048-token
  chunks: later chunks attend to a longer KV history, 82 KV blocks), then greedy decode; every token is
  checked against transformers' LlamaForCausalLM in fp32 on the same bf16-rounded weights with the
  per-step top-1 margin rule (teacher forced).
* bge-m3: XLM-R embeddings (position ids offset by padding_idx + 1, one token type, LN eps 1e-5) at
  bge-m3 widths (1024 / 16 heads / 4096), CLS pooling, with an XLM-R SentencePiece Unigram tokenizer
  (Precompiled nmt_nfkc charsmap) on texts up to ~3k tokens; tokenizer ids vs HF tokenizers and
  embeddings vs transformers' XLMRobertaModel in fp32.
Reference behaviour: /root/reference/llm/rag.py:50-58 (embedder + Llama generate)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
transformers = pytest.importorskip("transformers")

DEV = "cuda:0"


def test_llama_8b_width_chunked_prefill_5k_greedy_vs_hf_fp32(native):
    from rag_llm_k8s_amd.engine.llm_engine import LLMEngine, SamplingParams
    from rag_llm_k8s_amd.models import llama as L
    from rag_llm_k8s_amd.utils.synthetic import llama_state_dict

    cfg = L.llama31_8b()
    cfg.vocab_size, cfg.num_hidden_layers, cfg.bos_token_id, cfg.eos_token_id = 2048, 2, 1, [2]
    sd = llama_state_dict(cfg, seed=0, std=0.02)
    g = torch.Generator().manual_seed(5)
    prompt = torch.randint(3, cfg.vocab_size, (5200,), generator=g).tolist()
    m = L.LlamaModel(cfg, L.LlamaWeights.from_state_dict(cfg, sd, DEV), DEV, max_positions=8192)
    eng = LLMEngine(m, num_blocks=160, max_batch=2, max_prefill_tokens=2048, max_model_len=8192, use_graphs=False)
    out = eng.generate([prompt], SamplingParams(max_new_tokens=4, do_sample=False, ignore_eos=True))[0]
    assert eng.stats["prefill_steps"] >= 3  # 2048 + 2048 + 1104
    del eng, m
    torch.cuda.empty_cache()

    hf_cfg = transformers.LlamaConfig(**{k: v for k, v in cfg.to_hf_dict().items() if k != "architectures"})
    with torch.device(DEV):
        hf = transformers.LlamaForCausalLM(hf_cfg)
    hf.load_state_dict({k: v.float() for k, v in sd.items()})
    hf.eval()
    with torch.no_grad():
        lg = hf(input_ids=torch.tensor([prompt + out[:-1]], device=DEV)).logits[0].float().cpu()
    exact = 0
    for k, tok in enumerate(out):
        row = lg[len(prompt) - 1 + k]
        top, gap = float(row.max()), float(row.max() - row[tok])
        assert gap <= 0.02 * (top - float(row.min())), (k, tok, int(row.argmax()), gap)
        exact += int(gap == 0.0)
    assert exact >= 3, exact


def test_bge_m3_xlmr_unigram_vs_hf_fp32(native, tmp_path):
    from tokenizers import Tokenizer as HFTokenizer

    from rag_llm_k8s_amd.engine.encoder_engine import EmbeddingEngine
    from rag_llm_k8s_amd.models import encoder as E
    from rag_llm_k8s_amd.runtime.tokenizer import Tokenizer
    from rag_llm_k8s_amd.utils.synthetic import WordModel, encoder_state_dict, train_xlmr_unigram_tokenizer

    wm = WordModel(n_words=20000, seed=3)
    train_xlmr_unigram_tokenizer(str(tmp_path), wm, corpus_words=200_000, vocab=4000)
    rng = np.random.default_rng(0)
    texts = [wm.text(n, rng) for n in (5, 60, 700, 2200)] + ["Ｆｕｌｌｗｉｄｔｈ ＡＢＣ café ™ ½  two  spaces"]
    ours_tok = Tokenizer(str(tmp_path))
    hf_tok = HFTokenizer.from_file(str(tmp_path / "tokenizer.json"))
    ids = [hf_tok.encode(t).ids for t in texts]
    assert ours_tok.encode_batch(texts, add_special_tokens=True, max_length=8192) == ids
    assert all(i[0] == 0 and i[-1] == 2 for i in ids) and max(len(i) for i in ids) > 2000

    cfg = E.bge_m3()
    cfg.vocab_size, cfg.num_hidden_layers = 4000, 2
    sd = encoder_state_dict(cfg, seed=1, std=0.05)
    emb = EmbeddingEngine(E.EncoderModel(cfg, E.EncoderWeights.from_state_dict(cfg, sd, DEV), DEV), ours_tok)
    got = emb.embed(texts).float().cpu()

    hf_cfg = transformers.XLMRobertaConfig(vocab_size=4000, hidden_size=1024, num_hidden_layers=2,
                                           num_attention_heads=16, intermediate_size=4096, max_position_embeddings=8194,
                                           type_vocab_size=1, layer_norm_eps=1e-5, pad_token_id=1, hidden_act="gelu",
                                           hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
    with torch.device(DEV):
        hf = transformers.XLMRobertaModel(hf_cfg, add_pooling_layer=False)
    res = hf.load_state_dict({k: v.float() for k, v in sd.items()}, strict=False)
    assert not res.unexpected_keys and all(k.endswith(("position_ids", "token_type_ids")) for k in res.missing_keys)
    hf.eval()
    refs = []
    with torch.no_grad():
        for i in ids:
            hs = hf(input_ids=torch.tensor([i], device=DEV)).last_hidden_state[0, 0]
            refs.append(torch.nn.functional.normalize(hs.float(), dim=-1).cpu())
    ref = torch.stack(refs)
    cos = torch.nn.functional.cosine_similarity(got, ref, dim=-1)
    assert cos.min().item() > 0.995, cos
