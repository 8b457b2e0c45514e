"""Embedding engine ingest path (engine/encoder_engine.py): flat truncated tokenisation, greedy varlen
packing and the tokenise/encode pipeline give the same embeddings, in input order, as embedding each
text alone (the reference embeds one chunk at a time, /root/reference/llm/rag.py:54-55,100-101)."""
import numpy as np
import torch


def test_pipelined_embed_equals_one_by_one(tmp_path, monkeypatch):
    from rag_llm_k8s_amd.engine import encoder_engine as EE
    from rag_llm_k8s_amd.models import encoder as E
    from rag_llm_k8s_amd.runtime.tokenizer import Tokenizer
    from rag_llm_k8s_amd.utils.synthetic import WordModel, train_wordpiece_tokenizer

    wm = WordModel(n_words=5000, seed=2)
    train_wordpiece_tokenizer(str(tmp_path), wm, corpus_words=50000, vocab=1500)
    cfg = E.EncoderConfig(vocab_size=1500, hidden_size=64, num_hidden_layers=1, num_attention_heads=4,
                          intermediate_size=128, max_seq_length=48)
    model = E.EncoderModel(cfg, E.EncoderWeights.random(cfg, "cpu", seed=3), "cpu")
    emb = EE.EmbeddingEngine(model, Tokenizer(str(tmp_path)), max_batch_tokens=700)
    rng = np.random.default_rng(0)
    texts = [wm.text(int(n), rng) for n in rng.integers(1, 80, 300)]  # some longer than max_seq_length
    monkeypatch.setattr(EE, "PIPELINE_GROUP", 64)  # 5 pipeline stages
    got = emb.embed(texts)
    ids, lens = emb.tokenize_flat(texts)
    assert int(lens.max()) == 48 and int(lens.min()) >= 3
    ref = torch.stack([model.forward_packed(torch.tensor(emb.tokenize([t])[0], dtype=torch.int32),
                                            [int(lens[i])])[0] for i, t in enumerate(texts)])
    assert got.shape == (300, 64)
    assert torch.allclose(got, ref, atol=2e-3), (got - ref).abs().max()
    assert torch.allclose(emb.embed_ids(emb.tokenize(texts)), got, atol=1e-5)
