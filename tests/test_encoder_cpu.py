"""T2 encoder parity on CPU: the packed-varlen encoder (models/encoder.py) vs
transformers' BertModel / XLMRobertaModel with the same random-init weights, pooled (mean for the
MiniLM-style BERT, CLS for bge-m3's XLM-R) and L2-normalised as sentence-transformers does.
HF runs in fp32 on the bf16-rounded weights; ours keeps bf16 activations (kernel rounding points)."""
import pytest
import torch

transformers = pytest.importorskip("transformers")

from rag_llm_k8s_amd.models import encoder as E  # noqa: E402


def _hf_model(kind):
    common = dict(vocab_size=300, hidden_size=64, num_hidden_layers=2, num_attention_heads=4, intermediate_size=128,
                  hidden_act="gelu", hidden_dropout_prob=0.0, attention_probs_dropout_prob=0.0)
    if kind == "bert":
        cfg = transformers.BertConfig(max_position_embeddings=64, type_vocab_size=2, layer_norm_eps=1e-12,
                                      pad_token_id=0, **common)
        model = transformers.BertModel(cfg, add_pooling_layer=False)
    else:
        cfg = transformers.XLMRobertaConfig(max_position_embeddings=66, type_vocab_size=1, layer_norm_eps=1e-5,
                                            pad_token_id=1, **common)
        model = transformers.XLMRobertaModel(cfg, add_pooling_layer=False)
    torch.manual_seed(7)
    with torch.no_grad():  # wider than the default init so the layers do visible work
        for p in model.parameters():
            p.normal_(0.0, 0.08)
        for n, p in model.named_parameters():
            if "LayerNorm.weight" in n:
                p.add_(1.0)
            p.copy_(p.to(torch.bfloat16).float())  # the weights ours will hold
    model.eval()
    # "eager" attention: the SDPA path is fine too, eager keeps the oracle simple
    model.config._attn_implementation = "eager"
    return cfg, model


@pytest.mark.parametrize("kind,pooling", [("bert", "mean"), ("xlm-roberta", "cls")])
def test_encoder_matches_transformers(kind, pooling):
    hf_cfg, model = _hf_model(kind)
    cfg = E.EncoderConfig.from_dict(hf_cfg.to_dict(), pooling=pooling, max_seq_length=60)
    sd = {k: v.detach().clone() for k, v in model.state_dict().items()}
    ours = E.EncoderModel(cfg, E.EncoderWeights.from_state_dict(cfg, sd, "cpu"), "cpu")

    lens = [7, 12, 3, 1]
    g = torch.Generator().manual_seed(3)
    seqs = [torch.randint(3, cfg.vocab_size, (L,), generator=g) for L in lens]  # no pad id inside
    got = ours.forward_packed(torch.cat(seqs).to(torch.int32), lens).float()

    B, Lm = len(lens), max(lens)
    ids = torch.full((B, Lm), cfg.pad_token_id, dtype=torch.long)
    mask = torch.zeros((B, Lm), dtype=torch.long)
    for i, s in enumerate(seqs):
        ids[i, :len(s)] = s
        mask[i, :len(s)] = 1
    with torch.no_grad():
        hs = model(input_ids=ids, attention_mask=mask).last_hidden_state
    if pooling == "cls":
        ref = hs[:, 0]
    else:
        m = mask.unsqueeze(-1).float()
        ref = (hs * m).sum(1) / m.sum(1)
    ref = torch.nn.functional.normalize(ref, dim=-1)

    assert got.shape == ref.shape
    cos = torch.nn.functional.cosine_similarity(got, ref, dim=-1)
    assert cos.min().item() > 0.995, cos
    assert torch.allclose(got.norm(dim=-1), torch.ones(B), atol=1e-3)
    assert ((got - ref).norm() / ref.norm()).item() < 5e-2
