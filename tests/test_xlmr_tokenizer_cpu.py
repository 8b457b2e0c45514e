"""bge-m3 / XLM-R tokenizer path on the CPU: the synthetic SentencePiece Unigram tokenizer.json
(Precompiled nmt_nfkc charsmap + Metaspace + <s> $A </s>, XLM-R special ids) encodes identically in
the native runtime tokenizer and in HF tokenizers, and truncation keeps the trailing </s>."""
import numpy as np
import pytest

pytest.importorskip("sentencepiece")


def test_xlmr_unigram_runtime_matches_hf(tmp_path):
    from tokenizers import Tokenizer as HFTokenizer

    from rag_llm_k8s_amd.runtime.tokenizer import Tokenizer
    from rag_llm_k8s_amd.utils.synthetic import WordModel, train_xlmr_unigram_tokenizer

    wm = WordModel(n_words=8000, seed=4)
    train_xlmr_unigram_tokenizer(str(tmp_path), wm, corpus_words=80_000, vocab=1500)
    hf = HFTokenizer.from_file(str(tmp_path / "tokenizer.json"))
    ours = Tokenizer(str(tmp_path))
    rng = np.random.default_rng(1)
    texts = [wm.text(n, rng) for n in (1, 12, 300)] + ["Ｆｕｌｌｗｉｄｔｈ ＡＢＣ café ™ ½  two  spaces", ""]
    ref = [hf.encode(t).ids for t in texts]
    assert ours.encode_batch(texts, add_special_tokens=True) == ref
    assert all(r[0] == 0 and r[-1] == 2 for r in ref)
    assert [hf.token_to_id(t) for t in ("<s>", "<pad>", "</s>", "<unk>")] == [0, 1, 2, 3]
    cut = ours.encode(texts[2], add_special_tokens=True, max_length=64)
    assert len(cut) == 64 and cut[-1] == 2 and cut[:63] == ref[2][:63]
