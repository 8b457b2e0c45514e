"""C++ host runtime (_ragk_rt): tokenizers vs HF `tokenizers` (oracle), safetensors mmap reader
vs the `safetensors` package, faiss IxF2 I/O vs the Python writer, KV block manager vs PyBlockManager."""
import os

import numpy as np
import pytest
import torch

from rag_llm_k8s_amd.utils.synthetic import WordModel

LLAMA3_PAT = (r"(?i:'s|'t|'re|'ve|'m|'ll|'d)|[^\r\n\p{L}\p{N}]?\p{L}+|\p{N}{1,3}| ?[^\s\p{L}\p{N}]+[\r\n]*|"
              r"\s*[\r\n]+|\s+(?!\S)|\s+")

TEXTS = [
    "Hello world! It's a test: don't STOP, we'll see.  Double  spaces\tand\ttabs.\n\nNew paragraph 12345 678.",
    "Ünïcödé café naïve résumé — “quotes” ‘single’ … 漢字テスト 한국어 текст ١٢٣ 𝔘𝔫𝔦",
    "   leading spaces and trailing   ",
    "line1\r\nline2\n  \n\tindented\n",
    "a1b2c3 x=y+z (paren) [brack] {brace} <tag> #hash @at $5.00 50% 3.14159e-10",
    "I'M YOU'RE THEY'VE WE'D SHE'LL IT'S",
    "",
    "emoji 😀🚀 mixed👍text",
]


@pytest.fixture(scope="module")
def rt():
    from rag_llm_k8s_amd import _build
    from rag_llm_k8s_amd.runtime import native_rt

    _build.build_runtime()
    import rag_llm_k8s_amd.runtime as R

    R._tried = False
    m = native_rt()
    assert m is not None
    return m


@pytest.fixture(scope="module")
def corpus():
    wm = WordModel(n_words=30000, seed=3)
    lines = wm.corpus_lines(200000)
    return wm, lines + TEXTS * 50


def _check(rt, tok, path, texts, add_special=True):
    n = rt.Tokenizer(path)
    for t in texts:
        ref = tok.encode(t, add_special_tokens=add_special).ids
        got = n.encode(t, add_special)
        assert got == ref, (t[:80], got[:20], ref[:20])
        assert n.decode(got, True) == tok.decode(ref, skip_special_tokens=True), t[:80]
    assert n.vocab_size() == tok.get_vocab_size(with_added_tokens=True)


def test_bpe_gpt2_regex(rt, corpus, tmp_path):
    from tokenizers import Tokenizer, decoders, models, pre_tokenizers, trainers

    wm, lines = corpus
    tok = Tokenizer(models.BPE())
    tok.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False)
    tok.decoder = decoders.ByteLevel()
    tok.train_from_iterator(lines, trainers.BpeTrainer(vocab_size=4000, show_progress=False,
                                                       initial_alphabet=pre_tokenizers.ByteLevel.alphabet()))
    p = str(tmp_path / "gpt2.json")
    tok.save(p)
    _check(rt, tok, p, TEXTS + [wm.text(300) for _ in range(20)])


def test_bpe_llama3_split_regex_with_specials(rt, corpus, tmp_path):
    from tokenizers import AddedToken, Regex, Tokenizer, decoders, models, pre_tokenizers, processors, trainers

    wm, lines = corpus
    tok = Tokenizer(models.BPE(ignore_merges=True))
    tok.pre_tokenizer = pre_tokenizers.Sequence([
        pre_tokenizers.Split(Regex(LLAMA3_PAT), behavior="isolated", invert=False),
        pre_tokenizers.ByteLevel(add_prefix_space=False, use_regex=False)])
    tok.decoder = decoders.ByteLevel()
    tok.train_from_iterator(lines, trainers.BpeTrainer(vocab_size=6000, show_progress=False,
                                                       initial_alphabet=pre_tokenizers.ByteLevel.alphabet()))
    tok.add_special_tokens([AddedToken("<|begin_of_text|>", special=True), AddedToken("<|eot_id|>", special=True)])
    bos = tok.token_to_id("<|begin_of_text|>")
    tok.post_processor = processors.TemplateProcessing(single="<|begin_of_text|> $A",
                                                       special_tokens=[("<|begin_of_text|>", bos)])
    p = str(tmp_path / "llama3.json")
    tok.save(p)
    texts = TEXTS + [wm.text(200) + " <|eot_id|> tail" for _ in range(10)] + ["<|begin_of_text|>x<|eot_id|>"]
    _check(rt, tok, p, texts)
    _check(rt, tok, p, texts, add_special=False)
    # long prompts: the front end cuts them at pre-token boundaries and encodes the pieces in parallel
    from rag_llm_k8s_amd.runtime.tokenizer import Tokenizer as FrontTok

    ft = FrontTok(p, backend="native")
    longs = [" ".join(TEXTS) * 12, "\n\n".join(wm.text(400) for _ in range(12)) + " <|eot_id|> Question: why?",
             "x" * 9000, " ".join(["word"] * 3000), "Ünïcödé café " * 700]
    for t in longs:
        assert len(t) >= ft.SPLIT_MIN_CHARS
        for sp in (True, False):
            assert ft.encode(t, add_special_tokens=sp) == tok.encode(t, add_special_tokens=sp).ids, (t[:40], sp)
    assert ft._split_ok()
    # encode_batch of fewer texts than workers (C=1) cuts the long ones the same way, short ones mixed in
    for batch in ([longs[1]], longs[:3], [longs[0], "short text", longs[4]]):
        for sp in (True, False):
            want = [e.ids for e in tok.encode_batch(batch, add_special_tokens=sp)]
            assert [list(x) for x in ft.encode_batch(batch, add_special_tokens=sp)] == want, (len(batch), sp)


def test_encode_batch_concurrent_callers(rt, corpus, tmp_path):
    """Several Python threads in encode_batch at once (the server tokenizes long prompts on the shared
    C++ worker pool while the batcher encodes): every caller gets its own correct result."""
    import threading

    from tokenizers import Tokenizer, decoders, models, pre_tokenizers, trainers

    wm, lines = corpus
    tok = Tokenizer(models.BPE())
    tok.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False)
    tok.decoder = decoders.ByteLevel()
    tok.train_from_iterator(lines[:20000], trainers.BpeTrainer(vocab_size=2000, show_progress=False,
                                                               initial_alphabet=pre_tokenizers.ByteLevel.alphabet()))
    p = str(tmp_path / "bpe.json")
    tok.save(p)
    n = rt.Tokenizer(p)
    batches = [[wm.text(50 + 7 * i + j) for j in range(24)] for i in range(6)]
    refs = [[e.ids for e in tok.encode_batch(b)] for b in batches]
    errs = []

    def worker(i):
        try:
            for _ in range(20):
                if n.encode_batch(batches[i], True, 8, -1) != refs[i]:
                    errs.append(i)
                    return
        except Exception as e:  # noqa: BLE001
            errs.append(repr(e))

    th = [threading.Thread(target=worker, args=(i,)) for i in range(6)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs, errs


def test_wordpiece_bert(rt, corpus, tmp_path):
    from rag_llm_k8s_amd.utils.synthetic import train_wordpiece_tokenizer

    wm, lines = corpus
    d = str(tmp_path / "wp")
    tok = train_wordpiece_tokenizer(d, wm, corpus_words=100000, vocab=3000)
    _check(rt, tok, os.path.join(d, "tokenizer.json"), TEXTS + [wm.text(150) for _ in range(10)])


def test_unigram_metaspace(rt, corpus, tmp_path):
    from tokenizers import Tokenizer, decoders, models, pre_tokenizers, trainers

    wm, lines = corpus
    tok = Tokenizer(models.Unigram())
    tok.pre_tokenizer = pre_tokenizers.Metaspace()
    tok.decoder = decoders.Metaspace()
    tok.train_from_iterator(lines[:3000], trainers.UnigramTrainer(vocab_size=2000, show_progress=False,
                                                                 special_tokens=["<unk>"], unk_token="<unk>"))
    p = str(tmp_path / "uni.json")
    tok.save(p)
    texts = [wm.text(60) for _ in range(20)] + ["hello world", "zzqqxx unknownchars"]
    n = rt.Tokenizer(p)
    agree = 0
    for t in texts:
        ref = tok.encode(t).ids
        got = n.encode(t, True)
        agree += int(got == ref)
        assert n.decode(got, True) == tok.decode(ref)
    assert agree >= len(texts) - 2  # Viterbi ties may break differently


def test_native_wrapper_used_by_default(rt, corpus, tmp_path):
    from rag_llm_k8s_amd.runtime.tokenizer import Tokenizer as W
    from rag_llm_k8s_amd.utils.synthetic import train_small_bpe

    wm, _ = corpus
    d = str(tmp_path / "small")
    train_small_bpe(d, 600, wm)
    a, b = W(d, backend="native"), W(d, backend="hf")
    assert a.backend == "native" and b.backend == "hf"
    for t in TEXTS:
        assert a.encode(t) == b.encode(t)
        assert a.decode(a.encode(t)) == b.decode(b.encode(t))
    assert a.bos_id == b.bos_id


def test_safetensors_reader(rt, tmp_path):
    from safetensors.torch import save_file

    t = {"a": torch.randn(5, 7).bfloat16(), "b": torch.arange(12, dtype=torch.int64).reshape(3, 4),
         "c": torch.randn(3)}
    p = str(tmp_path / "x.safetensors")
    save_file(t, p, metadata={"format": "pt"})
    st = rt.SafeTensors(p)
    assert sorted(st.keys()) == ["a", "b", "c"] and st.metadata()["format"] == "pt"
    a = torch.from_numpy(st.view("a").copy()).view(torch.bfloat16)
    assert torch.equal(a, t["a"])
    assert torch.equal(torch.from_numpy(st.view("b").copy()), t["b"])
    sl = torch.from_numpy(st.slice("a", 1, 4, 2, 6)).view(torch.bfloat16)
    assert torch.equal(sl, t["a"][1:4, 2:6])
    assert torch.equal(torch.from_numpy(st.slice("b", 1, 3)), t["b"][1:3])
    # the Python reader prefers / matches the native one
    from rag_llm_k8s_amd.runtime.safetensors_io import SafeFile

    sf = SafeFile(p)
    assert torch.equal(sf.get("a", rows=(1, 4), cols=(2, 6)), t["a"][1:4, 2:6])


def test_faiss_io_native_vs_python(rt, tmp_path):
    from rag_llm_k8s_amd.index import faiss_io

    xb = np.random.default_rng(0).standard_normal((11, 6)).astype(np.float32)
    p1, p2 = str(tmp_path / "a"), str(tmp_path / "b")
    rt.write_flat_index(p1, xb)
    faiss_io.atomic_write(p2, lambda f: faiss_io.write_flat_l2(f, xb))
    assert open(p1, "rb").read() == open(p2, "rb").read()
    d, n, metric, x = rt.read_flat_index(p2)
    assert (d, n, metric) == (6, 11, 1) and np.array_equal(x, xb)
    with open(p1, "r+b") as f:
        f.truncate(40)
    with pytest.raises(RuntimeError):
        rt.read_flat_index(p1)


def test_block_manager_native_matches_python(rt):
    from rag_llm_k8s_amd.engine.kv_manager import PyBlockManager

    a, b = rt.BlockManager(20, True), PyBlockManager(20)
    rng = np.random.default_rng(1)
    live = set()
    for step in range(300):
        if live and rng.random() < 0.4:
            s = int(rng.choice(sorted(live)))
            a.free(s)
            b.free(s)
            live.discard(s)
        else:
            s = int(rng.integers(0, 8))
            n = int(rng.integers(1, 300))
            assert a.can_allocate(s, n) == b.can_allocate(s, n)
            if b.can_allocate(s, n):
                assert a.ensure(s, n) == b.ensure(s, n)
                live.add(s)
        assert a.free_blocks() == b.free_blocks()
        for s in live:
            assert a.table(s) == b.table(s)
    with pytest.raises(RuntimeError):
        a.ensure(99, 10 ** 6)


PC_TEXTS = ["Hello world café naïve Übermaß", "ｆｕｌｌｗｉｄｔｈ ＡＢＣ １２３", "① ② ㈱ ﬁ ﬂ ligature ™ ½",
            "東京 タワー ｶﾀｶﾅ ｸﾞ", "é ä ñ combining", "multiple   spaces\tand\ttabs  ",
            "emoji 👍🏽 👨‍👩‍👧 🇯🇵 flags", " nbsp emsp　ideo", "  leading and trailing  ",
            "Ⅻ ㎏ ㎡ ℃ № …", ""]


def test_unigram_precompiled_charsmap_matches_hf(rt, tmp_path):
    """XLM-R / bge-m3 style: SentencePiece nmt_nfkc charsmap (Precompiled normalizer) + Unigram;
    oracle = HF tokenizers (Rust) on a tokenizer.json assembled like transformers' SpmConverter."""
    spm = pytest.importorskip("sentencepiece")
    from sentencepiece import sentencepiece_model_pb2 as pb
    from tokenizers import Regex, Tokenizer, decoders, models, normalizers, pre_tokenizers

    from rag_llm_k8s_amd.utils.synthetic import WordModel

    wm = WordModel(n_words=3000, seed=9)
    lines = wm.corpus_lines(4000) + PC_TEXTS * 30
    corpus = tmp_path / "c.txt"
    corpus.write_text("\n".join(lines), encoding="utf-8")
    spm.SentencePieceTrainer.train(input=str(corpus), model_prefix=str(tmp_path / "m"), vocab_size=1200,
                                   model_type="unigram", normalization_rule_name="nmt_nfkc",
                                   character_coverage=1.0, minloglevel=2)
    proto = pb.ModelProto()
    proto.ParseFromString((tmp_path / "m.model").read_bytes())
    charsmap = proto.normalizer_spec.precompiled_charsmap
    assert len(charsmap) > 1000
    vocab = [(p.piece, p.score) for p in proto.pieces]
    for seq in ([normalizers.Precompiled(charsmap), normalizers.Replace(Regex(" {2,}"), " ")],
                [normalizers.Precompiled(charsmap), normalizers.Strip(left=False, right=True),
                 normalizers.Replace(Regex(" {2,}"), "▁")]):
        tok = Tokenizer(models.Unigram(vocab, unk_id=proto.trainer_spec.unk_id))
        tok.normalizer = normalizers.Sequence(seq)
        tok.pre_tokenizer = pre_tokenizers.Metaspace()
        tok.decoder = decoders.Metaspace()
        p = str(tmp_path / "tokenizer.json")
        tok.save(p)
        n = rt.Tokenizer(p)
        for t in PC_TEXTS + [wm.text(60) for _ in range(5)]:
            assert n.encode(t, False) == tok.encode(t, add_special_tokens=False).ids, t


def test_truncated_encode_equals_full_then_truncate(rt, corpus, tmp_path):
    """Budgeted native encode (stops once max_length body tokens exist; encoder ingest truncates 1000-word
    chunks to 256/512 tokens) == full encode + right truncation keeping the trailing special, for
    WordPiece (BERT), byte-level BPE with specials, and XLM-R Unigram."""
    from rag_llm_k8s_amd.runtime.tokenizer import Tokenizer
    from rag_llm_k8s_amd.utils.synthetic import train_wordpiece_tokenizer, train_xlmr_unigram_tokenizer

    wm, lines = corpus
    dirs = [str(tmp_path / "wp"), str(tmp_path / "uni")]
    train_wordpiece_tokenizer(dirs[0], wm, corpus_words=60000, vocab=2000)
    train_xlmr_unigram_tokenizer(dirs[1], wm, corpus_words=60000, vocab=1200)
    texts = TEXTS + [wm.text(n) for n in (3, 40, 400)]
    for d in dirs:
        nat = Tokenizer(d, backend="native")
        hf = Tokenizer(d, backend="hf")
        assert nat.backend == "native"
        for L in (1, 2, 3, 7, 64, 100000):
            got = nat.encode_batch(texts, add_special_tokens=True, max_length=L)
            ref = hf.encode_batch(texts, add_special_tokens=True, max_length=L)
            assert got == ref, (d, L)
            assert [nat.encode(t, True, max_length=L) for t in texts] == ref
            assert nat.encode_batch(texts, add_special_tokens=False, max_length=L) == \
                hf.encode_batch(texts, add_special_tokens=False, max_length=L)
