"""Host-code sanitizer tier (SURVEY §5 "Race detection / sanitizers"): the C++ runtime
(csrc/runtime: tokenizers, JSON, safetensors mmap reader, faiss I/O, KV block manager) built as a
standalone executable with AddressSanitizer + UndefinedBehaviorSanitizer and driven over fixtures
written here. Device sanitizers are not available on the GPU pool, so GPU kernels are covered by
host-side shape checks (ops/native.py) and the numerics tests instead.

Token ids from the sanitized build are also compared with HF `tokenizers` (the oracle).
"""
import os
import subprocess

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
RT = os.path.join(ROOT, "csrc", "runtime")
SRC = [os.path.join(ROOT, "tests", "cpp", "runtime_selftest.cpp"), os.path.join(RT, "tokenizer.cpp"),
       os.path.join(RT, "runtime.cpp")]
EXE = os.path.join(ROOT, "build", "asan", "runtime_selftest")
TSAN_EXE = os.path.join(ROOT, "build", "tsan", "runtime_selftest")
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:halt_on_error=1",
           UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")


def _build(path, san_flags):
    deps = SRC + [os.path.join(RT, h) for h in os.listdir(RT) if h.endswith(".h")]
    if not os.path.exists(path) or any(os.path.getmtime(s) > os.path.getmtime(path) for s in deps):
        os.makedirs(os.path.dirname(path), exist_ok=True)
        cmd = ["g++", "-std=c++17", "-O1", "-g", "-pthread", "-fno-omit-frame-pointer"] + san_flags + \
            ["-I" + RT] + SRC + ["-o", path]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
        assert r.returncode == 0, r.stderr[-4000:]
    return path


@pytest.fixture(scope="module")
def exe():
    return _build(EXE, ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined"])


@pytest.fixture(scope="module")
def tsan_exe():
    return _build(TSAN_EXE, ["-fsanitize=thread"])


def run(exe, *args):
    r = subprocess.run([exe] + [str(a) for a in args], capture_output=True, text=True, timeout=600, env=ENV)
    assert "Sanitizer" not in r.stderr and "runtime error" not in r.stderr, r.stderr[-4000:]
    assert r.returncode == 0, (r.returncode, r.stderr[-2000:])
    return r.stdout


TEXTS = ["Hello world! The quick brown fox's 42 jumps.", "  leading spaces and\ttabs", "I'M YOU'RE 1234567",
         "ｆｕｌｌｗｉｄｔｈ ① ㈱ ﬁ ｶﾀｶﾅ 👨‍👩‍👧 🇯🇵",
         "unicode: café naïve Übermaß 東京 😀🚀", "", "a" * 300, "newline-free line with trailing space "]


@pytest.fixture(scope="module")
def tokenizers_(tmp_path_factory):
    from tokenizers import Regex, Tokenizer, decoders, models, pre_tokenizers, trainers

    from rag_llm_k8s_amd.utils.synthetic import WordModel

    d = tmp_path_factory.mktemp("tok")
    wm = WordModel(n_words=5000, seed=5)
    lines = wm.corpus_lines(20000) + TEXTS * 20
    out = {}
    # Llama-3 style byte-level BPE
    pat = (r"(?i:'s|'t|'re|'ve|'m|'ll|'d)|[^\r\n\p{L}\p{N}]?\p{L}+|\p{N}{1,3}| ?[^\s\p{L}\p{N}]+[\r\n]*|\s*[\r\n]+"
           r"|\s+(?!\S)|\s+")
    bpe = Tokenizer(models.BPE(ignore_merges=True))
    bpe.pre_tokenizer = pre_tokenizers.Sequence([pre_tokenizers.Split(Regex(pat), behavior="isolated"),
                                                 pre_tokenizers.ByteLevel(add_prefix_space=False, use_regex=False)])
    bpe.decoder = decoders.ByteLevel()
    bpe.train_from_iterator(lines, trainers.BpeTrainer(vocab_size=2000, show_progress=False,
                                                       initial_alphabet=pre_tokenizers.ByteLevel.alphabet()))
    out["bpe"] = bpe
    uni = Tokenizer(models.Unigram())
    uni.pre_tokenizer = pre_tokenizers.Metaspace()
    uni.decoder = decoders.Metaspace()
    uni.train_from_iterator(lines, trainers.UnigramTrainer(vocab_size=1500, show_progress=False, unk_token="<unk>",
                                                           special_tokens=["<unk>"]))
    out["unigram"] = uni
    try:  # XLM-R style Precompiled (SentencePiece nmt_nfkc charsmap) normalizer: trie walks under ASan
        import sentencepiece as spm
        from sentencepiece import sentencepiece_model_pb2 as pb
        from tokenizers import normalizers

        (d / "c.txt").write_text("\n".join(lines), encoding="utf-8")
        spm.SentencePieceTrainer.train(input=str(d / "c.txt"), model_prefix=str(d / "m"), vocab_size=800,
                                       model_type="unigram", normalization_rule_name="nmt_nfkc",
                                       character_coverage=1.0, minloglevel=2)
        proto = pb.ModelProto()
        proto.ParseFromString((d / "m.model").read_bytes())
        pc = Tokenizer(models.Unigram([(p.piece, p.score) for p in proto.pieces], unk_id=proto.trainer_spec.unk_id))
        pc.normalizer = normalizers.Sequence([normalizers.Precompiled(proto.normalizer_spec.precompiled_charsmap),
                                              normalizers.Replace(Regex(" {2,}"), " ")])
        pc.pre_tokenizer = pre_tokenizers.Metaspace()
        pc.decoder = decoders.Metaspace()
        out["precompiled"] = pc
    except ImportError:
        pass
    paths = {}
    for k, t in out.items():
        p = str(d / ("%s.json" % k))
        t.save(p)
        paths[k] = p
    return out, paths, str(d)


def test_tokenizers_under_asan_match_hf(exe, tokenizers_):
    toks, paths, d = tokenizers_
    texts = os.path.join(d, "texts.txt")
    with open(texts, "w", encoding="utf-8") as f:
        f.write("\n".join(TEXTS) + "\n")
    for k, tok in toks.items():
        got = run(exe, "tok", paths[k], texts).splitlines()
        for t, line in zip(TEXTS, got):
            ids = [int(x) for x in line.split()] if line.strip() else []
            assert ids == tok.encode(t, add_special_tokens=True).ids, (k, t)


def test_tokenizer_threads_under_asan_and_tsan(exe, tsan_exe, tokenizers_):
    """encode_batch (8 worker threads sharing the BPE word cache) == sequential encode; ThreadSanitizer
    build must report no data race (the race detection tier of SURVEY §5)."""
    _, paths, d = tokenizers_
    texts = os.path.join(d, "texts.txt")
    with open(texts, "w", encoding="utf-8") as f:
        f.write("\n".join(TEXTS) + "\n")
    for k, p in paths.items():
        assert "tokmt ok" in run(exe, "tokmt", p, texts)
        r = subprocess.run([tsan_exe, "tokmt", p, texts], capture_output=True, text=True, timeout=600,
                           env=dict(os.environ, TSAN_OPTIONS="halt_on_error=1"))
        assert "ThreadSanitizer" not in r.stderr and r.returncode == 0, r.stderr[-3000:]


def test_tokenizer_fuzz_under_asan(exe, tokenizers_):
    _, paths, _ = tokenizers_
    for k, p in paths.items():
        assert "fuzz ok" in run(exe, "fuzz", p, 7, 400)


def test_safetensors_faiss_blockmanager_json_under_asan(exe, tmp_path):
    from safetensors.torch import save_file

    from rag_llm_k8s_amd.index import faiss_io

    t = {"w": torch.randn(9, 13).bfloat16(), "v": torch.arange(7, dtype=torch.int32), "m": torch.randn(4, 5)}
    p = str(tmp_path / "x.safetensors")
    save_file(t, p)
    out = run(exe, "st", p)
    assert len(out.splitlines()) == 3
    xb = np.random.default_rng(0).standard_normal((17, 8)).astype(np.float32)
    a, b = str(tmp_path / "idx"), str(tmp_path / "idx.rt")
    faiss_io.atomic_write(a, lambda f: faiss_io.write_flat_l2(f, xb))
    assert run(exe, "faiss", a, b).split() == ["8", "17"]
    assert open(a, "rb").read() == open(b, "rb").read()
    # truncated file: must fail cleanly (exception -> exit 2), never read out of bounds
    with open(b, "r+b") as f:
        f.truncate(50)
    r = subprocess.run([exe, "faiss", b, b + ".2"], capture_output=True, text=True, env=ENV, timeout=60)
    assert r.returncode == 2 and "Sanitizer" not in r.stderr
    for seed in (1, 2, 3):
        assert "bm ok" in run(exe, "bm", seed)
    assert "json threw" in run(exe, "json")
