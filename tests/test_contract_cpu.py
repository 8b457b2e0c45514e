"""T0 unit tier: exact reference semantics (chunking, prompt bytes, faiss file format, metadata, PDF)."""
import io
import os
import pickle
import struct

import numpy as np
import pytest
import torch

from rag_llm_k8s_amd.index import faiss_io
from rag_llm_k8s_amd.index.flat import FLT_MAX, FlatL2Index
from rag_llm_k8s_amd.ingest import pdf
from rag_llm_k8s_amd.ingest.text import SYSTEM_MESSAGE, build_context, build_prompt, postprocess, split_text


def ref_split_text(text, chunk_size=1000, overlap=200):  # literal re-statement of rag.py:39-45
    words = text.split()
    chunks = []
    for i in range(0, len(words), chunk_size - overlap):
        chunks.append(" ".join(words[i:i + chunk_size]))
    return chunks


@pytest.mark.parametrize("n", [0, 1, 799, 800, 801, 1000, 1001, 1600, 2401, 16200])
def test_split_text_matches_reference(n):
    text = "\n".join(("w%d" % i) + ("  " if i % 7 else "\t") for i in range(n))
    assert split_text(text) == ref_split_text(text)
    assert split_text(text, 10, 3) == ref_split_text(text, 10, 3)


def test_split_text_counts():
    # 16.2k words -> 21 windows (SURVEY R29 derivation), trailing window always emitted
    assert len(split_text(" ".join(["x"] * 16200))) == 21
    assert len(split_text(" ".join(["x"] * 1000))) == 2


def test_prompt_bytes():
    assert SYSTEM_MESSAGE.startswith("You are a helpful assistant. Answer the user's question based ONLY")
    assert SYSTEM_MESSAGE.count("\n") == 2
    res = [({"filename": "a.pdf", "chunk_id": 3, "text": "alpha"}, 0.123456),
           ({"filename": "b.pdf", "chunk_id": 0, "text": "beta"}, 1.0),
           ({"filename": "c.pdf", "chunk_id": 9, "text": "gamma"}, 2.5),
           ({"filename": "d.pdf", "chunk_id": 1, "text": "delta"}, 3.0)]
    ctx = build_context(res, 3)
    assert ctx == ("Document 'a.pdf' (chunk 3, score: 0.1235): alpha\n\n"
                   "Document 'b.pdf' (chunk 0, score: 1.0000): beta\n\n"
                   "Document 'c.pdf' (chunk 9, score: 2.5000): gamma\n\n")
    p = build_prompt(ctx, "what is wazero?")
    assert p == f"{SYSTEM_MESSAGE}\n\nContext: {ctx}\n\nUser: what is wazero?\n\nChatbot:"
    assert postprocess(p + " It is a runtime.  ") == "It is a runtime."
    assert postprocess("no marker here ") == "no marker here"


def test_faiss_flat_golden_bytes(tmp_path):
    xb = np.arange(6, dtype=np.float32).reshape(2, 3)
    buf = io.BytesIO()
    faiss_io.write_flat_l2(buf, xb)
    b = buf.getvalue()
    expect = (b"IxF2" + struct.pack("<i", 3) + struct.pack("<q", 2) + struct.pack("<q", 1 << 20) * 2 +
              b"\x01" + struct.pack("<i", 1) + struct.pack("<Q", 6) + xb.tobytes())
    assert b == expect
    r = faiss_io.read_index_stream(io.BytesIO(b))
    assert r["d"] == 3 and r["ntotal"] == 2 and np.array_equal(r["xb"], xb)
    # empty index (reference ensure_index_exists writes one)
    buf = io.BytesIO()
    faiss_io.write_flat_l2(buf, np.zeros((0, 1024), np.float32))
    assert len(buf.getvalue()) == 4 + 4 + 8 * 3 + 1 + 4 + 8
    with pytest.raises(ValueError):
        faiss_io.read_index_stream(io.BytesIO(b[:-3]))


def test_faiss_ivf_roundtrip():
    rng = np.random.default_rng(0)
    cents = rng.standard_normal((4, 8)).astype(np.float32)
    lists = [rng.standard_normal((n, 8)).astype(np.float32) for n in (3, 0, 5, 1)]
    ids = [np.arange(s, s + len(l), dtype=np.int64) for s, l in zip((0, 3, 3, 8), lists)]
    for ls, iss in ((lists, ids), ([lists[0]] + [np.zeros((0, 8), np.float32)] * 3,
                                   [ids[0]] + [np.zeros(0, np.int64)] * 3)):
        buf = io.BytesIO()
        faiss_io.write_ivf_flat(buf, 8, cents, ls, iss, nprobe=2)
        r = faiss_io.read_index_stream(io.BytesIO(buf.getvalue()))
        assert r["type"] == "ivf_flat" and r["nlist"] == 4 and r["nprobe"] == 2
        for a, b in zip(r["lists"], ls):
            assert np.array_equal(a, b)
        for a, b in zip(r["ids"], iss):
            assert np.array_equal(a, b)


def test_metadata_pickle_roundtrip_and_safety(tmp_path):
    p = str(tmp_path / "faiss_index.metadata")
    meta = [{"filename": "a.pdf", "chunk_id": 0, "text": "hello"}]
    faiss_io.save_metadata(p, meta)
    with open(p, "rb") as f:
        assert pickle.load(f) == meta  # readable by the reference's plain pickle.load
    assert faiss_io.load_metadata(p) == meta

    class Evil:
        def __reduce__(self):
            return (os.system, ("echo pwned",))

    with open(p, "wb") as f:
        pickle.dump([Evil()], f)
    with pytest.raises(pickle.UnpicklingError):
        faiss_io.load_metadata(p)


def test_flat_index_cpu_semantics():
    idx = FlatL2Index(4)
    D, I = idx.search(torch.zeros(1, 4), 3)
    assert I.tolist() == [[-1, -1, -1]] and D[0, 0].item() == FLT_MAX
    idx.add(torch.tensor([[0, 0, 0, 0], [1, 0, 0, 0], [0, 2, 0, 0.]]))
    D, I = idx.search(torch.tensor([[0.9, 0, 0, 0]]), 5)
    assert I.tolist() == [[1, 0, 2, -1, -1]]
    assert abs(D[0, 0].item() - 0.01) < 1e-6 and abs(D[0, 1].item() - 0.81) < 1e-6


def test_pdf_roundtrip_variants():
    pages = [["Hello (world) one", "second line \\ back"], ["page two text"]]
    for compress in (False, True):
        for objstm in (False, True):
            data = pdf.write_pdf(pages, compress=compress, object_streams=objstm)
            txt = pdf.extract_text(data)
            assert txt == "Hello (world) one\nsecond line \\ back\npage two text\n", (compress, objstm)


REF_PDF = "/root/reference/tr_technology_radar_vol_29_en.pdf"


@pytest.mark.skipif(not os.path.exists(REF_PDF), reason="reference PDF fixture not present")
def test_reference_pdf_extraction():
    """The reference sample (47 pages; ~16.2k words per SURVEY's PyPDF2-based estimate).
    PyPDF2 is not installed, so exact word parity is unpinned; we check the page count,
    a plausible word count and that the 'wazero' answer text from post.png is present."""
    with open(REF_PDF, "rb") as f:
        pages = pdf.extract_pages(f.read())
    assert len(pages) == 47
    text = "".join(p + "\n" for p in pages)
    n = len(text.split())
    assert 14000 <= n <= 20000, n
    assert "wazero" in text
    assert 18 <= len(split_text(text)) <= 26
