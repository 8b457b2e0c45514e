"""Property-based tests (hypothesis): the reference chunker contract, the paged-KV
block manager (C++ and Python implementations agree and never hand out a block twice), the
prefill micro-batch splitter and the decode split-K partition planner."""
import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from rag_llm_k8s_amd.engine.kv_manager import PyBlockManager, make_block_manager
from rag_llm_k8s_amd.engine.llm_engine import LLMEngine
from rag_llm_k8s_amd.ingest.text import split_text


@settings(max_examples=200, deadline=None)
@given(n_words=st.integers(0, 3000), size=st.integers(2, 1200), overlap=st.integers(0, 1199))
def test_split_text_windows(n_words, size, overlap):
    """/root/reference/llm/rag.py:39-45: windows of `size` words every `size - overlap` words, a
    window for every start < len(words) (trailing ones included)."""
    if overlap >= size:
        with pytest.raises(ValueError):
            split_text("w " * n_words, size, overlap)
        return
    words = ["w%d" % i for i in range(n_words)]
    chunks = split_text(" ".join(words), size, overlap)
    step = size - overlap
    assert len(chunks) == len(range(0, n_words, step))
    for j, c in enumerate(chunks):
        assert c.split() == words[j * step:j * step + size]
    covered = set(w for c in chunks for w in c.split())
    assert covered == set(words)


@settings(max_examples=60, deadline=None)
@given(ops=st.lists(st.tuples(st.integers(0, 5), st.integers(0, 300), st.booleans()), max_size=40))
def test_block_manager_matches_python_and_never_double_allocates(ops):
    nb = 24
    mgrs = [make_block_manager(nb), PyBlockManager(nb)]
    for sid, n, free in ops:
        res = []
        for m in mgrs:
            if free:
                m.free(sid)
                res.append(None)
            else:
                ok = m.can_allocate(sid, n)
                if ok:
                    m.ensure(sid, n)
                res.append(ok)
        assert res[0] == res[1]
        tables = [[m.table(s) for s in range(6)] for m in mgrs]
        assert tables[0] == tables[1]
        used = [b for t in tables[0] for b in t]
        assert len(used) == len(set(used)), "a block is owned by two sequences"
        assert mgrs[0].free_blocks() == mgrs[1].free_blocks()


@settings(max_examples=200, deadline=None)
@given(ns=st.lists(st.integers(1, 500), min_size=1, max_size=8), parts=st.integers(1, 4))
def test_split_chunks_partitions_the_token_stream(ns, parts):
    seqs = [object() for _ in ns]
    chunks = [(s, 3 * i, n) for i, (s, n) in enumerate(zip(seqs, ns))]
    groups = LLMEngine._split_chunks(chunks, parts)
    flat = [(s, a, n) for g in groups for (s, a, n) in g]
    # same tokens, same order, contiguous pieces of each original chunk
    for s, start, n in chunks:
        pieces = [(a, m) for (t, a, m) in flat if t is s]
        assert pieces[0][0] == start and sum(m for _, m in pieces) == n
        for (a0, m0), (a1, _) in zip(pieces, pieces[1:]):
            assert a1 == a0 + m0
    sizes = [sum(n for _, _, n in g) for g in groups]
    target = -(-sum(ns) // parts)
    assert sum(sizes) == sum(ns) and len(groups) <= parts
    assert all(x == target for x in sizes[:-1]) and 0 < sizes[-1] <= target
    if parts == 2:  # the TP micro-batch split: halves within one token
        assert max(sizes) - min(sizes) <= 1 or len(groups) == 1


@settings(max_examples=300, deadline=None)
@given(max_len=st.integers(1, 131072), batch=st.integers(1, 256), hkv=st.sampled_from([1, 2, 4, 8]),
       kv_len=st.integers(1, 131072))
def test_decode_partitions_cover_every_tile(max_len, batch, hkv, kv_len):
    """attention.hip:decode_part_tiles: with the planner's (part_tiles, max_parts), every sequence's
    KV tiles fall in the launched partitions, each partition non-empty."""
    from rag_llm_k8s_amd.ops.native import decode_partitions

    kv_len = min(kv_len, max_len)
    pt, mp = decode_partitions(max_len, batch, hkv)
    assert pt >= 1 and mp >= 1
    n_kt = -(-kv_len // 64)
    eff = max(pt, -(-n_kt // mp))
    nparts = -(-n_kt // eff)
    assert 1 <= nparts <= mp
    assert (nparts - 1) * eff < n_kt <= nparts * eff
