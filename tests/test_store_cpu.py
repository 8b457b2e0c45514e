"""DocumentStore concurrency (SURVEY §5 race detection): the background snapshot writer, appends and
maybe_reload() interleaved deterministically. The reference's unlocked read-modify-write is
/root/reference/llm/rag.py:68-86; its per-request re-read is :153-155."""
import os
import threading
import time

import numpy as np

from rag_llm_k8s_amd.index.faiss_io import read_index
from rag_llm_k8s_amd.index.store import DocumentStore


def _meta(name, n, start=0):
    return [{"filename": name, "chunk_id": start + i, "text": "t%d" % (start + i)} for i in range(n)]


def _vecs(n, d=8, seed=0):
    return np.random.default_rng(seed).standard_normal((n, d)).astype(np.float32)


def test_reload_ignores_own_snapshot_in_flight(tmp_path):
    st = DocumentStore(str(tmp_path / "faiss_index"), 8).ensure_exists()
    st.add(_vecs(4), _meta("a.pdf", 4), persist=False)
    st.persist()

    entered, release = threading.Event(), threading.Event()
    orig = st._snapshot

    def slow_snapshot():
        writer, meta = orig()

        def w(path):
            writer(path)  # the index file is replaced (new mtime) ...
            os.utime(path, (time.time() + 3, time.time() + 3))
            entered.set()
            release.wait(10)  # ... and the metadata file is not yet

        return w, meta

    st._snapshot = slow_snapshot
    st.add(_vecs(3, seed=1), _meta("b.pdf", 3))  # starts the background writer
    assert entered.wait(10)
    st._snapshot = orig
    # appends that land while the snapshot is being written
    st.add(_vecs(2, seed=2), _meta("c.pdf", 2))
    st.maybe_reload()  # disk mtimes changed under our own writer: must not reload the older snapshot
    assert st.index.ntotal == 9 and len(st.metadata) == 9
    release.set()
    st.flush()
    assert st._persister is None
    r = read_index(str(tmp_path / "faiss_index"))
    assert r["ntotal"] == 9
    st.maybe_reload()  # nothing changed by anyone else
    assert st.index.ntotal == 9
    # a file replaced by ANOTHER writer is still picked up
    other = DocumentStore(str(tmp_path / "faiss_index"), 8).ensure_exists()
    other.add(_vecs(1, seed=3), _meta("d.pdf", 1), persist=False)
    time.sleep(0.01)
    other.persist()
    t = time.time() + 7
    os.utime(str(tmp_path / "faiss_index"), (t, t))
    st.maybe_reload()
    assert st.index.ntotal == 10


def test_no_lost_wakeup_between_writer_exit_and_add(tmp_path):
    st = DocumentStore(str(tmp_path / "faiss_index"), 8).ensure_exists()
    n = 0
    for i in range(40):  # appends racing the writer's exit path
        st.add(_vecs(1, seed=i), _meta("f%d.pdf" % i, 1))
        n += 1
        if i % 3 == 0:
            time.sleep(0.001)
    deadline = time.time() + 10
    while time.time() < deadline:  # without flush(): the writer alone must catch up
        t = st._persister
        if t is None and not st._dirty:
            break
        time.sleep(0.01)
    assert st._persister is None and not st._dirty
    assert read_index(str(tmp_path / "faiss_index"))["ntotal"] == n


def test_concurrent_adds_and_searches_stay_consistent(tmp_path):
    st = DocumentStore(str(tmp_path / "faiss_index"), 8).ensure_exists()
    errs = []

    def writer(k):
        try:
            for i in range(15):
                st.add(_vecs(2, seed=100 * k + i), _meta("w%d.pdf" % k, 2, start=2 * i))
        except Exception as e:  # pragma: no cover - surfaced below
            errs.append(e)

    def reader():
        try:
            for _ in range(50):
                st.maybe_reload()
                for res in st.search(_vecs(2, seed=9), 5):
                    for m, d in res:
                        assert isinstance(m, dict) and d >= 0
        except Exception as e:  # pragma: no cover
            errs.append(e)

    ts = [threading.Thread(target=writer, args=(k,)) for k in range(3)] + [threading.Thread(target=reader)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    st.flush()
    assert not errs
    assert st.index.ntotal == 90 == len(st.metadata)
    assert read_index(str(tmp_path / "faiss_index"))["ntotal"] == 90
