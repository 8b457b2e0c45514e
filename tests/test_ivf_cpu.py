"""IVF-Flat index on the CPU path: k-means, list assignment, exactness at nprobe = nlist, incremental
appends and faiss-format persistence (the reference only has IndexFlatL2,
/root/reference/llm/rag.py:61,80,116)."""
import io

import numpy as np
import torch

from rag_llm_k8s_amd.index import faiss_io
from rag_llm_k8s_amd.index.ivf import IVFFlatIndex, assign, kmeans


def _data(n, d, seed=0, centers=16):
    g = np.random.default_rng(seed)
    c = g.normal(size=(centers, d)).astype(np.float32) * 4
    return (c[g.integers(0, centers, n)] + g.normal(size=(n, d)).astype(np.float32)).astype(np.float32)


def _exact(xb, q, k):
    d = ((q[:, None, :].astype(np.float64) - xb[None].astype(np.float64)) ** 2).sum(-1)
    return np.argsort(d, axis=1, kind="stable")[:, :k], np.sort(d, axis=1)[:, :k]


def test_kmeans_reduces_inertia_and_subsamples():
    x = torch.from_numpy(_data(4000, 32))
    c = kmeans(x, 16, iters=10)
    a = assign(x, c)
    inertia = ((x - c[a]) ** 2).sum()
    c0 = x[:16]
    inertia0 = ((x - c0[assign(x, c0)]) ** 2).sum()
    assert c.shape == (16, 32) and inertia < 0.7 * inertia0
    # faiss cap: 256 points per centroid -> 4 centroids train on 1024 sampled points, still sane
    c4 = kmeans(x, 4, iters=5, max_points_per_centroid=256)
    assert c4.shape == (4, 32) and torch.isfinite(c4).all()


def test_ivf_nprobe_all_equals_flat_and_incremental_appends():
    d, k = 32, 5
    xb = _data(3000, d, seed=1)
    q = _data(20, d, seed=2)
    idx = IVFFlatIndex(d, nlist=24, nprobe=24)
    idx.train(xb[:2000])
    for lo in range(0, 3000, 700):  # several appends into already-populated lists
        idx.add(xb[lo:lo + 700])
    assert idx.ntotal == 3000 and sum(len(i) for i in idx.ids) == 3000
    D, I = idx.search(torch.from_numpy(q), k)
    ei, ed = _exact(xb, q, k)
    assert np.array_equal(I.numpy(), ei)
    assert np.allclose(D.numpy(), ed, rtol=1e-4, atol=1e-3)


def test_ivf_low_nprobe_recall_and_roundtrip():
    d, k = 32, 4
    xb = _data(4000, d, seed=3)
    q = xb[::97] + 0.01
    idx = IVFFlatIndex(d, nlist=32, nprobe=4)
    idx.add(xb)
    D, I = idx.search(torch.from_numpy(q), k)
    ei, _ = _exact(xb, q, k)
    recall = np.mean([len(set(a) & set(b)) / k for a, b in zip(I.numpy(), ei)])
    assert recall > 0.9
    buf = io.BytesIO()
    idx.snapshot_writer()  # snapshot under the lock must not fail
    faiss_io.write_ivf_flat(buf, d, idx.centroids.numpy(), idx.lists, idx.ids, idx.nprobe)
    buf.seek(0)
    r = faiss_io.read_index_stream(buf)
    idx2 = IVFFlatIndex.from_lists(r)
    D2, I2 = idx2.search(torch.from_numpy(q), k)
    assert torch.equal(I, I2) and torch.allclose(D, D2)


def test_ivf_cpu_every_vector_found_at_nprobe_1_and_chunked_lists():
    from rag_llm_k8s_amd.index.ivf import probes

    d = 16
    xb = _data(1500, d, seed=7)
    idx = IVFFlatIndex(d, nlist=12, nprobe=1)
    idx.train(xb)
    for lo in range(0, 1500, 50):  # many small appends: one chunk per touched list, no re-concatenation
        idx.add(xb[lo:lo + 50])
    assert max(len(c) for c in idx._xchunks) > 1
    x = torch.from_numpy(xb)
    assert torch.equal(probes(x, idx.centroids, idx._cnorm, 3)[:, 0], assign(x, idx.centroids))
    D, I = idx.search(x, 1)
    assert (I[:, 0].numpy() == np.arange(1500)).all()
    w = idx.snapshot_writer()  # concatenates outside the lock, then compacts what it wrote
    buf = io.BytesIO()
    from rag_llm_k8s_amd.index.faiss_io import atomic_write  # noqa: F401  (writer uses it)
    import tempfile, os
    p = os.path.join(tempfile.mkdtemp(), "ivf.index")
    w(p)
    assert max(len(c) for c in idx._xchunks) == 1
    r = faiss_io.read_index(p)
    idx2 = IVFFlatIndex.from_lists(r)
    D2, I2 = idx2.search(x[:50], 3)
    D1, I1 = idx.search(x[:50], 3)
    assert torch.equal(I1, I2)
    del buf
