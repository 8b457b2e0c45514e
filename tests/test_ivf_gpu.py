"""IVF-Flat on the GPU: the MFMA k-means assignment kernel vs an fp64 torch argmin, the ivf_scan kernel
vs an exact scan of the same probed lists, nprobe = nlist == brute force, appends into spare list
capacity (and regrows), faiss-format reload onto the GPU. SURVEY §2.4 V3 (config 4)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda:0"


def _data(n, d, seed=0, centers=64):
    g = np.random.default_rng(seed)
    c = g.normal(size=(centers, d)).astype(np.float32) * 2
    return (c[g.integers(0, centers, n)] + g.normal(size=(n, d)).astype(np.float32)).astype(np.float32)


@pytest.mark.parametrize("n,d,k", [(5001, 384, 300), (2048, 1024, 64), (777, 64, 1000)])
def test_kmeans_assign_matches_fp64_argmin(n, d, k):
    from rag_llm_k8s_amd.ops import native

    x = torch.from_numpy(_data(n, d, seed=n)).to(DEV)
    c = torch.from_numpy(_data(k, d, seed=k + 1)).to(DEV)
    a, dist = native.kmeans_assign(x, c)
    torch.cuda.synchronize()
    ref = torch.cdist(x.double(), c.double()) ** 2
    best = ref.min(1).values
    got = ref.gather(1, a.long()[:, None])[:, 0]
    # chosen centroid is the nearest up to fp32 rounding of the distance expansion
    tol = 1e-5 * (x.double() ** 2).sum(1) + 1e-5 * (c.double() ** 2).sum(1).max()
    assert bool(((got - best) <= tol).all())
    assert (a.long() == ref.argmin(1)).float().mean() > 0.999
    assert torch.allclose(dist.double(), got, rtol=1e-4, atol=float(tol.max()))


def test_ivf_gpu_exact_and_appends():
    from rag_llm_k8s_amd.index.ivf import IVFFlatIndex

    d, k = 384, 8
    xb = _data(20000, d, seed=5)
    q = torch.from_numpy(_data(33, d, seed=6))
    idx = IVFFlatIndex(d, device=DEV, nlist=64, nprobe=64)
    idx.train(xb[:8000])
    for lo in range(0, 20000, 3000):  # appends into spare capacity + at least one regrow
        idx.add(xb[lo:lo + 3000])
    assert idx.ntotal == 20000 and idx.regrows >= 1
    assert int(idx._size.sum()) == 20000 and bool((idx._size <= idx._lcap).all())
    # nprobe = nlist: brute force (fp64 reference)
    D, I = idx.search(q, k)
    ref = torch.cdist(q.double(), torch.from_numpy(xb).double()) ** 2
    rd, ri = ref.topk(k, dim=1, largest=False)
    assert (I == ri).float().mean() > 0.99
    assert torch.allclose(D.double(), rd, rtol=1e-4, atol=1e-2)
    # low nprobe: the kernel equals an exact scan of the same probed lists
    idx.nprobe = 6
    D6, I6 = idx.search(q, k)
    probes = idx._coarse_device(q.to(DEV), 6).cpu()
    Dh, Ih = idx._search_host(q, probes, k)
    assert (I6 == Ih).float().mean() > 0.99
    assert torch.allclose(D6, Dh, rtol=1e-4, atol=1e-2)


def test_ivf_gpu_reload_from_faiss_lists(tmp_path):
    from rag_llm_k8s_amd.index import faiss_io
    from rag_llm_k8s_amd.index.ivf import IVFFlatIndex

    d, k = 128, 4
    xb = _data(6000, d, seed=9)
    q = torch.from_numpy(xb[::301] + 0.01)
    idx = IVFFlatIndex(d, device=DEV, nlist=32, nprobe=8)
    idx.add(xb)
    D, I = idx.search(q, k)
    p = str(tmp_path / "ivf.index")
    idx.write(p)
    idx2 = IVFFlatIndex.from_lists(faiss_io.read_index(p), device=DEV)
    D2, I2 = idx2.search(q, k)
    assert torch.equal(I, I2) and torch.allclose(D, D2)
    assert (I[:, 0] == torch.arange(0, 6000, 301)).all()


def test_ivf_every_stored_vector_found_at_nprobe_1():
    """Probing and list assignment rank centroids by the same numbers (MFMA scores, ties -> lower
    id): a query at a stored vector's own position finds it with nprobe = 1 -- including vectors
    placed exactly half-way between two centroids (ties) and exact duplicates of centroids."""
    from rag_llm_k8s_amd.index.ivf import IVFFlatIndex, assign, probes

    d = 128
    xb = _data(3000, d, seed=21, centers=16)
    idx = IVFFlatIndex(d, device=DEV, nlist=16, nprobe=1)
    idx.train(xb)
    c = idx.centroids.cpu().numpy()
    mids = np.stack([(c[i] + c[(i + 1) % 16]) / 2 for i in range(16)]).astype(np.float32)
    allx = np.concatenate([xb, mids, c]).astype(np.float32)
    idx.add(allx)
    xd = torch.from_numpy(allx).to(DEV)
    a = assign(xd, idx.centroids, idx._cnorm)
    p = probes(xd, idx.centroids, idx._cnorm, 4)
    assert torch.equal(p[:, 0], a)  # top-1 probe == assignment, row by row
    p1 = probes(xd[:1], idx.centroids, idx._cnorm, 1)  # batch size does not change the ranking
    assert int(p1[0, 0]) == int(a[0])
    D, I = idx.search(torch.from_numpy(allx), 1)
    assert (D[:, 0] <= 1e-3).all()
    found = I[:, 0].numpy()
    ok = (found == np.arange(len(allx))) | (D[:, 0].numpy() == 0)
    assert ok.all()
