"""IVF-Flat index (faiss IndexIVFFlat semantics; BASELINE config 4: 1M-chunk IVF-Flat in HBM).

Coarse quantizer = k-means centroids (trained on the GPU with MFMA matmuls); each vector
is stored in the inverted list of its nearest centroid. All lists live in ONE
list-ordered, column-major HBM store (rows of a list are contiguous), so a probe is a
contiguous row range. Search: coarse top-nprobe over the centroids, then the gfx950
``ivf_scan`` kernel scans every (query, probe) range and keeps a per-range top-k, merged by
``topk_merge``. Exact within the probed lists (nprobe = nlist == brute force).
"""
from __future__ import annotations

import threading

import numpy as np
import torch

from .flat import FLT_MAX, FlatL2Index


def kmeans(x: torch.Tensor, k: int, iters: int = 20, seed: int = 0):
    """Lloyd's k-means (faiss-like: random init from the data, empty clusters re-seeded)."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    n = x.shape[0]
    k = min(k, n)
    c = x[torch.randperm(n, generator=g)[:k].to(x.device)].clone()
    for _ in range(iters):
        d = (x * x).sum(1, keepdim=True) - 2 * x @ c.t() + (c * c).sum(1)[None]
        a = d.argmin(1)
        s = torch.zeros_like(c).index_add_(0, a, x)
        cnt = torch.bincount(a, minlength=k).float()
        empty = cnt == 0
        c = torch.where(empty[:, None], c, s / cnt.clamp_min(1)[:, None])
        if bool(empty.any()):
            ne = int(empty.sum())
            c[empty] = x[torch.randint(0, n, (ne,), generator=g).to(x.device)]
    return c


class IVFFlatIndex:
    def __init__(self, d, device="cpu", nlist=1024, nprobe=32):
        self.d, self.device = int(d), torch.device(device)
        self.nlist, self.nprobe = int(nlist), int(nprobe)
        self.is_trained = False
        self.centroids = None
        self.quant = None
        self.lists = []  # host: per-list float32 [n_i, d]
        self.ids = []  # host: per-list int64 [n_i]
        self.ntotal = 0
        self.metric = 1
        self._dirty = True
        self._lock = threading.RLock()
        self._store = None

    def train(self, x):
        x = torch.as_tensor(np.asarray(x, dtype=np.float32)).to(self.device)
        c = kmeans(x, self.nlist)
        self.nlist = c.shape[0]
        self._set_centroids(c)

    def _set_centroids(self, c):
        self.centroids = c.float().contiguous()
        self.quant = FlatL2Index(self.d, device=self.device, capacity=self.nlist)
        self.quant.add(self.centroids.cpu())
        self.lists = [np.zeros((0, self.d), np.float32) for _ in range(self.nlist)]
        self.ids = [np.zeros(0, np.int64) for _ in range(self.nlist)]
        self.is_trained = True

    def add(self, x):
        x = np.asarray(x.cpu() if hasattr(x, "cpu") else x, dtype=np.float32).reshape(-1, self.d)
        if len(x) == 0:
            return
        with self._lock:
            if not self.is_trained:
                self.train(x)
            _, a = self.quant.search(torch.from_numpy(x), 1)
            a = a[:, 0].numpy()
            ids = np.arange(self.ntotal, self.ntotal + len(x), dtype=np.int64)
            for li in np.unique(a):
                m = a == li
                self.lists[li] = np.concatenate([self.lists[li], x[m]])
                self.ids[li] = np.concatenate([self.ids[li], ids[m]])
            self.ntotal += len(x)
            self._dirty = True

    def _build(self):
        sizes = np.array([len(i) for i in self.ids], dtype=np.int64)
        self._offsets = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
        allx = np.concatenate(self.lists) if self.ntotal else np.zeros((0, self.d), np.float32)
        allid = np.concatenate(self.ids) if self.ntotal else np.zeros(0, np.int64)
        self._store = FlatL2Index(self.d, device=self.device, capacity=max(1, self.ntotal))
        self._store.add(allx)
        self._ids_dev = torch.from_numpy(allid.astype(np.int32)).to(self.device)
        self._ids_host = torch.from_numpy(allid)
        self._off_dev = torch.from_numpy(self._offsets.astype(np.int32)).to(self.device)
        self._dirty = False

    def search(self, q, k):
        q = torch.as_tensor(q).reshape(-1, self.d).float().contiguous()
        nq = q.shape[0]
        with self._lock:
            if self.ntotal == 0:
                return torch.full((nq, k), FLT_MAX), torch.full((nq, k), -1, dtype=torch.int64)
            if self._dirty:
                self._build()
            nprobe = min(self.nprobe, self.nlist)
            _, probes = self.quant.search(q, nprobe)  # [nq, nprobe] host
            if self.device.type == "cuda" and k <= 64:
                from ..ops import native

                D, I = native.ivf_search(self._store._xt, self._store._cap, q.to(self.device),
                                         probes.to(self.device).int(), self._off_dev, self._ids_dev, k)
                return D.cpu(), I.cpu()
            return self._search_torch(q, probes, k)

    def _search_torch(self, q, probes, k):
        xb = self._store.reconstruct_all()
        xb = torch.from_numpy(xb)
        nq = q.shape[0]
        D = torch.full((nq, k), FLT_MAX)
        I = torch.full((nq, k), -1, dtype=torch.int64)
        for qi in range(nq):
            rows = [torch.arange(int(self._offsets[p]), int(self._offsets[p + 1])) for p in probes[qi].tolist()]
            rows = torch.cat(rows) if rows else torch.zeros(0, dtype=torch.int64)
            if len(rows) == 0:
                continue
            x = xb[rows]
            d = ((x - q[qi][None]) ** 2).sum(1)
            ids = self._ids_host[rows]
            order = torch.argsort(d, stable=True)
            kk = min(k, len(order))
            D[qi, :kk] = d[order[:kk]]
            I[qi, :kk] = ids[order[:kk]]
        return D, I

    def snapshot_writer(self):
        """Consistent copy of centroids + inverted lists now; the callable writes it atomically."""
        with self._lock:
            cents = self.centroids.cpu().numpy() if self.centroids is not None else np.zeros((0, self.d), np.float32)
            lists, ids, nprobe, d = list(self.lists), list(self.ids), self.nprobe, self.d

        def write(path):
            from .faiss_io import atomic_write, write_ivf_flat

            atomic_write(path, lambda f: write_ivf_flat(f, d, cents, lists, ids, nprobe))
        return write

    def write(self, path):
        self.snapshot_writer()(path)

    @classmethod
    def from_lists(cls, r, device="cpu"):
        idx = cls(r["d"], device=device, nlist=r["nlist"], nprobe=max(1, r["nprobe"]))
        idx._set_centroids(torch.from_numpy(r["centroids"]).to(idx.device))
        idx.lists = [np.asarray(x, np.float32) for x in r["lists"]]
        idx.ids = [np.asarray(x, np.int64) for x in r["ids"]]
        idx.ntotal = int(sum(len(x) for x in idx.ids))
        idx._dirty = True
        return idx
