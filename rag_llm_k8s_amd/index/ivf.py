"""IVF-Flat index (faiss IndexIVFFlat semantics; BASELINE config 4: 1M-chunk IVF-Flat in HBM).

The reference only has IndexFlatL2 (/root/reference/llm/rag.py:61,80,116); IVF is the config-4
extension of SURVEY §2.4 V3.

* Coarse quantizer = k-means centroids. Training runs on the GPU: the assignment step is the MFMA
  distance-GEMM + argmin kernel (ops/native.kmeans_assign in csrc/kernels/search.hip; exact fp32
  products), the centroid update a scatter-add. faiss defaults: at most 256 training points per
  centroid (random subsample), empty clusters re-seeded from the data.
* Storage: every list lives in ONE column-major HBM store [d][cap] with spare capacity per list
  (start, size, capacity). An append writes the new rows straight into their lists' free slots (one
  scatter kernel); only when some list runs out of room is the store regrown (capacities x1.5, so
  amortised O(1) per vector) -- an append never rebuilds the store from the host lists.
* Search: coarse top-nprobe over the centroids, then the ``ivf_scan`` kernel scans every (query,
  probe) list with a wave-resident running top-k, merged by ``topk_lists_merge``. Exact within the
  probed lists (nprobe = nlist == brute force).
* Probing and list assignment rank the centroids by the SAME numbers (as faiss, which uses its
  quantizer for both): on the GPU the MFMA kernel's scores -(||c||^2 - 2 x.c) (argmin for the
  assignment, topk_lds for the probes, ties -> lower id); elsewhere a row-independent elementwise
  form. So a query at a stored vector's own position finds it with nprobe = 1.
* Host copies of the lists are kept for faiss-format persistence (faiss_io.write_ivf_flat) as
  per-list chunk lists: an append adds one chunk per touched list (O(batch), no re-concatenation);
  a snapshot concatenates outside the index lock and compacts the chunks it wrote.
"""
from __future__ import annotations

import threading

import numpy as np
import torch

from .flat import FLT_MAX

MAX_POINTS_PER_CENTROID = 256  # faiss ClusteringParameters default


def _native_assign_ok(x):
    return x.is_cuda and x.dtype == torch.float32 and x.shape[1] % 64 == 0 and x.shape[1] <= 1024


def _scores_torch(x: torch.Tensor, c: torch.Tensor):
    """||x - c||^2 of every (row, centroid), elementwise (each row's numbers do not depend on the
    other rows of the batch, unlike a GEMM whose kernel choice depends on the shape)."""
    x, c = x.float(), c.float()
    out = torch.empty((x.shape[0], c.shape[0]), dtype=torch.float32, device=x.device)
    step = max(1, (1 << 24) // max(1, c.shape[0] * c.shape[1]))
    for i in range(0, x.shape[0], step):
        out[i:i + step] = ((x[i:i + step, None, :] - c[None]) ** 2).sum(-1)
    return out


def assign(x: torch.Tensor, c: torch.Tensor, cnorm=None):
    """Nearest centroid of every row (ties -> lower id): MFMA kernel on the GPU, torch elsewhere."""
    if _native_assign_ok(x):
        from ..ops import native

        a, _ = native.kmeans_assign(x.contiguous(), c.float().contiguous(), cnorm)
        return a.long()
    return _scores_torch(x, c).argmin(1)


def probes(x: torch.Tensor, c: torch.Tensor, cnorm, nprobe):
    """The nprobe nearest centroids of every row, ranked by the numbers assign() ranks (top-1 ==
    assign), ties -> lower id. int64 [n, nprobe] on x's device."""
    nprobe = min(nprobe, c.shape[0])
    if _native_assign_ok(x):
        from ..ops import native

        cf = c.float().contiguous()
        if c.shape[0] <= 24576 and nprobe <= 256:
            return native.coarse_probes(x.contiguous(), cf, cnorm, nprobe).long()
        # past the top-k kernel's limits: the assignment kernel's own scores -(||c||^2 - 2 x.c), sorted
        # (descending = nearest first, stable -> ties to the lower id), in row chunks of <= 64 MB
        xc = x.contiguous()
        out = torch.empty((x.shape[0], nprobe), dtype=torch.long, device=x.device)
        step = max(1, (16 << 20) // c.shape[0])
        for i in range(0, x.shape[0], step):
            xs = xc[i:i + step]
            sc = torch.empty((xs.shape[0], c.shape[0]), dtype=torch.float32, device=x.device)
            native.kmeans_assign(xs, cf, cnorm, scores=sc)
            out[i:i + step] = torch.sort(sc, dim=1, descending=True, stable=True)[1][:, :nprobe]
        return out
    return torch.sort(_scores_torch(x, c), dim=1, stable=True)[1][:, :nprobe]


def _assign_train(x: torch.Tensor, c: torch.Tensor):
    """k-means training assignment: the MFMA kernel on the GPU; elsewhere one GEMM per row chunk
    (argmin of ||c||^2 - 2 x.c). Training needs no row independence, only speed -- the elementwise
    form of _scores_torch is for search-time probing, where a row's ranking must not depend on
    the batch it arrives in."""
    if _native_assign_ok(x):
        return assign(x, c)
    xf, cf = x.float(), c.float()
    cn = (cf * cf).sum(1)
    out = torch.empty(xf.shape[0], dtype=torch.long, device=xf.device)
    step = max(1, (1 << 24) // max(1, cf.shape[0]))
    for i in range(0, xf.shape[0], step):
        out[i:i + step] = torch.addmm(cn[None, :], xf[i:i + step], cf.t(), alpha=-2.0).argmin(1)
    return out


def kmeans(x: torch.Tensor, k: int, iters: int = 20, seed: int = 0,
           max_points_per_centroid: int = MAX_POINTS_PER_CENTROID):
    """Lloyd's k-means (faiss-like: training subsample of at most max_points_per_centroid * k points,
    random init from the data, empty clusters re-seeded)."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    x = x.float().contiguous()
    n = x.shape[0]
    k = min(k, n)
    if max_points_per_centroid and n > max_points_per_centroid * k:
        x = x[torch.randperm(n, generator=g)[:max_points_per_centroid * k].to(x.device)].contiguous()
        n = x.shape[0]
    c = x[torch.randperm(n, generator=g)[:k].to(x.device)].clone()
    for _ in range(iters):
        a = _assign_train(x, c)
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
        self._cnorm = None
        self._xchunks = []  # host: per list, float32 [m, d] chunks (persistence, CPU search)
        self._ichunks = []  # host: per list, int64 [m] id chunks
        self.ntotal = 0
        self.metric = 1
        self.regrows = 0
        self._lock = threading.RLock()
        self._reset_store()

    # ------------------------------------------------------------------ device store
    def _reset_store(self):
        self._xt, self._cap = None, 0
        self._start = np.zeros(self.nlist, np.int64)
        self._size = np.zeros(self.nlist, np.int64)
        self._lcap = np.zeros(self.nlist, np.int64)
        self._ids_dev = self._start_dev = self._end_dev = None

    def _regrow(self, need):
        """New store with max(16, 1.5 x need) slots per list (multiple of 16); live rows move over."""
        lcap = np.maximum(16, np.ceil(need * 1.5 / 16).astype(np.int64) * 16)
        start = np.concatenate([[0], np.cumsum(lcap)[:-1]]).astype(np.int64)
        cap = int(lcap.sum())
        if cap >= 2 ** 31:
            raise ValueError("IVF store of %d rows exceeds int32 row addressing" % cap)
        xt = torch.zeros(self.d, cap, dtype=torch.float32, device=self.device)
        ids = torch.full((cap,), -1, dtype=torch.int32, device=self.device)
        live = self._size > 0
        if live.any():
            src = np.concatenate([np.arange(s, s + z) for s, z in zip(self._start[live], self._size[live])])
            dst = np.concatenate([np.arange(s, s + z) for s, z in zip(start[live], self._size[live])])
            src_d, dst_d = torch.from_numpy(src).to(self.device), torch.from_numpy(dst).to(self.device)
            xt[:, dst_d] = self._xt[:, src_d]
            ids[dst_d] = self._ids_dev[src_d]
        self._xt, self._cap, self._ids_dev = xt, cap, ids
        self._start, self._lcap = start, lcap
        self.regrows += 1

    def _append_device(self, x, a, ids):
        """Rows x [n, d] (fp32, on the device) into lists a [n] (host int64) with original ids [n]."""
        from ..ops import native

        counts = np.bincount(a, minlength=self.nlist).astype(np.int64)
        need = self._size + counts
        if self._xt is None or bool((need > self._lcap).any()):
            self._regrow(need)
        order = np.argsort(a, kind="stable")
        first = np.concatenate([[0], np.cumsum(counts)[:-1]])
        rank = np.empty(len(a), np.int64)
        rank[order] = np.arange(len(a)) - first[a[order]]
        pos = torch.from_numpy((self._start[a] + self._size[a] + rank).astype(np.int32)).to(self.device)
        native.l2_scatter(self._xt, self._cap, pos, x.contiguous())
        self._ids_dev[pos.long()] = torch.from_numpy(ids.astype(np.int32)).to(self.device)
        self._size = need
        self._start_dev = torch.from_numpy(self._start.astype(np.int32)).to(self.device)
        self._end_dev = torch.from_numpy((self._start + self._size).astype(np.int32)).to(self.device)

    # ------------------------------------------------------------------ training / adds
    def train(self, x):
        if isinstance(x, torch.Tensor):
            x = x.detach().float().reshape(-1, self.d).to(self.device)
        else:
            x = torch.as_tensor(np.asarray(x, dtype=np.float32)).reshape(-1, self.d).to(self.device)
        c = kmeans(x, self.nlist)
        self.nlist = c.shape[0]
        self._set_centroids(c)

    def _set_centroids(self, c):
        self.centroids = c.float().contiguous()
        self._cnorm = (self.centroids * self.centroids).sum(1)
        self._xchunks = [[] for _ in range(self.nlist)]  # per list: float32 [m, d] arrays, in order
        self._ichunks = [[] for _ in range(self.nlist)]  # per list: int64 [m] ids
        self.ntotal = 0
        self._reset_store()
        self.is_trained = True

    def add(self, x):
        x = np.asarray(x.cpu() if hasattr(x, "cpu") else x, dtype=np.float32).reshape(-1, self.d)
        if len(x) == 0:
            return
        with self._lock:
            if not self.is_trained:
                self.train(x)
            xd = torch.from_numpy(x).to(self.device)
            a = assign(xd, self.centroids, self._cnorm).cpu().numpy().astype(np.int64)  # == probes(..)[:, 0]
            ids = np.arange(self.ntotal, self.ntotal + len(x), dtype=np.int64)
            order = np.argsort(a, kind="stable")
            bounds = np.searchsorted(a[order], np.arange(self.nlist + 1))
            for li in np.nonzero(np.diff(bounds))[0]:
                sel = order[bounds[li]:bounds[li + 1]]
                self._xchunks[li].append(x[sel])
                self._ichunks[li].append(ids[sel])
            if self.device.type == "cuda":
                self._append_device(xd, a, ids)
            self.ntotal += len(x)

    # ------------------------------------------------------------------ query
    def search(self, q, k):
        q = torch.as_tensor(q).reshape(-1, self.d).float().contiguous()
        nq = q.shape[0]
        with self._lock:
            if self.ntotal == 0:
                return torch.full((nq, k), FLT_MAX), torch.full((nq, k), -1, dtype=torch.int64)
            nprobe = min(self.nprobe, self.nlist)
            if self.device.type == "cuda" and k <= 64:
                from ..ops import native

                qd = q.to(self.device, non_blocking=True)
                pr = self._coarse_device(qd, nprobe)  # stays on the device: one host sync per search
                D, I = native.ivf_search(self._xt, self._cap, qd, pr, self._start_dev, self._ids_dev, k,
                                         max_list=int(self._size.max()), ends=self._end_dev)
                return D.cpu(), I.cpu()
            pr = probes(q.to(self.centroids.device), self.centroids, self._cnorm, nprobe).cpu()
            return self._search_host(q, pr, k)

    def _coarse_device(self, qd, nprobe):
        """Top-nprobe centroids per query as int32 [nq, nprobe] on the device."""
        return probes(qd, self.centroids, self._cnorm, nprobe).int().contiguous()

    def _search_host(self, q, probes, k):
        nq = q.shape[0]
        D = torch.full((nq, k), FLT_MAX)
        I = torch.full((nq, k), -1, dtype=torch.int64)
        lists, idl = self.lists, self.ids
        for qi in range(nq):
            ls = [p for p in probes[qi].tolist() if p >= 0 and len(idl[p])]
            if not ls:
                continue
            x = torch.from_numpy(np.concatenate([lists[p] for p in ls]))
            ids = torch.from_numpy(np.concatenate([idl[p] for p in ls]))
            d = ((x - q[qi][None]) ** 2).sum(1)
            order = torch.argsort(d, stable=True)
            kk = min(k, len(order))
            D[qi, :kk] = d[order[:kk]]
            I[qi, :kk] = ids[order[:kk]]
        return D, I

    # ------------------------------------------------------------------ host lists
    def _compact(self, li):
        xs, ids = self._xchunks[li], self._ichunks[li]
        if len(xs) > 1:
            self._xchunks[li] = [np.concatenate(xs)]
            self._ichunks[li] = [np.concatenate(ids)]

    @property
    def lists(self):
        """Per-list float32 [n_i, d] host arrays (compacts the chunk lists)."""
        with self._lock:
            out = []
            for li in range(len(self._xchunks)):
                self._compact(li)
                out.append(self._xchunks[li][0] if self._xchunks[li] else np.zeros((0, self.d), np.float32))
            return out

    @property
    def ids(self):
        with self._lock:
            out = []
            for li in range(len(self._ichunks)):
                self._compact(li)
                out.append(self._ichunks[li][0] if self._ichunks[li] else np.zeros(0, np.int64))
            return out

    # ------------------------------------------------------------------ persistence
    def snapshot_writer(self):
        """Consistent copy of centroids + inverted lists now (the chunk lists are shallow-copied under
        the lock: O(nlist)); the callable concatenates and writes them atomically, then compacts the
        chunks it wrote (only if nothing replaced them meanwhile)."""
        with self._lock:
            cents = self.centroids.cpu().numpy() if self.centroids is not None else np.zeros((0, self.d), np.float32)
            xch = [list(c) for c in self._xchunks]
            ich = [list(c) for c in self._ichunks]
            nprobe, d = self.nprobe, self.d

        def write(path):
            from .faiss_io import atomic_write, write_ivf_flat

            lists = [np.concatenate(c) if c else np.zeros((0, d), np.float32) for c in xch]
            ids = [np.concatenate(c) if c else np.zeros(0, np.int64) for c in ich]
            atomic_write(path, lambda f: write_ivf_flat(f, d, cents, lists, ids, nprobe))
            with self._lock:
                for li, (c, x, i) in enumerate(zip(xch, lists, ids)):
                    cur = self._xchunks[li] if li < len(self._xchunks) else None
                    if cur is not None and len(c) > 1 and len(cur) >= len(c) and all(a is b for a, b in zip(cur, c)):
                        self._xchunks[li] = [x] + cur[len(c):]
                        self._ichunks[li] = [i] + self._ichunks[li][len(c):]
        return write

    def write(self, path):
        self.snapshot_writer()(path)

    @classmethod
    def from_lists(cls, r, device="cpu"):
        idx = cls(r["d"], device=device, nlist=r["nlist"], nprobe=max(1, r["nprobe"]))
        idx._set_centroids(torch.from_numpy(np.asarray(r["centroids"], np.float32)).to(idx.device))
        lists = [np.asarray(x, np.float32).reshape(-1, idx.d) for x in r["lists"]]
        ids = [np.asarray(x, np.int64) for x in r["ids"]]
        idx._xchunks = [[x] if len(x) else [] for x in lists]
        idx._ichunks = [[i] if len(i) else [] for i in ids]
        idx.ntotal = int(sum(len(x) for x in ids))
        if idx.device.type == "cuda" and idx.ntotal:
            a = np.concatenate([np.full(len(i), li, np.int64) for li, i in enumerate(ids)])
            x = torch.from_numpy(np.concatenate(lists)).to(idx.device)
            idx._append_device(x, a, np.concatenate(ids))
        return idx
