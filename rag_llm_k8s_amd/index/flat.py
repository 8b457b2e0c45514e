"""HBM-resident exact L2 index (faiss IndexFlatL2 semantics) + IVF-Flat.

Reference: faiss.IndexFlatL2(1024), index.add, index.search(q, k) (/root/reference/llm/rag.py:61,80,116),
with the whole index re-read from the PVC on every request (:153-155).

Here the vectors live in GPU memory in a column-major [d][capacity] fp32 layout (fully
coalesced streaming in the search kernel), capacity doubles on growth, and search is
the gfx950 l2_block_topk + topk_merge kernels. On CPU the same class uses torch.
Results follow faiss: squared L2, ascending, (-1, FLT_MAX) padding when k > ntotal.
"""
from __future__ import annotations

import threading

import numpy as np
import torch

FLT_MAX = float(np.finfo(np.float32).max)


class FlatL2Index:
    def __init__(self, d: int, device="cpu", capacity: int = 1024):
        self.d = int(d)
        self.device = torch.device(device)
        self.ntotal = 0
        self.metric = 1
        self._cap = max(1, capacity)
        self._lock = threading.RLock()
        if self.device.type == "cuda":
            from ..ops import native

            self._n = native
            self._xt = torch.zeros(self.d, self._cap, dtype=torch.float32, device=self.device)
        else:
            self._n = None
            self._xb = torch.zeros(self._cap, self.d, dtype=torch.float32)

    # ---------------------------------------------------------------- mutation
    def _grow(self, need):
        if need <= self._cap:
            return
        cap = max(need, 2 * self._cap)
        if self._n is not None:
            nxt = torch.zeros(self.d, cap, dtype=torch.float32, device=self.device)
            nxt[:, :self.ntotal] = self._xt[:, :self.ntotal]
            self._xt = nxt
        else:
            nxb = torch.zeros(cap, self.d, dtype=torch.float32)
            nxb[:self.ntotal] = self._xb[:self.ntotal]
            self._xb = nxb
        self._cap = cap

    def add(self, x):
        x = torch.as_tensor(np.asarray(x, dtype=np.float32) if not isinstance(x, torch.Tensor) else x)
        x = x.reshape(-1, self.d).float().contiguous()
        n = x.shape[0]
        if n == 0:
            return
        with self._lock:
            self._grow(self.ntotal + n)
            if self._n is not None:
                self._n.l2_append(self._xt, self._cap, self.ntotal, x.to(self.device))
            else:
                self._xb[self.ntotal:self.ntotal + n] = x
            self.ntotal += n

    def reset(self):
        with self._lock:
            self.ntotal = 0

    # ---------------------------------------------------------------- query
    def search(self, q, k):
        """q: [nq, d] -> (D fp32 [nq,k], I int64 [nq,k]) on the host."""
        q = torch.as_tensor(q).reshape(-1, self.d).float().contiguous()
        nq = q.shape[0]
        if nq == 0:
            return torch.zeros(0, k), torch.zeros(0, k, dtype=torch.int64)
        with self._lock:
            if self._n is not None:
                if k > 64:
                    raise ValueError("k <= 64 on the GPU path")
                D, I = self._n.l2_search(self._xt, self._cap, self.ntotal, q.to(self.device), k)
                return D.cpu(), I.cpu()
            return self._cpu_search(q, k)

    def search_device(self, q, k):
        """GPU-only: q on device -> (D, I) on device (no host sync)."""
        with self._lock:
            return self._n.l2_search(self._xt, self._cap, self.ntotal, q, k)

    def _cpu_search(self, q, k):
        n = self.ntotal
        D = torch.full((q.shape[0], k), FLT_MAX)
        I = torch.full((q.shape[0], k), -1, dtype=torch.int64)
        if n == 0:
            return D, I
        xb = self._xb[:n]
        # faiss' BLAS path: ||x||^2 + ||q||^2 - 2 q.x (clamped at 0), ties -> lower id
        d = (q * q).sum(1, keepdim=True) + (xb * xb).sum(1)[None, :] - 2.0 * (q @ xb.t())
        d = d.clamp_min_(0.0)
        kk = min(k, n)
        dv, di = torch.sort(d, dim=1, stable=True)
        D[:, :kk] = dv[:, :kk]
        I[:, :kk] = di[:, :kk]
        return D, I

    def reconstruct_all(self) -> np.ndarray:
        with self._lock:
            if self._n is not None:
                return self._xt[:, :self.ntotal].t().contiguous().cpu().numpy()
            return self._xb[:self.ntotal].numpy().copy()

    # ---------------------------------------------------------------- persistence
    def snapshot_writer(self):
        """Host copy of the vectors now; the returned callable writes it (faiss IxF2) atomically."""
        xb = self.reconstruct_all()
        d = self.d

        def write(path):
            from ..runtime import native_rt
            from .faiss_io import atomic_write, write_flat_l2

            rt = native_rt()
            if rt is not None:  # C++ writer: temp file + fsync + rename
                rt.write_flat_index(path, xb.reshape(-1, d))
            else:
                atomic_write(path, lambda f: write_flat_l2(f, xb))
        return write

    def write(self, path):
        self.snapshot_writer()(path)

    @classmethod
    def read(cls, path, device="cpu"):
        from .faiss_io import read_index

        r = read_index(path)
        if r["type"] != "flat":
            raise ValueError("not an IndexFlat file")
        idx = cls(r["d"], device=device, capacity=max(1024, r["ntotal"]))
        if r["ntotal"]:
            idx.add(torch.from_numpy(r["xb"]))
        return idx

    def memory_bytes(self):
        return self.d * self._cap * 4
