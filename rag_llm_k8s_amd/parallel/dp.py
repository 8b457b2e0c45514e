"""Data-parallel embedding and a row-sharded vector index over RCCL / gloo.

* embed_distributed: rank r embeds texts[r::world] (length-sorted packing happens inside each
  rank's EmbeddingEngine), then a variable-size all-gather (pad to the max count + counts)
  reassembles the original order on every rank (SURVEY §2.5 "Data parallel (embedding)").
* ShardedFlatIndex: rows are dealt round-robin to ranks (global id g lives on rank g % world
  at local slot g // world). A query batch is all-gathered, every rank computes its local top-k
  for all queries with the HBM kernel, the (distance, global id) candidates are all-gathered and
  merged -- exact, because the global top-k is contained in the union of local top-ks.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ..index.flat import FLT_MAX, FlatL2Index


def _gather_var(x: torch.Tensor, group=None):
    """all-gather tensors whose first dim differs per rank -> list of per-rank tensors."""
    world = dist.get_world_size(group)
    n = torch.tensor([x.shape[0]], dtype=torch.int64, device=x.device)
    counts = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(counts, n, group=group)
    counts = [int(c.item()) for c in counts]
    m = max(counts) if counts else 0
    pad = torch.zeros((m,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    pad[:x.shape[0]] = x
    outs = [torch.zeros_like(pad) for _ in range(world)]
    dist.all_gather(outs, pad, group=group)
    return [o[:c] for o, c in zip(outs, counts)]


def embed_distributed(embedder, texts, group=None):
    """Every rank passes the SAME `texts`; each embeds a strided shard; all get the full result."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return embedder.embed(texts)
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    mine = list(texts[rank::world])
    local = embedder.embed(mine) if mine else torch.zeros((0, embedder.dim), device=embedder.device)
    parts = _gather_var(local.float().contiguous(), group)
    out = torch.empty((len(texts), embedder.dim), dtype=torch.float32, device=local.device)
    for r, p in enumerate(parts):
        out[r::world] = p
    return out


class ShardedFlatIndex:
    def __init__(self, d, device="cpu", group=None):
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.local = FlatL2Index(d, device=device)
        self.d = d
        self.ntotal = 0

    @property
    def device(self):
        return self.local.device

    def load_local(self, xb, ntotal):
        """This rank's rows (from its shard file) and the global vector count."""
        if xb is not None and len(xb):
            self.local.add(torch.as_tensor(xb))
        self.ntotal = int(ntotal)

    def snapshot_writer(self):
        """This rank's rows as a faiss IndexFlatL2 file (the store names it <index>.shard<r>of<W>)."""
        return self.local.snapshot_writer()

    def write(self, path):
        self.snapshot_writer()(path)

    def add(self, x):
        """All ranks pass the same full batch; each keeps its round-robin share."""
        x = torch.as_tensor(x).float().reshape(-1, self.d)
        n = x.shape[0]
        gids = torch.arange(self.ntotal, self.ntotal + n)
        keep = (gids % self.world) == self.rank
        self.local.add(x[keep])
        self.ntotal += n

    def search(self, q_local, k):
        """Each rank passes ITS OWN queries; returns (D, I) for them with global ids."""
        q_local = torch.as_tensor(q_local).float().reshape(-1, self.d)
        dev = self.local.device
        if self.world == 1:
            return self.local.search(q_local, k)
        comm_dev = dev if dev.type == "cuda" else torch.device("cpu")
        qs = _gather_var(q_local.to(comm_dev).contiguous(), self.group)
        allq = torch.cat(qs, 0)
        D, I = self.local.search(allq, k)
        # local slot -> global id
        gI = torch.where(I >= 0, I * self.world + self.rank, I)
        dl = [torch.zeros_like(D.to(comm_dev)) for _ in range(self.world)]
        il = [torch.zeros_like(gI.to(comm_dev)) for _ in range(self.world)]
        dist.all_gather(dl, D.to(comm_dev).contiguous(), group=self.group)
        dist.all_gather(il, gI.to(comm_dev).contiguous(), group=self.group)
        Dc = torch.cat([x.cpu() for x in dl], 1)
        Ic = torch.cat([x.cpu() for x in il], 1)
        Dc = torch.where(Ic >= 0, Dc, torch.full_like(Dc, FLT_MAX))
        # ascending by (distance, id), ties -> lower id
        key_i = torch.where(Ic >= 0, Ic, torch.full_like(Ic, 2 ** 62))
        order = torch.argsort(key_i, dim=1, stable=True)
        Dc, Ic = torch.gather(Dc, 1, order), torch.gather(Ic, 1, order)
        order = torch.argsort(Dc, dim=1, stable=True)
        Dm, Im = torch.gather(Dc, 1, order)[:, :k], torch.gather(Ic, 1, order)[:, :k]
        off = sum(x.shape[0] for x in qs[:self.rank])
        return Dm[off:off + q_local.shape[0]], Im[off:off + q_local.shape[0]]
