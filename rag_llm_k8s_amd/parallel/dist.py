"""Process-group setup: one process per GPU, torch.distributed over RCCL ("nccl" on ROCm).

The reference has no distribution at all. Here a job of WORLD_SIZE ranks
is split into tensor-parallel groups of `tp` consecutive ranks (one xGMI-connected node)
and data-parallel replicas across groups. A parallel gloo group carries small control
messages (request broadcast for TP serving) without touching the GPUs.
"""
from __future__ import annotations

import datetime
import os
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist


@dataclass
class DistCtx:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    tp: int = 1
    tp_rank: int = 0
    dp_rank: int = 0
    dp: int = 1
    device: str = "cpu"
    tp_group: Optional[object] = None
    tp_cpu_group: Optional[object] = None
    dp_group: Optional[object] = None
    initialized: bool = False
    device_ids: Optional[list] = None  # device_identity() of every rank (multi-GPU jobs)

    @property
    def is_first(self):
        return self.rank == 0


def init_distributed(tp: int = 1, backend: Optional[str] = None, timeout_s: int = 1800) -> DistCtx:
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    use_cuda = torch.cuda.is_available()
    ctx = DistCtx(rank=rank, world=world, local_rank=local, tp=tp)
    if use_cuda:
        torch.cuda.set_device(local)
        ctx.device = "cuda:%d" % local
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # RCCL errors / timed-out collectives abort the process instead of hanging it (comm watchdog)
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
        be = backend or ("nccl" if use_cuda else "gloo")
        kw = dict(backend=be, timeout=datetime.timedelta(seconds=timeout_s))
        if be == "nccl":
            kw["device_id"] = torch.device(ctx.device)
        dist.init_process_group(**kw)
        ctx.initialized = True
    if world % tp:
        raise ValueError("WORLD_SIZE %d not divisible by tp %d" % (world, tp))
    if world > 1 and use_cuda:
        idents = [None] * world
        dist.all_gather_object(idents, device_identity(ctx.device))
        ctx.device_ids = idents
        check_distinct_devices(idents, allow_shared=os.environ.get("RAGK_ALLOW_SHARED_DEVICE", "0") == "1")
    ctx.dp = world // tp
    ctx.tp_rank = rank % tp
    ctx.dp_rank = rank // tp
    if world > 1:
        for g in range(ctx.dp):
            ranks = list(range(g * tp, (g + 1) * tp))
            grp = dist.new_group(ranks) if tp > 1 else None
            cgrp = dist.new_group(ranks, backend="gloo") if tp > 1 else None
            if rank in ranks:
                ctx.tp_group, ctx.tp_cpu_group = grp, cgrp
        for t in range(tp):
            ranks = list(range(t, world, tp))
            grp = dist.new_group(ranks) if ctx.dp > 1 else None
            if rank in ranks:
                ctx.dp_group = grp
    return ctx


def device_identity(device) -> str:
    """A string naming the PHYSICAL GPU behind `device` (stable across processes on one host): PCI
    domain/bus/device, else the device uuid, else host + ordinal. CPU devices: host + "cpu"."""
    import socket

    host = socket.gethostname()
    dev = torch.device(device)
    if dev.type != "cuda":
        return "%s/cpu" % host
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    try:
        p = torch.cuda.get_device_properties(idx)
        pci = (getattr(p, "pci_domain_id", None), getattr(p, "pci_bus_id", None), getattr(p, "pci_device_id", None))
        if all(v is not None for v in pci) and any(pci):
            return "%s/pci:%04x:%02x:%02x" % (host, *pci)
        uuid = str(getattr(p, "uuid", "") or "")
        if uuid:
            return "%s/uuid:%s" % (host, uuid)
    except Exception:
        pass
    return "%s/cuda:%d" % (host, idx)


def shared_device_ranks(idents):
    """Groups of ranks whose identities (device_identity) name the same physical GPU: [[r, r', ...], ...]
    (empty when every rank has its own device)."""
    by = {}
    for r, d in enumerate(idents):
        by.setdefault(d, []).append(r)
    return [rs for rs in by.values() if len(rs) > 1]


def check_distinct_devices(idents, allow_shared=False):
    """Self-test of a multi-GPU job: every rank must drive its own GPU. N processes on one device run
    (the single-GPU TP rehearsals do exactly that), but a job that CLAIMS N GPUs while two ranks share
    one would report single-device numbers as multi-GPU ones, and its peer-mapped collectives would
    skip the cross-device fences. Raises unless allow_shared (RAGK_ALLOW_SHARED_DEVICE=1)."""
    shared = [rs for rs in shared_device_ranks(idents) if not str(idents[rs[0]]).endswith("/cpu")]
    if shared and not allow_shared:
        raise RuntimeError("ranks %s share a GPU (%s) while the job claims one GPU per rank; set "
                           "RAGK_ALLOW_SHARED_DEVICE=1 for a deliberate single-device rehearsal"
                           % (shared, ", ".join(sorted({idents[rs[0]] for rs in shared}))))
    return shared


def barrier(ctx: DistCtx):
    if ctx.initialized:
        if ctx.device.startswith("cuda"):
            dist.barrier(device_ids=[ctx.local_rank])
        else:
            dist.barrier()


def all_reduce_max(ctx: DistCtx, value: float) -> float:
    if not ctx.initialized:
        return value
    dev = ctx.device if ctx.device.startswith("cuda") else "cpu"
    t = torch.tensor([value], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def all_reduce_sum(ctx: DistCtx, value: float) -> float:
    if not ctx.initialized:
        return value
    dev = ctx.device if ctx.device.startswith("cuda") else "cpu"
    t = torch.tensor([value], dtype=torch.float64, device=dev)
    dist.all_reduce(t)
    return float(t.item())


def all_gather_object(ctx: DistCtx, obj):
    if not ctx.initialized:
        return [obj]
    out = [None] * ctx.world
    dist.all_gather_object(out, obj)
    return out


def shutdown(ctx: DistCtx):
    if ctx.initialized:
        dist.destroy_process_group()
