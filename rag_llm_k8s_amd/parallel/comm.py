"""Tensor-parallel communicator.

Llama TP (Megatron layout) needs two all-reduces of the [T, hidden] residual per layer and one
all-gather of the sampler's per-rank top-k candidates per step.
* Default: RCCL all_reduce / all_gather through torch.distributed on the TP group (ring/tree over
  xGMI; capturable in the decode hipGraph).
* Small / medium messages (decode: 8 KB x batch) are latency-bound on a ring over 7
  point-to-point xGMI links; the peer-mapped path (parallel/ipc_allreduce.py, kernels in
  csrc/comm/allreduce.hip) maps every peer's staging buffer into each rank (hipIpc handles
  exchanged over the gloo group) and does the collective in one kernel with direct xGMI
  loads: one-shot <= 512 KB, two-shot <= 8 MB, RCCL above; the candidate all-gather goes the
  same way, so a TP decode step issues no RCCL call. On by default on GPUs
  (RAGK_IPC_ALLREDUCE=0 disables); it is cross-checked against a host sum at start-up and
  disabled, loudly, if the check fails on any rank.

Comm watchdog: every peer wait in those kernels is bounded; a peer that never arrives sets a pinned
host word. :meth:`TPComm.check` (called by the engine after every step) turns it into
:class:`CommError`, after which the communicator refuses every further call -- the epochs of the
ranks are out of step, so continuing would all-reduce stale data (reference error path: the 500
of /root/reference/llm/rag.py:179-181; here the engine loop fails and /healthz reports 503).
"""
from __future__ import annotations

import logging
import os
import time

import torch
import torch.distributed as dist

from ..utils import faults

log = logging.getLogger(__name__)


class CommError(RuntimeError):
    """A tensor-parallel collective failed (a peer did not arrive within the bounded wait)."""


class TPComm:
    def __init__(self, group, size, rank, device, cpu_group=None, ipc_max_bytes=None, ipc_spin_limit=None):
        """ipc_spin_limit: bound of one peer wait in microseconds, applied after the self-test."""
        self.group, self.size, self.rank, self.device = group, size, rank, device
        self.cpu_group = cpu_group
        self.ipc = None
        self.broken = None  # error message once a collective failed
        self._side = None  # side stream for asynchronous peer-mapped all-reduces
        want = os.environ.get("RAGK_IPC_ALLREDUCE", "1") == "1"
        if want and size > 1 and str(device).startswith("cuda") and cpu_group is not None:
            ok, ipc = 0, None
            try:
                from .ipc_allreduce import MAX_BYTES, IPCAllReduce

                ipc = IPCAllReduce(group, cpu_group, size, rank, device, max_bytes=ipc_max_bytes or MAX_BYTES)
                ok = 1 if ipc.self_test(cpu_group) else 0  # at the default (long) peer-wait bound
                if ok and ipc_spin_limit:
                    ipc.set_timeout_us(ipc_spin_limit)
            except Exception as e:  # fall back to RCCL, loudly
                log.warning("IPC all-reduce unavailable on rank %d (%s); using RCCL", rank, e)
            flag = torch.tensor([ok], dtype=torch.int32)
            dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=cpu_group)  # all ranks agree
            if int(flag.item()) == 1:
                self.ipc = ipc
            else:
                if ipc is not None:
                    log.warning("IPC all-reduce self-test failed; using RCCL")
                    ipc.close()

    # ------------------------------------------------------------------ watchdog
    def check(self):
        """Raise CommError if a peer-mapped collective gave up waiting for a peer (cheap: reads a
        pinned host word). Once raised, every later call raises too."""
        if self.broken is None and self.ipc is not None and self.ipc.error():
            from .ipc_allreduce import describe_error

            self.broken = "peer-mapped collective timed out on rank %d: %s" % (
                self.rank, describe_error(self.ipc.error_record()))
            log.critical(self.broken)
        if self.broken is not None:
            raise CommError(self.broken)

    def _guard(self):
        if self.broken is not None:
            raise CommError(self.broken)
        skew = faults.value("comm_skew_ms")
        if skew:  # fault injection: this rank reaches the collective late by a per-call, per-rank amount
            self._calls = getattr(self, "_calls", 0) + 1
            time.sleep(float(skew) * ((self._calls * 7 + self.rank * 3) % 5) / 4e3)

    # ------------------------------------------------------------------ collectives
    def all_reduce(self, x: torch.Tensor):
        if self.size == 1:
            return x
        self._guard()
        if self.ipc is not None and self.ipc.fits(x):
            return self.ipc.all_reduce(x)
        if not x.is_cuda and x.dtype == torch.bfloat16:  # gloo: reduce in fp32, round once
            y = x.float()
            dist.all_reduce(y, group=self.group)
            x.copy_(y)
            return x
        dist.all_reduce(x, group=self.group)
        return x

    def add_partials_rmsnorm(self, P: torch.Tensor, h: torch.Tensor, w: torch.Tensor, eps: float, be):
        """Consumer of a row-parallel split-K decode GEMM (o_proj / down): h <- bf16(h + bf16(sum over
        ranks and slabs of P)), returns rmsnorm(h) * w. On GPUs one kernel does the cross-rank sum over
        the peer mappings (no standalone all-reduce launch); elsewhere an fp32 all-reduce of the summed
        slabs with the same rounding points."""
        if self.size == 1:
            return be.add_partials_rmsnorm(P, h, w, eps)
        self._guard()
        M, H = h.shape
        if self.ipc is not None and P.is_cuda and self.ipc.fused_ok(M, H):
            return self.ipc.add_rmsnorm(P, h, w, eps, torch.empty_like(h))
        part = P.float().sum(0)
        dist.all_reduce(part, group=self.group)  # fp32, identical on every rank
        h.copy_((h.float() + part.to(h.dtype).float()).to(h.dtype))
        return be.rmsnorm(h, w, eps)

    def fused_decode_ok(self, M: int, H: int) -> bool:
        """The decode step may use the fused row-parallel reduction at batch M (always true off the
        peer-mapped path: the fallback is an ordinary all-reduce)."""
        return self.ipc is None or self.ipc.fused_ok(M, H)

    @property
    def shares_device(self) -> bool:
        """Another rank of this group drives the same GPU (single-GPU rehearsals)."""
        return bool(self.ipc is not None and getattr(self.ipc, "shares_device", False)) or (
            self.ipc is None and str(self.device).startswith("cuda") and self.size > 1
            and os.environ.get("RAGK_ALLOW_SHARED_DEVICE", "0") == "1")

    def all_reduce_async(self, x: torch.Tensor):
        """Start an in-place all-reduce of x; returns a handle whose wait() makes the CURRENT stream
        (GPU) or the host (gloo) wait for it. x must not be touched until then."""
        if self.size == 1:
            return _Done()
        self._guard()
        if self.ipc is not None and self.ipc.fits(x):
            cur = torch.cuda.current_stream(x.device)
            if self._side is None:
                self._side = torch.cuda.Stream(device=x.device)
            self._side.wait_stream(cur)
            with torch.cuda.stream(self._side):
                self.ipc.all_reduce(x)
                ev = torch.cuda.Event()
                ev.record(self._side)
            x.record_stream(self._side)
            return _StreamWait(ev, x.device)
        if not x.is_cuda and x.dtype == torch.bfloat16:  # gloo: fp32 sum, rounded once (as all_reduce)
            y = x.float()
            work = dist.all_reduce(y, group=self.group, async_op=True)
            return _CopyBack(work, y, x)
        return dist.all_reduce(x, group=self.group, async_op=True)

    def all_gather_into(self, out: torch.Tensor, x: torch.Tensor):
        """out[r*S:(r+1)*S] = rank r's x (S = x.shape[0]): peer-mapped kernel when it fits, else RCCL
        all-gather; gloo via a list gather."""
        if self.size == 1:
            out.copy_(x)
            return out
        self._guard()
        if self.ipc is not None and out.is_contiguous() and self.ipc.gather_fits(x):
            self.ipc.all_gather(x.contiguous(), out=out.view(-1))
        elif x.is_cuda:
            dist.all_gather_into_tensor(out, x, group=self.group)
        else:
            dist.all_gather(list(out.chunk(self.size)), x.contiguous(), group=self.group)
        return out

    def gather_candidates(self, cv: torch.Tensor, ci: torch.Tensor):
        """Vocab-parallel sampler exchange: per-rank top-k candidates [B, K] (fp32 values, int32 ids)
        -> [B, size*K] each, rank-major within a row (identical on every rank)."""
        B, K = cv.shape
        if self.size == 1:
            return cv, ci
        self._guard()
        if self.ipc is not None and cv.is_cuda:
            packed = torch.cat([cv.contiguous().view(torch.int32).reshape(-1), ci.contiguous().reshape(-1)])
            if self.ipc.gather_fits(packed):
                g = self.ipc.all_gather(packed).view(self.size, 2, B, K)
                gv = g[:, 0].view(torch.float32)
                gi = g[:, 1]
                return (gv.permute(1, 0, 2).reshape(B, self.size * K).contiguous(),
                        gi.permute(1, 0, 2).reshape(B, self.size * K).contiguous())
        if cv.is_cuda:
            gv = torch.empty((self.size, B, K), dtype=cv.dtype, device=cv.device)
            gi = torch.empty((self.size, B, K), dtype=ci.dtype, device=ci.device)
            dist.all_gather_into_tensor(gv, cv.contiguous(), group=self.group)
            dist.all_gather_into_tensor(gi, ci.contiguous(), group=self.group)
        else:  # gloo (CPU plumbing / tests)
            lv = [torch.empty_like(cv) for _ in range(self.size)]
            li = [torch.empty_like(ci) for _ in range(self.size)]
            dist.all_gather(lv, cv.contiguous(), group=self.group)
            dist.all_gather(li, ci.contiguous(), group=self.group)
            gv, gi = torch.stack(lv), torch.stack(li)
        return gv.permute(1, 0, 2).reshape(B, self.size * K).contiguous(), \
            gi.permute(1, 0, 2).reshape(B, self.size * K).contiguous()

    def reduce_scatter(self, x: torch.Tensor, out: torch.Tensor = None):
        """Sum of every rank's x [size*S, ...], this rank's S-row slice: RCCL reduce-scatter (each
        byte crosses xGMI once, half an all-reduce); gloo has none -- fp32 all-reduce + slice."""
        S = x.shape[0] // self.size
        if out is None:
            out = torch.empty((S,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
        if self.size == 1:
            out.copy_(x)
            return out
        self._guard()
        if x.is_cuda and self.ipc is not None and self.ipc.fits(x):
            self.ipc.all_reduce(x)  # peer-mapped two-shot: the slice of the full sum
            out.copy_(x[self.rank * S:(self.rank + 1) * S])
        elif x.is_cuda:
            dist.reduce_scatter_tensor(out, x, group=self.group)
        else:
            y = x.float()
            dist.all_reduce(y, group=self.group)
            out.copy_(y[self.rank * S:(self.rank + 1) * S])
        return out


class SingleRankTPComm:
    shares_device = False  # one process: the fused decode launches are safe

    """One-GPU stand-in for rank `rank` of a `size`-way TP group (probes of a TP shard's step time):
    the model and engine take their TP code paths, and every collective is replaced by a same-sized
    call of the peer-mapped kernels on a ONE-rank communicator (the barrier and the loads hit local
    HBM instead of xGMI) -- so launches, kernels and bytes moved per rank are those of the real TP
    step, minus the xGMI latency."""

    def __init__(self, size, rank, device, max_bytes=None, fused_rows=256, fused_h=8192):
        from .ipc_allreduce import MAX_BYTES, IPCAllReduce

        self.size, self.rank, self.device = size, rank, device
        self.group = self.cpu_group = None
        self.broken = None
        self.ipc = IPCAllReduce(None, None, 1, 0, device, max_bytes=max_bytes or MAX_BYTES, fused_rows=fused_rows,
                                fused_h=fused_h)

    def check(self):
        if self.ipc.error():
            raise CommError("single-rank peer-mapped kernel timed out")

    def all_reduce(self, x):
        if self.ipc.fits(x):
            self.ipc.all_reduce(x)
        return x

    def add_partials_rmsnorm(self, P, h, w, eps, be):
        return self.ipc.add_rmsnorm(P, h, w, eps, torch.empty_like(h))

    def fused_decode_ok(self, M, H):
        return self.ipc.fused_ok(M, H)

    def gather_candidates(self, cv, ci):
        B, K = cv.shape
        packed = torch.cat([cv.contiguous().view(torch.int32).reshape(-1), ci.contiguous().reshape(-1)])
        g = self.ipc.all_gather(packed.repeat(self.size)).view(self.size, 2, B, K)  # size x the bytes
        gv, gi = g[:, 0].view(torch.float32), g[:, 1]
        return (gv.permute(1, 0, 2).reshape(B, self.size * K).contiguous(),
                gi.permute(1, 0, 2).reshape(B, self.size * K).contiguous())


class _Done:
    def wait(self):
        return None


class _StreamWait:
    def __init__(self, ev, device):
        self.ev, self.device = ev, device

    def wait(self):
        torch.cuda.current_stream(self.device).wait_event(self.ev)


class _CopyBack:
    def __init__(self, work, y, x):
        self.work, self.y, self.x = work, y, x

    def wait(self):
        self.work.wait()
        self.x.copy_(self.y)
