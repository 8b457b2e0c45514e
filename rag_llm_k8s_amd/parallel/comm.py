"""Tensor-parallel communicator.

Llama TP (Megatron layout) needs two all-reduces of the [T, hidden] residual per layer.
* Default: RCCL all_reduce through torch.distributed on the TP group (ring/tree over xGMI;
  capturable in the decode hipGraph).
* Small / medium messages (decode: 8 KB x batch) are latency-bound on a ring over 7
  point-to-point xGMI links; the peer-mapped path (parallel/ipc_allreduce.py, kernel in
  csrc/comm/allreduce.hip) maps every peer's staging buffer into each rank (hipIpc handles
  exchanged over the gloo group) and does the collective in one kernel with direct xGMI
  loads: one-shot <= 512 KB, two-shot <= 8 MB, RCCL above. On by default on GPUs
  (RAGK_IPC_ALLREDUCE=0 disables); it is cross-checked against RCCL at start-up and
  disabled, loudly, if the check fails.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


class TPComm:
    def __init__(self, group, size, rank, device, cpu_group=None):
        self.group, self.size, self.rank, self.device = group, size, rank, device
        self.cpu_group = cpu_group
        self.ipc = None
        self._side = None  # side stream for asynchronous peer-mapped all-reduces
        want = os.environ.get("RAGK_IPC_ALLREDUCE", "1") == "1"
        if want and size > 1 and str(device).startswith("cuda") and cpu_group is not None:
            import logging

            log = logging.getLogger(__name__)
            try:
                from .ipc_allreduce import IPCAllReduce

                ipc = IPCAllReduce(group, cpu_group, size, rank, device)
                ok = torch.tensor([1 if ipc.self_test(group) else 0], device=device)
                dist.all_reduce(ok, op=dist.ReduceOp.MIN, group=group)  # all ranks agree
                if int(ok.item()) == 1:
                    self.ipc = ipc
                else:
                    log.warning("IPC all-reduce self-test failed; using RCCL")
                    ipc.close()
            except Exception as e:  # fall back to RCCL, loudly
                log.warning("IPC all-reduce unavailable (%s); using RCCL", e)
                self.ipc = None

    def all_reduce(self, x: torch.Tensor):
        if self.size == 1:
            return x
        if self.ipc is not None and self.ipc.fits(x):
            return self.ipc.all_reduce(x)
        if not x.is_cuda and x.dtype == torch.bfloat16:  # gloo: reduce in fp32, round once
            y = x.float()
            dist.all_reduce(y, group=self.group)
            x.copy_(y)
            return x
        dist.all_reduce(x, group=self.group)
        return x

    def all_reduce_async(self, x: torch.Tensor):
        """Start an in-place all-reduce of x; returns a handle whose wait() makes the CURRENT stream
        (GPU) or the host (gloo) wait for it. x must not be touched until then."""
        if self.size == 1:
            return _Done()
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
        """out[r*S:(r+1)*S] = rank r's x (S = x.shape[0]): RCCL all-gather; gloo via a list gather."""
        if self.size == 1:
            out.copy_(x)
            return out
        if x.is_cuda:
            dist.all_gather_into_tensor(out, x, group=self.group)
        else:
            dist.all_gather(list(out.chunk(self.size)), x.contiguous(), group=self.group)
        return out

    def reduce_scatter(self, x: torch.Tensor, out: torch.Tensor = None):
        """Sum of every rank's x [size*S, ...], this rank's S-row slice: RCCL reduce-scatter (each
        byte crosses xGMI once, half an all-reduce); gloo has none -- fp32 all-reduce + slice."""
        S = x.shape[0] // self.size
        if out is None:
            out = torch.empty((S,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
        if self.size == 1:
            out.copy_(x)
            return out
        if x.is_cuda:
            dist.reduce_scatter_tensor(out, x, group=self.group)
        else:
            y = x.float()
            dist.all_reduce(y, group=self.group)
            out.copy_(y[self.rank * S:(self.rank + 1) * S])
        return out


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
