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

    def all_gather_into(self, out: torch.Tensor, x: torch.Tensor):
        dist.all_gather_into_tensor(out, x, group=self.group)
        return out
