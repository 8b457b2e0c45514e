"""Tensor-parallel communicator.

Llama TP (Megatron layout) needs two all-reduces of the [T, hidden] residual per layer.
* Default: RCCL all_reduce through torch.distributed on the TP group (ring/tree over xGMI;
  capturable in the decode hipGraph).
* Small messages (decode: 8 KB x batch) are latency-bound on a ring over 7 point-to-point
  xGMI links; the IPC one-shot path (``ragk_allreduce_ipc``) maps every peer's staging
  buffer into each rank (hipIpc handles exchanged over the gloo group) and reduces all 8
  slices with direct xGMI loads in one kernel -- enabled with RAGK_IPC_ALLREDUCE=1 once
  validated on the node (it needs all peers on one host).
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
        if os.environ.get("RAGK_IPC_ALLREDUCE", "0") == "1":
            try:
                from .ipc_allreduce import IPCAllReduce

                self.ipc = IPCAllReduce(group, cpu_group, size, rank, device)
            except Exception as e:  # fall back to RCCL, loudly
                import logging

                logging.getLogger(__name__).warning("IPC all-reduce unavailable (%s); using RCCL", e)
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
