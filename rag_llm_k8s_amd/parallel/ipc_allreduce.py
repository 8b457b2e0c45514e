"""xGMI peer-mapped all-reduce for tensor-parallel decode (csrc/comm/allreduce.hip).

Each rank allocates one uncached HBM region, exports it as a hipIpc handle, and the
handles are exchanged over the TP group's gloo (CPU) channel; every rank then maps all
peers' regions. One kernel per call does the whole collective over the point-to-point
xGMI links (no RCCL proxy, no ring): one-shot for latency-bound messages (decode:
8 KB x batch), two-shot (reduce-scatter + all-gather through peer loads) for medium
ones; bulk prefill messages stay on RCCL (TPComm decides with :meth:`fits`).

The reference has no collectives at all (/root/reference/llm/rag.py:22-31
loads one CPU model); this is the "IPC one-shot all-reduce" component of the new comm
layer. All ranks must call with the same sizes in the same order (as TP layers do).
"""
from __future__ import annotations

import ctypes
import os

import torch
import torch.distributed as dist

from ..ops import _lib
from ..ops._lib import check, stream_ptr

ONE_SHOT_MAX = int(os.environ.get("RAGK_AR_ONESHOT_MAX", str(512 << 10)))
MAX_BYTES = int(os.environ.get("RAGK_AR_MAX_BYTES", str(8 << 20)))
BLOCKS = int(os.environ.get("RAGK_AR_BLOCKS", "64"))


class IPCAllReduce:
    def __init__(self, group, cpu_group, size, rank, device, max_bytes=MAX_BYTES, blocks=BLOCKS):
        if size > 8:
            raise ValueError("peer-mapped all-reduce supports <= 8 ranks (one xGMI node)")
        self.size, self.rank, self.device = size, rank, torch.device(device)
        L = _lib.lib()
        self.L = L
        with torch.cuda.device(self.device):
            h = L.ragk_ar_create(rank, size, int(max_bytes), int(blocks))
        if not h:
            raise _lib.NativeLibraryError("ragk_ar_create failed (uncached HBM allocation)")
        self.h = ctypes.c_void_p(h)
        self.max_bytes = int(L.ragk_ar_max_bytes(self.h))
        hs = L.ragk_ar_handle_size()
        buf = ctypes.create_string_buffer(hs)
        check(L.ragk_ar_ipc_handle(self.h, buf), "hipIpcGetMemHandle")
        handles = [None] * size
        dist.all_gather_object(handles, bytes(buf.raw), group=cpu_group)
        joined = ctypes.create_string_buffer(b"".join(handles), hs * size)
        with torch.cuda.device(self.device):
            check(L.ragk_ar_open_peers(self.h, joined), "hipIpcOpenMemHandle")
        # every rank must have mapped its peers before anyone signals into them
        dist.barrier(group=cpu_group)

    def self_test(self, group=None) -> bool:
        """Cross-check one call of each mode against RCCL/gloo; False disables the path."""
        ok = True
        for n, mode in ((8 * 4096, 0), (min(self.max_bytes // 2, 1 << 20) // 8 * 8, 1)):
            g = torch.Generator(device="cpu").manual_seed(1234 + self.rank)
            x = torch.randn(n, generator=g).bfloat16().to(self.device)
            ref = x.float()
            dist.all_reduce(ref, group=group)
            y = self.all_reduce(x.clone(), mode=mode)
            ok &= bool(torch.allclose(y.float(), ref, rtol=1e-2, atol=1e-2)) and not self.error()
        return ok

    def fits(self, x: torch.Tensor) -> bool:
        return (x.is_cuda and x.dtype == torch.bfloat16 and x.is_contiguous() and x.numel() % 8 == 0
                and x.numel() * 2 <= self.max_bytes and x.data_ptr() % 16 == 0)

    def all_reduce(self, x: torch.Tensor, out: torch.Tensor | None = None, mode: int | None = None):
        out = x if out is None else out
        if not self.fits(x) or out.shape != x.shape or not out.is_contiguous():
            raise ValueError("IPC all-reduce: bf16 contiguous, numel % 8 == 0, <= %d bytes" % self.max_bytes)
        if mode is None:
            mode = 0 if x.numel() * 2 <= ONE_SHOT_MAX else 1
        check(self.L.ragk_ar_allreduce(self.h, x.data_ptr(), out.data_ptr(), x.numel(), int(mode), stream_ptr()),
              "ragk_ar_allreduce")
        return out

    def error(self) -> bool:
        """True if a peer failed to arrive within the kernel's bounded spin (comm watchdog)."""
        return self.L.ragk_ar_error(self.h) != 0

    def close(self):
        if getattr(self, "h", None):
            self.L.ragk_ar_destroy(self.h)
            self.h = None

    def __del__(self):  # pragma: no cover - interpreter shutdown order
        try:
            self.close()
        except Exception:
            pass
