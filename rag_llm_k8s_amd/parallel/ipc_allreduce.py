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

ONE_SHOT_MAX = 512 << 10
SPIN_LIMIT = int(os.environ.get("RAGK_AR_TIMEOUT_US", "0"))  # 0 = kernel default (5 s per peer wait)
MAX_BYTES = 8 << 20
BLOCKS = 64
# fused decode reduction (ar_add_rmsnorm): row slots and max hidden size of the row area
FUSED_ROWS = 256
FUSED_H = 8192
# one-shot (every rank reads every peer's fp32 row) while the total read stays below this; two-shot
# (reduce-scatter of column slices + gather of the bf16 slices, 2 barriers) above it
FUSED_ONESHOT_BYTES = 512 << 10


def fences_for(cross_device: bool, env=None) -> bool:
    """Fence policy of the fused row barriers. Peers on other GPUs (xGMI): always on -- the uncached
    staging region orders payload before flag only within one device's memory controller. All peers
    on this device (single-GPU rehearsals / probes): RAGK_AR_FENCES=1 turns them on, default off."""
    env = os.environ.get("RAGK_AR_FENCES", "") if env is None else env
    if cross_device:
        if env == "0":
            import logging

            logging.getLogger(__name__).warning("RAGK_AR_FENCES=0 ignored: peer regions live on other GPUs")
        return True
    return env == "1"


class IPCAllReduce:
    def __init__(self, group, cpu_group, size, rank, device, max_bytes=MAX_BYTES, blocks=BLOCKS, spin_limit=None,
                 fused_rows=FUSED_ROWS, fused_h=FUSED_H):
        """spin_limit: bound of one peer wait inside the kernels, in microseconds (None: env / 5 s).
        fused_rows / fused_h: geometry of the fused decode-reduction area (0 rows = none)."""
        if size > 8:
            raise ValueError("peer-mapped all-reduce supports <= 8 ranks (one xGMI node)")
        self.size, self.rank, self.device = size, rank, torch.device(device)
        L = _lib.lib()
        self.L = L
        self.fused_h = int(fused_h) if fused_rows else 0
        with torch.cuda.device(self.device):
            h = L.ragk_ar_create(rank, size, int(max_bytes), int(blocks), int(fused_rows), self.fused_h)
        if not h:
            raise _lib.NativeLibraryError("ragk_ar_create failed (uncached HBM allocation)")
        self.h = ctypes.c_void_p(h)
        self.max_bytes = int(L.ragk_ar_max_bytes(self.h))
        self.fused_rows = int(L.ragk_ar_fused_rows(self.h))
        spin = SPIN_LIMIT if spin_limit is None else int(spin_limit)
        if spin > 0:
            self.set_timeout_us(spin)
        ep = L.ragk_ar_error_host_ptr(self.h)
        # pinned host word the kernel sets when a peer wait gives up: polled after every engine step
        self._err_word = ctypes.c_uint.from_address(ep) if ep else None
        hs = L.ragk_ar_handle_size()
        buf = ctypes.create_string_buffer(hs)
        check(L.ragk_ar_ipc_handle(self.h, buf), "hipIpcGetMemHandle")
        from .dist import device_identity

        me = (bytes(buf.raw), device_identity(self.device))
        recs = [me]
        if size > 1:  # a one-rank communicator (single-GPU probes) has no peers to map
            recs = [None] * size
            dist.all_gather_object(recs, me, group=cpu_group)
        handles = [r[0] for r in recs]
        self.peer_devices = [r[1] for r in recs]
        self.cross_device = any(d != me[1] for d in self.peer_devices)
        # another rank drives this same GPU (single-GPU rehearsals): the fused decode launches, whose blocks
        # wait on other blocks of the same launch, must not run -- other processes' waiting blocks could hold
        # the CU slots their producers need (ops/native.py attn_oproj)
        self.shares_device = sum(d == me[1] for d in self.peer_devices) > 1
        self.set_fences(fences_for(self.cross_device))
        joined = ctypes.create_string_buffer(b"".join(handles), hs * size)
        with torch.cuda.device(self.device):
            check(L.ragk_ar_open_peers(self.h, joined), "hipIpcOpenMemHandle")
        if size > 1:  # every rank must have mapped its peers before anyone signals into them
            dist.barrier(group=cpu_group)

    def self_test(self, group=None) -> bool:
        """Cross-check one call of each mode against a host (gloo) sum; False disables the path."""
        ok = True
        for n, mode in ((8 * 4096, 0), (min(self.max_bytes // 2, 1 << 20) // 8 * 8, 1)):
            g = torch.Generator(device="cpu").manual_seed(1234 + self.rank)
            xh = torch.randn(n, generator=g).bfloat16()
            ref = xh.float()
            dist.all_reduce(ref, group=group)
            y = self.all_reduce(xh.to(self.device), mode=mode)
            ok &= bool(torch.allclose(y.float().cpu(), ref, rtol=1e-2, atol=1e-2)) and not self.error()
        mine = torch.arange(64, dtype=torch.int32) + 1000 * self.rank
        got = self.all_gather(mine.to(self.device)).cpu()
        ok &= bool(torch.equal(got, torch.cat([torch.arange(64, dtype=torch.int32) + 1000 * r
                                               for r in range(self.size)])))
        return ok

    def set_fences(self, on: bool):
        """System-scope release/acquire fences around the fused row barriers (allreduce.hip row_barrier)."""
        check(self.L.ragk_ar_set_fences(self.h, int(bool(on))), "ragk_ar_set_fences")

    @property
    def fences(self) -> bool:
        return self.L.ragk_ar_get_fences(self.h) == 1

    def set_timeout_us(self, us: int):
        """Bound of one peer wait inside the kernels (a rank's first launch of a kernel can lag its
        peers by tens of ms while the code object loads: keep this well above that)."""
        check(self.L.ragk_ar_set_spin_limit(self.h, int(us)), "ragk_ar_set_spin_limit")

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

    def all_gather(self, x: torch.Tensor, out: torch.Tensor | None = None):
        """out = cat over ranks of x (any dtype; x.nbytes % 16 == 0, <= max_bytes): one kernel,
        peer loads over xGMI, graph-capturable."""
        nb = x.numel() * x.element_size()
        _ok = x.is_cuda and x.is_contiguous() and nb % 16 == 0 and nb <= self.max_bytes and x.data_ptr() % 16 == 0
        if not _ok:
            raise ValueError("IPC all-gather: contiguous, nbytes % 16 == 0, <= %d bytes" % self.max_bytes)
        if out is None:
            out = torch.empty((self.size * x.numel(),), dtype=x.dtype, device=x.device)
        if not (out.is_contiguous() and out.numel() == self.size * x.numel() and out.dtype == x.dtype):
            raise ValueError("IPC all-gather: out must hold world * x")
        check(self.L.ragk_ar_allgather(self.h, x.data_ptr(), out.data_ptr(), nb, stream_ptr()), "ragk_ar_allgather")
        return out

    def fused_ok(self, M: int, H: int) -> bool:
        return 0 < M <= self.fused_rows and H <= self.fused_h and H % 8 == 0

    def add_rmsnorm(self, P: torch.Tensor, h: torch.Tensor, w: torch.Tensor, eps: float, out: torch.Tensor,
                    mode: int | None = None):
        """Fused row-parallel reduction of a split-K decode GEMM's fp32 slabs P [S, M, H] across the TP
        ranks + residual add into h [M, H] (bf16, in place) + RMSNorm -> out (csrc/comm/allreduce.hip
        ar_add_rmsnorm). Every rank computes the same bits."""
        S, M, H = P.shape
        ok = (P.is_cuda and P.dtype == torch.float32 and P.is_contiguous() and h.dtype == torch.bfloat16
              and h.shape == (M, H) and h.stride(1) == 1 and out.shape == (M, H) and out.stride(1) == 1
              and w.dtype == torch.bfloat16 and w.is_contiguous() and w.numel() == H and self.fused_ok(M, H)
              and h.stride(0) % 8 == 0 and out.stride(0) % 8 == 0)
        if not ok:
            raise ValueError("fused all-reduce+rmsnorm: P fp32 [S, M, H], h / out bf16 [M, H], M <= %d, H <= %d"
                             % (self.fused_rows, self.fused_h))
        if mode is None:
            mode = 0 if M * H * 4 * self.size <= FUSED_ONESHOT_BYTES else 1
        check(self.L.ragk_ar_add_rmsnorm(self.h, P.data_ptr(), S, M, h.data_ptr(), h.stride(0), w.data_ptr(),
                                         out.data_ptr(), out.stride(0), H, float(eps), int(mode), stream_ptr()),
              "ragk_ar_add_rmsnorm")
        return out

    def gather_fits(self, x: torch.Tensor) -> bool:
        nb = x.numel() * x.element_size()
        return x.is_cuda and x.is_contiguous() and nb % 16 == 0 and nb <= self.max_bytes and x.data_ptr() % 16 == 0

    def error(self) -> bool:
        """True if a peer failed to arrive within the kernel's bounded spin (comm watchdog). Reads the
        pinned host word (no device sync); falls back to a device read."""
        return self.error_record() != 0

    def error_record(self) -> int:
        """The error record of a failed peer wait (0 = healthy; see describe_error)."""
        if self._err_word is not None:
            return int(self._err_word.value)
        return max(0, int(self.L.ragk_ar_error(self.h)))

    def close(self):
        if getattr(self, "h", None):
            self.L.ragk_ar_destroy(self.h)
            self.h = None

    def __del__(self):  # pragma: no cover - interpreter shutdown order
        try:
            self.close()
        except Exception:
            pass


SITES = {1: "all-reduce (start barrier)", 2: "all-reduce (two-shot mid barrier)", 3: "all-gather",
         4: "fused reduce+norm row (start barrier)", 5: "fused reduce+norm row (two-shot mid barrier)"}


def describe_error(rec: int) -> str:
    """Decode an error record of csrc/comm/allreduce.hip (ar_record): 1 | site << 1 | peer << 4 |
    block-or-row << 7 | (epoch & 0xffff) << 15."""
    if not rec:
        return "no error"
    site, peer, slot, ep = (rec >> 1) & 7, (rec >> 4) & 7, (rec >> 7) & 255, (rec >> 15) & 0xFFFF
    what = SITES.get(site, "site %d" % site)
    return "%s, block/row %d, call %d (mod 65536): peer rank %d never arrived" % (what, slot, ep, peer)
