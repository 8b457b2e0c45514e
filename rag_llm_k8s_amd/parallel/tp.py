"""Tensor-parallel serving: one process per GPU, rank 0 serves HTTP.

The engine is deterministic given its inputs, so TP ranks only need to agree on WHICH requests
enter WHEN. Rank 0's engine loop drains newly submitted requests once per step and publishes one
control record per step on a channel to the follower ranks before stepping; followers receive
the same record, add the same sequences in the same order and step. All GPU-side exchange (2
all-reduces per layer, top-k candidate all-gather) runs over xGMI inside the step.

Control record = fixed 16-byte header (kind, payload bytes) + a payload only when there is
something to admit or to abort: the new requests (prompt ids as one int32 buffer, params, seed,
and rank 0's key of the sequence) and the keys of sequences to abort. Every rank applies the
aborts at the start of the same step, so a timed-out request frees its KV blocks everywhere
(the reference fails such a request with a 500, /root/reference/llm/rag.py:179-181). Two
transports:
* ``ShmChannel`` (default when every TP rank is on this host, i.e. one xGMI node): a POSIX
  shared-memory mailbox; rank 0 writes payload then header then bumps a sequence word, followers
  poll it (spin briefly, then back off) and acknowledge. A step with nothing to admit costs a few
  microseconds, not a gloo round trip.
* ``GlooChannel``: a fixed-size int64 header broadcast over the TP gloo group every step, plus a
  uint8 payload broadcast only when there is something to admit.
The reference has no distribution; this is the "step metadata broadcast" row of the
collective table in SURVEY §2.6.
"""
from __future__ import annotations

import dataclasses
import logging
import os
import pickle
import socket
import threading
import time
import uuid

import numpy as np
import torch
import torch.distributed as dist

from ..engine.llm_engine import SamplingParams, Sequence
from ..utils import faults

log = logging.getLogger(__name__)

HEARTBEAT_S = 30.0
K_STEP, K_NOOP, K_SHUTDOWN, K_JOB = 1, 2, 3, 4


class GlooChannel:
    """Header [kind, nbytes] (int64) broadcast per record; payload bytes only when nbytes > 0."""

    def __init__(self, cpu_group, src=0):
        self.group, self.src = cpu_group, src

    def send(self, kind, payload=b""):
        hdr = torch.tensor([kind, len(payload)], dtype=torch.int64)
        dist.broadcast(hdr, src=self.src, group=self.group)
        if payload:
            dist.broadcast(torch.frombuffer(bytearray(payload), dtype=torch.uint8), src=self.src, group=self.group)

    def recv(self):
        hdr = torch.zeros(2, dtype=torch.int64)
        dist.broadcast(hdr, src=self.src, group=self.group)
        kind, n = int(hdr[0]), int(hdr[1])
        payload = b""
        if n:
            buf = torch.empty(n, dtype=torch.uint8)
            dist.broadcast(buf, src=self.src, group=self.group)
            payload = buf.numpy().tobytes()
        return kind, payload

    def close(self):
        pass


class ShmChannel:
    """Single-producer mailbox in POSIX shared memory (every TP rank on one host).

    Layout (int64 words): [0] seq, [1] kind, [2] nbytes, [8 + r] ack of rank r, then the payload
    area. Rank 0 waits until every follower acknowledged record seq-1, writes payload, kind,
    nbytes, then seq (x86 stores are not reordered with other stores, and numpy writes them in
    program order), so a follower that sees the new seq reads a complete record."""

    HDR_WORDS = 64
    POLL_SPIN_S = 0.002

    @classmethod
    def create(cls, cpu_group, rank, world, capacity=1 << 20, src=0, timeout_s=600.0):
        """Collective constructor: the channel on every rank, or None on every rank."""
        from multiprocessing import shared_memory

        shm, name = None, [None]
        if rank == src:
            try:
                name[0] = "ragk_tp_%s" % uuid.uuid4().hex[:16]
                shm = shared_memory.SharedMemory(name=name[0], create=True, size=cls.HDR_WORDS * 8 + capacity)
                shm.buf[:cls.HDR_WORDS * 8] = bytes(cls.HDR_WORDS * 8)
            except Exception as e:
                log.warning("cannot create the TP control segment: %s", e)
                name[0] = None
        dist.broadcast_object_list(name, src=src, group=cpu_group)
        if rank != src and name[0] is not None:
            try:
                shm = shared_memory.SharedMemory(name=name[0], create=False)
                try:  # the producer owns the segment; followers must not unlink it at exit
                    from multiprocessing import resource_tracker
                    resource_tracker.unregister(shm._name, "shared_memory")
                except Exception:
                    pass
            except Exception as e:
                log.warning("cannot attach the TP control segment: %s", e)
                shm = None
        ok = torch.tensor([1 if shm is not None else 0], dtype=torch.int32)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN, group=cpu_group)  # every rank mapped it (or none uses it)
        if rank == src and shm is not None:  # the name can go now (the mappings stay)
            shm.unlink()
        if int(ok.item()) == 0:
            if shm is not None:
                shm.close()
            return None
        return cls(cpu_group, rank, world, shm, src=src, timeout_s=timeout_s)

    def __init__(self, cpu_group, rank, world, shm, src=0, timeout_s=600.0):
        self.rank, self.world, self.src, self.timeout_s = rank, world, src, timeout_s
        self.shm = shm
        self.words = np.ndarray((self.HDR_WORDS,), dtype=np.int64, buffer=self.shm.buf)
        self.cap = len(self.shm.buf) - self.HDR_WORDS * 8
        self.seq = 0
        self.group = cpu_group  # big payloads (> capacity) go over gloo

    def _wait(self, cond, what):
        t0 = time.monotonic()
        while not cond():
            dt = time.monotonic() - t0
            if dt > self.POLL_SPIN_S:
                time.sleep(min(0.001, dt * 0.1))
            if dt > self.timeout_s:
                raise TimeoutError("TP control channel: %s timed out after %.0fs" % (what, dt))

    def send(self, kind, payload=b""):
        w = self.words
        if self.seq > 0:  # previous record consumed by every follower
            self._wait(lambda: all(int(w[8 + r]) >= self.seq for r in range(self.world) if r != self.src),
                       "follower acknowledgement")
        big = len(payload) > self.cap
        if not big and payload:
            self.shm.buf[self.HDR_WORDS * 8:self.HDR_WORDS * 8 + len(payload)] = payload
        w[1] = kind
        w[2] = -len(payload) if big else len(payload)
        self.seq += 1
        w[0] = self.seq
        if big:
            dist.broadcast(torch.frombuffer(bytearray(payload), dtype=torch.uint8), src=self.src, group=self.group)

    def recv(self):
        w = self.words
        nxt = self.seq + 1
        self._wait(lambda: int(w[0]) >= nxt, "waiting for rank 0")
        kind, n = int(w[1]), int(w[2])
        if n >= 0:
            payload = bytes(self.shm.buf[self.HDR_WORDS * 8:self.HDR_WORDS * 8 + n]) if n else b""
        else:
            buf = torch.empty(-n, dtype=torch.uint8)
            dist.broadcast(buf, src=self.src, group=self.group)
            payload = buf.numpy().tobytes()
        self.seq = nxt
        w[8 + self.rank] = nxt
        return kind, payload

    def close(self):
        try:
            self.words = None
            self.shm.close()
        except Exception:
            pass


def make_channel(cpu_group, rank, world, src=0):
    """Shared memory when every TP rank runs on this host (RAGK_TP_CONTROL=gloo forces gloo). Every
    rank reaches the same choice: a segment that cannot be created or attached on ANY rank (e.g.
    /dev/shm not writable) falls back to gloo everywhere, loudly."""
    mode = os.environ.get("RAGK_TP_CONTROL", "auto")
    if mode != "gloo":
        hosts = [None] * world
        dist.all_gather_object(hosts, socket.gethostname(), group=cpu_group)
        if len(set(hosts)) == 1:
            ch = ShmChannel.create(cpu_group, rank, world, src=src)
            if ch is not None:
                return ch
            log.warning("shared-memory TP control channel unavailable; using gloo")
    return GlooChannel(cpu_group, src)


def _encode(seqs, aborts=()):
    """Step record payload: new sequences (key, int32 prompt buffer, params, seed) + abort keys."""
    new = [(s.id, np.asarray(s.prompt, dtype=np.int32).tobytes(), dataclasses.asdict(s.params), s.seed)
           for s in seqs]
    return pickle.dumps((new, list(aborts)), protocol=pickle.HIGHEST_PROTOCOL)


def _decode(payload):
    if not payload:
        return [], []
    new, aborts = pickle.loads(payload)
    out = []
    for key, ids, params, seed in new:
        p = dict(params)
        p["stop_token_ids"] = tuple(p.get("stop_token_ids", ()))
        out.append((key, np.frombuffer(ids, dtype=np.int32), SamplingParams(**p), seed))
    return out, aborts


class TPControl:
    """Rank-0 side: queue of submitted sequences, published in order once per engine step."""

    def __init__(self, cpu_group, src_rank=0, channel=None):
        self.group = cpu_group
        self.src = src_rank
        if channel is None:
            world = dist.get_world_size(cpu_group)
            channel = make_channel(cpu_group, dist.get_rank(cpu_group), world, src_rank)
        self.chan = channel
        self.pending = []
        self.aborts = []
        self.lock = threading.Lock()
        self.last_publish = time.time()

    def enqueue(self, seq: Sequence):
        with self.lock:
            self.pending.append(seq)

    def abort(self, seq: Sequence):
        """Cancel a sequence on every TP rank (request timeout). Not yet published: dropped here;
        published: its key rides on the next step record and every rank aborts it at that step."""
        with self.lock:
            if seq in self.pending:
                self.pending.remove(seq)
                seq.status, seq.finish_reason, seq.t_done = 2, "abort", time.perf_counter()
                seq.done.set()
                return
            self.aborts.append(seq)

    def has_pending(self):
        with self.lock:
            return bool(self.pending) or bool(self.aborts)

    def publish_step(self, engine):
        with self.lock:
            new, self.pending = self.pending, []
            ab, self.aborts = self.aborts, []
        self.chan.send(K_STEP, _encode(new, [s.id for s in ab]) if (new or ab) else b"")
        self.last_publish = time.time()
        for s in ab:
            engine.abort(s)
        for s in new:
            engine.add_sequence(s)

    def publish_job(self, name, args):
        """A collective job (data-parallel ingest, sharded search) every rank runs before its next step."""
        self.chan.send(K_JOB, pickle.dumps((name, args), protocol=pickle.HIGHEST_PROTOCOL))
        self.last_publish = time.time()

    def publish_heartbeat(self):
        self.chan.send(K_NOOP)
        self.last_publish = time.time()

    def publish_shutdown(self):
        try:
            self.chan.send(K_SHUTDOWN)
        except Exception:
            pass


def follow(engine, cpu_group, src_rank=0, channel=None, jobs=None):
    """Follower loop (ranks != 0): mirror rank 0's admissions, steps and collective jobs until shutdown.
    `jobs`: name -> callable(args), the same functions rank 0's engine loop runs (RagService.job_fns)."""
    if channel is None:
        channel = make_channel(cpu_group, dist.get_rank(cpu_group), dist.get_world_size(cpu_group), src_rank)
    live, key_of = {}, {}  # rank 0's sequence key <-> this rank's mirror (for aborts)
    try:
        while True:
            kind, payload = channel.recv()
            if kind == K_SHUTDOWN:
                return
            if kind == K_NOOP:
                continue
            if kind == K_JOB:
                name, args = pickle.loads(payload)
                jobs[name](args)
                continue
            hang = faults.value("comm_hang_s")
            if hang:  # fault injection: this rank stalls, rank 0's collectives wait (watchdog path)
                time.sleep(float(hang))
            new, aborts = _decode(payload)
            for key in aborts:
                s = live.pop(key, None)
                if s is not None:
                    key_of.pop(id(s), None)
                    engine.abort(s)
            for key, prompt, params, seed in new:
                s = engine.add_request(prompt.tolist(), params, seed=seed)
                live[key], key_of[id(s)] = s, key
            for s in engine.step():
                live.pop(key_of.pop(id(s), None), None)
    finally:
        channel.close()


def run_tp_server(cfg, rank, world):
    """torchrun --nproc-per-node TP llm/rag.py  (TP_SIZE == WORLD_SIZE)."""
    from ..server.app import create_app
    from ..server.builder import build_service
    from .comm import TPComm
    from .dist import init_distributed

    # a collective that outlives two watchdog periods is dead: fail it so the pod restarts
    ctx = init_distributed(tp=world, timeout_s=int(max(600, 2 * cfg.step_timeout_s)))
    comm = TPComm(ctx.tp_group, ctx.tp, ctx.tp_rank, ctx.device, ctx.tp_cpu_group)
    chan = make_channel(ctx.tp_cpu_group, ctx.tp_rank, ctx.tp)
    control = TPControl(ctx.tp_cpu_group, channel=chan) if rank == 0 else None
    svc = build_service(cfg, start_threads=(rank == 0), tp_rank=ctx.tp_rank, tp_size=ctx.tp, comm=comm,
                        tp_group=ctx.tp_group, control=control)
    if rank != 0:
        if svc.store.sharded:  # every rank serves (and persists) its own row shard
            svc.store.ensure_exists()
        follow(svc.engine, ctx.tp_cpu_group, channel=chan, jobs=svc.job_fns())
        return
    svc.store.ensure_exists()
    svc.ingest_directory()
    svc.ready = True
    app = create_app(svc)
    app.run(host=cfg.host, port=cfg.port, threaded=True)
