"""Tensor-parallel serving: one process per GPU, rank 0 serves HTTP.

The engine is deterministic given its inputs, so TP ranks only need to agree on WHICH requests
enter WHEN. Rank 0's engine loop drains newly submitted requests once per step and broadcasts
them (token ids, sampling params, seed) over a gloo control group before stepping; followers
receive the same list, add the same sequences in the same order and step. All GPU-side
exchange (2 all-reduces per layer, top-k candidate all-gather) runs over RCCL inside the step.
"""
from __future__ import annotations

import dataclasses
import logging
import threading
import time

import torch
import torch.distributed as dist

from ..engine.llm_engine import SamplingParams, Sequence
from ..utils import faults

log = logging.getLogger(__name__)

HEARTBEAT_S = 30.0


class TPControl:
    """Rank-0 side: queue of submitted sequences, published in order once per engine step."""

    def __init__(self, cpu_group, src_rank=0):
        self.group = cpu_group
        self.src = src_rank
        self.pending = []
        self.lock = threading.Lock()
        self.last_publish = time.time()

    def enqueue(self, seq: Sequence):
        with self.lock:
            self.pending.append(seq)

    def has_pending(self):
        with self.lock:
            return bool(self.pending)

    def _bcast(self, msg):
        obj = [msg]
        dist.broadcast_object_list(obj, src=self.src, group=self.group)
        self.last_publish = time.time()

    def publish_step(self, engine):
        with self.lock:
            new, self.pending = self.pending, []
        self._bcast(("step", [(s.prompt, dataclasses.asdict(s.params), s.seed) for s in new]))
        for s in new:
            engine.add_sequence(s)

    def publish_heartbeat(self):
        self._bcast(("noop", []))

    def publish_shutdown(self):
        try:
            self._bcast(("shutdown", []))
        except Exception:
            pass


def follow(engine, cpu_group, src_rank=0):
    """Follower loop (ranks != 0): mirror rank 0's admissions and steps until shutdown."""
    while True:
        obj = [None]
        dist.broadcast_object_list(obj, src=src_rank, group=cpu_group)
        kind, reqs = obj[0]
        if kind == "shutdown":
            return
        if kind == "noop":
            continue
        hang = faults.value("comm_hang_s")
        if hang:  # fault injection: this rank stalls, rank 0's collectives wait (watchdog path)
            time.sleep(float(hang))
        for prompt, params, seed in reqs:
            p = dict(params)
            p["stop_token_ids"] = tuple(p.get("stop_token_ids", ()))
            engine.add_request(prompt, SamplingParams(**p), seed=seed)
        engine.step()


def run_tp_server(cfg, rank, world):
    """torchrun --nproc-per-node TP llm/rag.py  (TP_SIZE == WORLD_SIZE)."""
    from ..server.app import create_app
    from ..server.builder import build_service
    from .comm import TPComm
    from .dist import init_distributed

    # a collective that outlives two watchdog periods is dead: fail it so the pod restarts
    ctx = init_distributed(tp=world, timeout_s=int(max(600, 2 * cfg.step_timeout_s)))
    comm = TPComm(ctx.tp_group, ctx.tp, ctx.tp_rank, ctx.device, ctx.tp_cpu_group)
    control = TPControl(ctx.tp_cpu_group) if rank == 0 else None
    svc = build_service(cfg, start_threads=(rank == 0), tp_rank=ctx.tp_rank, tp_size=ctx.tp, comm=comm,
                        tp_group=ctx.tp_group, control=control)
    if rank != 0:
        follow(svc.engine, ctx.tp_cpu_group)
        return
    svc.store.ensure_exists()
    svc.ingest_directory()
    svc.ready = True
    app = create_app(svc)
    app.run(host=cfg.host, port=cfg.port, threaded=True)
