"""Observability: Prometheus metrics + lightweight per-request spans (tracing).

Reference has only DEBUG logging (/root/reference/llm/rag.py:13-14) and no metrics/tracing.
"""
from __future__ import annotations

import logging
import time
from contextlib import contextmanager

try:
    import prometheus_client as prom
except Exception:  # pragma: no cover
    prom = None

_REG = None
_M = {}


def registry():
    global _REG
    if prom is None:
        return None
    if _REG is None:
        _REG = prom.CollectorRegistry()
        b = (0.005, 0.01, 0.025, 0.05, 0.1, 0.25, 0.5, 1, 2.5, 5, 10, 30, 60)
        _M["stage"] = prom.Histogram("rag_stage_seconds", "RAG request stage latency", ["stage"], buckets=b,
                                     registry=_REG)
        _M["request"] = prom.Histogram("rag_request_seconds", "end-to-end /generate latency", buckets=b,
                                       registry=_REG)
        _M["ttft"] = prom.Histogram("rag_ttft_seconds", "time to first generated token", buckets=b, registry=_REG)
        _M["tpot"] = prom.Histogram("rag_tpot_seconds", "time per output token after the first (per request)",
                                    buckets=(0.001, 0.002, 0.003, 0.005, 0.0075, 0.01, 0.015, 0.02, 0.03, 0.05, 0.1,
                                             0.25), registry=_REG)
        _M["tokens"] = prom.Counter("rag_generated_tokens_total", "generated tokens", registry=_REG)
        _M["prompt_tokens"] = prom.Counter("rag_prompt_tokens_total", "prompt tokens", registry=_REG)
        _M["timeouts"] = prom.Counter("rag_request_timeouts_total", "requests aborted by request_timeout_s",
                                      registry=_REG)
        _M["requests"] = prom.Counter("rag_requests_total", "requests", ["route", "status"], registry=_REG)
        _M["batch"] = prom.Gauge("rag_decode_batch", "running sequences after the last engine step", registry=_REG)
        _M["kv_free"] = prom.Gauge("rag_kv_free_blocks", "free KV-cache blocks", registry=_REG)
        _M["index"] = prom.Gauge("rag_index_vectors", "vectors in the index", registry=_REG)
        _M["hbm"] = prom.Gauge("rag_hbm_bytes_allocated", "HBM allocated by torch", registry=_REG)
    return _REG


def m(name):
    registry()
    return _M.get(name)


def observe(name, value, **labels):
    x = m(name)
    if x is None:
        return
    (x.labels(**labels) if labels else x).observe(value)


def inc(name, n=1, **labels):
    x = m(name)
    if x is None:
        return
    (x.labels(**labels) if labels else x).inc(n)


def set_gauge(name, v):
    x = m(name)
    if x is not None:
        x.set(v)


def exposition():
    if prom is None:
        return b"", "text/plain"
    return prom.generate_latest(registry()), prom.CONTENT_TYPE_LATEST


class Trace:
    """Per-request span recorder: `with tr.span('embed'): ...` -> tr.spans['embed'] seconds."""

    def __init__(self, name="request"):
        self.name = name
        self.t0 = time.perf_counter()
        self.spans = {}

    @contextmanager
    def span(self, stage):
        t = time.perf_counter()
        try:
            yield
        finally:
            dt = time.perf_counter() - t
            self.spans[stage] = self.spans.get(stage, 0.0) + dt
            observe("stage", dt, stage=stage)

    def add(self, stage, dt):
        self.spans[stage] = self.spans.get(stage, 0.0) + dt
        observe("stage", dt, stage=stage)

    def total(self):
        return time.perf_counter() - self.t0

    def summary_ms(self):
        d = {k: round(v * 1e3, 3) for k, v in self.spans.items()}
        d["total"] = round(self.total() * 1e3, 3)
        return d


def setup_logging(level="INFO"):
    logging.basicConfig(level=getattr(logging, str(level).upper(), logging.INFO),
                        format="%(asctime)s %(levelname)s %(name)s: %(message)s")
