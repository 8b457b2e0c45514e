"""Env-driven fault injection (SURVEY §5 "Failure detection / elastic recovery / fault injection").

The reference has none: a failed model load crashes the pod (/root/reference/llm/rag.py:29-31),
the downloader swallows errors (llm/download_model.py:32-33), and a torn index file is read as-is
(rag.py:68-86,153-155). Here every recovery path has a hook that tests (and chaos runs of the
real server) can switch on without code changes:

  RAGK_FAULTS="index_read_error,missing_shard=2,engine_crash_at_step=5,step_delay_ms=300,embed_error"

  index_read_error       DocumentStore.load() sees an unreadable/corrupt index file
  missing_shard=N        the N-th (1-based) safetensors shard of the checkpoint is absent
  engine_crash_at_step=N LLMEngine.step() raises on its N-th call (engine-loop failure path)
  step_delay_ms=X        every engine step sleeps X ms (request timeouts, step watchdog)
  embed_error            the embedder raises (retrieval failure -> HTTP 500)
  comm_hang_s=X          a TP follower stalls X s before stepping (collective watchdog)
  bench_tp_hang_s=X      bench.py's TP=N C=1 phase stalls X s (its watchdog must exit non-zero)
  comm_skew_ms=X         every TP collective starts late on each rank by 0..X ms (per call and rank)
  mlp_engine_timeout_at_step=N  the N-th decode step's persistent MLP launches get a one-tick deadline
                         (every in-kernel wait gives up: the engine must discard and recompute the step)

`set_faults()` overrides the environment in-process (tests).
"""
from __future__ import annotations

import os
import threading

_lock = threading.Lock()
_override = None
_counters = {}


class FaultInjected(RuntimeError):
    pass


def _parse(spec):
    out = {}
    for item in (spec or "").split(","):
        item = item.strip()
        if not item:
            continue
        k, _, v = item.partition("=")
        out[k.strip()] = v.strip() if v else "1"
    return out


_env_cache = ("", {})


def faults():
    global _env_cache
    if _override is not None:
        return _override
    spec = os.environ.get("RAGK_FAULTS", "")
    if spec != _env_cache[0]:
        _env_cache = (spec, _parse(spec))
    return _env_cache[1]


def set_faults(spec):
    """In-process override ('' clears; None returns to the environment)."""
    global _override
    with _lock:
        _override = None if spec is None else _parse(spec)
        _counters.clear()


def value(name, default=None):
    return faults().get(name, default)


def active(name) -> bool:
    return name in faults()


def check(name, what=None):
    """Raise FaultInjected if fault `name` is on."""
    if name in faults():
        raise FaultInjected("injected fault %s%s" % (name, (": " + what) if what else ""))


def tick(name) -> int:
    """Per-fault call counter (1-based), for '..._at_step=N' style faults."""
    with _lock:
        _counters[name] = _counters.get(name, 0) + 1
        return _counters[name]
