"""RAG orchestration (reference L6, /root/reference/llm/rag.py:88-181).

Query path (reference generate_text, :146-181), per request:
  embed query -> search k -> top context_k into the prompt template -> tokenize (BOS, no chat
  template) -> generate(max_new_tokens, temperature, top_p) -> decode full sequence ->
  split("Chatbot:")[-1].strip() -> {"generated_text", "context"}.

Differences by design: concurrent requests are micro-batched through the embedder and the
index (one encoder forward + one search kernel per batch), and all generations share one
continuous-batching engine driven by a dedicated loop thread (the reference runs
independent model.generate calls per Flask thread). Ingest embeds every chunk of a PDF in
packed batches instead of one chunk at a time.
"""
from __future__ import annotations

import faulthandler
import logging
import os
import queue
import sys
import threading
import time

import numpy as np
import torch

from ..engine.llm_engine import SamplingParams
from ..ingest import pdf as pdfmod
from ..ingest.text import NO_RESULTS, build_context, build_prompt, chunk_metadata, postprocess, split_text
from ..utils import faults, metrics
from ..utils.metrics import Trace

log = logging.getLogger(__name__)


def _tp_bcast_prompts(comm, rows, flat_ids, lens, seeds):
    """TP leader -> every TP rank: row indices, token ids and seeds of the prompts to queue, as int
    buffers over the TP gloo group (no pickling, no per-token Python). flat_ids / lens: the leader's
    encode_batch_flat() output. Returns (rows, [int32 prompt arrays], seeds)."""
    import torch.distributed as dist

    grp = comm.cpu_group if comm.cpu_group is not None else comm.group
    src = dist.get_global_rank(grp, 0) if grp is not None else 0
    if comm.rank == 0:
        hdr = torch.tensor([len(rows), int(flat_ids.shape[0])], dtype=torch.int64)
    else:
        hdr = torch.zeros(2, dtype=torch.int64)
    dist.broadcast(hdr, src=src, group=grp)
    nr, nt = int(hdr[0]), int(hdr[1])
    if comm.rank == 0:
        meta = torch.from_numpy(np.stack([np.asarray(rows, dtype=np.int64), np.asarray(lens, dtype=np.int64),
                                          np.asarray(seeds, dtype=np.int64)]).reshape(3, nr))
        flat = torch.from_numpy(np.ascontiguousarray(flat_ids, dtype=np.int32))
    else:
        meta = torch.zeros((3, nr), dtype=torch.int64)
        flat = torch.zeros(nt, dtype=torch.int32)
    dist.broadcast(meta, src=src, group=grp)
    if nt:
        dist.broadcast(flat, src=src, group=grp)
    m = meta.numpy()
    out = np.split(flat.numpy(), np.cumsum(m[1])[:-1]) if nr else []
    return m[0].tolist(), out, m[2].tolist()


class _Job:
    def __init__(self, name, args):
        self.name, self.args = name, args
        self.done = threading.Event()
        self.result = self.error = None


class EngineLoop(threading.Thread):
    """Drives LLMEngine.step() on one thread; wakes when requests arrive.

    Collective jobs (tensor-parallel serving): work that every TP rank must run together -- the
    data-parallel ingest of an uploaded PDF, a search of a row-sharded index -- is queued here and run
    by this thread BETWEEN engine steps, after the job record has been published to the follower ranks
    (parallel/tp.py), so every rank executes the same collectives in the same order as its steps."""

    def __init__(self, engine, control=None):
        super().__init__(daemon=True, name="llm-engine-loop")
        self.engine = engine
        self.cv = threading.Condition()
        self.stop_flag = False
        self.control = control  # TP control channel (rank 0 side), see parallel/tp.py
        self.error = None
        self.step_started = None  # monotonic start of the step in flight (watchdog)
        self.steps = 0
        self.jobs = []
        self.job_fns = {}

    def run_job(self, name, args, timeout=None):
        """Run job `name` on every TP rank between two engine steps; returns this rank's result."""
        if self.error is not None:
            raise RuntimeError("engine loop failed: %r" % (self.error,))
        job = _Job(name, args)
        with self.cv:
            self.jobs.append(job)
            self.cv.notify()
        if not job.done.wait(timeout):
            with self.cv:  # not started yet: withdraw it, so the client's failure means "not done"
                if job in self.jobs:
                    self.jobs.remove(job)
                    raise TimeoutError("collective job %s not run within %ss (withdrawn)" % (name, timeout))
            raise TimeoutError("collective job %s still running after %ss" % (name, timeout))
        if job.error is not None:
            raise job.error
        return job.result

    def _run_jobs(self):
        with self.cv:
            jobs, self.jobs = self.jobs, []
        for job in jobs:
            try:
                if self.control is not None:
                    self.control.publish_job(job.name, job.args)
                job.result = self.job_fns[job.name](job.args)
            except Exception as e:
                job.error = e
                if self.control is not None:  # a half-run collective leaves the ranks out of step
                    raise
            finally:
                job.done.set()

    def submit(self, prompt_ids, params, seed=None):
        if self.control is not None:  # TP: admission is broadcast to the follower ranks first
            s = self.engine.make_sequence(prompt_ids, params, seed if seed is not None else 0)
            self.control.enqueue(s)
        else:
            s = self.engine.add_request(prompt_ids, params, seed=seed)
        with self.cv:
            self.cv.notify()
        return s

    def _idle(self):
        eng = self.engine
        pending = self.control.has_pending() if self.control is not None else False
        return not eng.has_work() and not pending and not self.jobs

    def run(self):
        from ..parallel.tp import HEARTBEAT_S

        eng = self.engine
        try:
            while not self.stop_flag:
                with self.cv:
                    while self._idle() and not self.stop_flag:
                        self.cv.wait(timeout=0.5)
                        if self.control is not None and time.time() - self.control.last_publish > HEARTBEAT_S:
                            self.control.publish_heartbeat()
                if self.stop_flag:
                    break
                if self.jobs:
                    self._run_jobs()
                    if self._idle():
                        continue
                self.step_started = time.monotonic()
                if self.control is not None:
                    self.control.publish_step(eng)
                fin = eng.step()
                self.step_started = None
                self.steps += 1
                metrics.set_gauge("kv_free", eng.bm.free_blocks())
                metrics.set_gauge("batch", len(eng.running))
                if self.steps % 64 == 1 and torch.cuda.is_available():
                    metrics.set_gauge("hbm", torch.cuda.memory_allocated())
                for s in fin:
                    metrics.inc("tokens", len(s.out))
                    if s.t_first is not None and s.t_done is not None and len(s.out) > 1:
                        metrics.observe("tpot", (s.t_done - s.t_first) / (len(s.out) - 1))
        except Exception as e:  # surface engine failure to every waiter
            log.exception("engine loop failed")
            self.error = e
            for s in list(eng.running) + list(eng.waiting):
                s.finish_reason = "error"
                s.done.set()
            with self.cv:
                jobs, self.jobs = self.jobs, []
            for job in jobs:
                job.error = RuntimeError("engine loop failed: %r" % (e,))
                job.done.set()
        finally:
            if self.control is not None:
                self.control.publish_shutdown()

    def stop(self):
        self.stop_flag = True
        with self.cv:
            self.cv.notify_all()


class Watchdog(threading.Thread):
    """Declares the engine hung when one step (its kernels + RCCL collectives) exceeds
    `step_timeout_s`: liveness turns 503 and, with `exit_on_hang`, the process dumps every
    thread's stack and exits so k8s restarts the pod (a wedged collective never returns)."""

    def __init__(self, loop, step_timeout_s, exit_on_hang, poll_s=1.0):
        super().__init__(daemon=True, name="engine-watchdog")
        self.loop, self.timeout, self.exit_on_hang, self.poll = loop, step_timeout_s, exit_on_hang, poll_s
        self.hung = False
        self.stop_flag = False

    def check(self, now=None):
        t0 = self.loop.step_started
        now = time.monotonic() if now is None else now
        if t0 is not None and now - t0 > self.timeout and not self.hung:
            self.hung = True
            log.critical("engine step running for %.1fs > step_timeout_s=%.1fs: declaring the engine hung",
                         now - t0, self.timeout)
            faulthandler.dump_traceback(file=sys.stderr, all_threads=True)
            if self.exit_on_hang:
                os._exit(70)
        return self.hung

    def run(self):
        while not self.stop_flag:
            time.sleep(self.poll)
            self.check()


class MicroBatcher(threading.Thread):
    """Collects concurrent retrieval requests for `window_s`, then embeds + searches them together."""

    def __init__(self, fn, window_s=0.002, max_batch=256):
        super().__init__(daemon=True, name="embed-batcher")
        self.fn, self.window_s, self.max_batch = fn, window_s, max_batch
        self.q = queue.Queue()

    def submit(self, item):
        ev = threading.Event()
        box = {}
        self.q.put((item, ev, box))
        ev.wait()
        if "error" in box:
            raise box["error"]
        return box["result"]

    def run(self):
        while True:
            first = self.q.get()
            batch = [first]
            deadline = time.perf_counter() + self.window_s
            while len(batch) < self.max_batch:
                t = deadline - time.perf_counter()
                if t <= 0:
                    break
                try:
                    batch.append(self.q.get(timeout=t))
                except queue.Empty:
                    break
            try:
                res = self.fn([b[0] for b in batch])
                for (item, ev, box), r in zip(batch, res):
                    box["result"] = r
                    ev.set()
            except Exception as e:
                for item, ev, box in batch:
                    box["error"] = e
                    ev.set()


class RagService:
    def __init__(self, cfg, llm_engine, llm_tokenizer, embedder, store, gen_config=None, start_threads=True,
                 control=None, tp_group=None):
        self.cfg = cfg
        self.engine = llm_engine
        self.tok = llm_tokenizer
        self.embedder = embedder
        self.store = store
        gen = gen_config or {}
        do_sample = cfg.do_sample if cfg.do_sample is not None else bool(gen.get("do_sample", True))
        eos = gen.get("eos_token_id")
        stop = tuple(eos) if isinstance(eos, list) else ((eos,) if eos is not None else ())
        self.params = SamplingParams(max_new_tokens=cfg.max_new_tokens, temperature=cfg.temperature,
                                     top_p=cfg.top_p, top_k=cfg.top_k, do_sample=do_sample, stop_token_ids=stop,
                                     ignore_eos=bool(getattr(cfg, "ignore_eos", False)))
        self.loop = EngineLoop(llm_engine, control=control)
        # tensor-parallel group (set by the TP server): PDF ingest is data-parallel over it and, with
        # INDEX_SHARDED, every rank holds a row shard of the index (both run as collective jobs)
        self.tp_group = tp_group
        self.collective = control is not None
        self.loop.job_fns.update(self.job_fns())
        self.watchdog = Watchdog(self.loop, cfg.step_timeout_s, cfg.watchdog_exit)
        self.batcher = MicroBatcher(self._retrieve_batch)
        self._seed = cfg.seed
        self._seed_lock = threading.Lock()
        self.ready = False
        if start_threads:
            self.loop.start()
            self.batcher.start()
            self.watchdog.start()

    # ------------------------------------------------------------------ retrieval
    # ------------------------------------------------------------------ collective jobs
    def job_fns(self):
        """Jobs every TP rank runs together (rank 0: engine-loop thread; followers: parallel/tp.follow)."""
        return {"ingest": self._job_ingest, "search": self._job_search}

    def _job_ingest(self, args):
        """Data-parallel embedding of one upload's chunks: rank r embeds chunks[r::world], the vectors are
        all-gathered (RCCL on GPUs) and added to the index -- by rank 0 only (replicated-index mode: only
        rank 0 retrieves), or by every rank for its row shard (INDEX_SHARDED)."""
        from ..parallel.dp import embed_distributed

        filename, chunks, dedupe, persist = args
        if self.collective or (self.tp_group is not None and not self.loop.is_alive()):
            vecs = embed_distributed(self.embedder, chunks, group=self.tp_group)
        else:  # single process (or a DP replica): never a collective over the default group
            vecs = self.embedder.embed(chunks)
        rank0 = self.tp_group is None or torch.distributed.get_rank(self.tp_group) == 0
        if rank0 or getattr(self.store, "sharded", False):
            self.store.add(vecs, chunk_metadata(filename, chunks), dedupe=dedupe, persist=persist)
        return len(chunks)

    def _job_search(self, args):
        """Row-sharded index: every rank searches its shard for rank 0's queries (followers pass none)."""
        q, k = args
        if q is None:
            q = torch.zeros((0, self.store.dim), dtype=torch.float32)
        return self.store.search(q, k)

    def _retrieve_batch(self, prompts):
        tr = Trace("retrieve")
        with tr.span("embed"):
            faults.check("embed_error")
            q = self.embedder.embed(list(prompts))
        with tr.span("search"):
            self.store.maybe_reload()
            if self.collective and getattr(self.store, "sharded", False):
                res = self.loop.run_job("search", (q.cpu(), self.cfg.retrieve_k), timeout=self.cfg.request_timeout_s)
            else:
                res = self.store.search(q, self.cfg.retrieve_k)
        return [(r, tr.spans) for r in res]

    def retrieve(self, prompt):
        return self.batcher.submit(prompt)

    # ------------------------------------------------------------------ generation
    def _next_seed(self):
        with self._seed_lock:
            self._seed += 1
            return self._seed

    def _decode_answer(self, prompt_ids, out_ids):
        """decode(prompt + out) as the reference does before its split on "Chatbot:", without
        re-decoding the ~5k prompt tokens: when the prompt's bytes end with "Chatbot:" (an ASCII
        boundary, so byte-level decoding of the concatenation is the concatenation of the decodes),
        the text after the last "Chatbot:" only depends on the generated part."""
        tail = self.tok.decode(prompt_ids[-8:], skip_special_tokens=True)
        if tail.endswith("Chatbot:"):
            return "Chatbot:" + self.tok.decode(out_ids, skip_special_tokens=True)
        return self.tok.decode(list(prompt_ids) + list(out_ids), skip_special_tokens=True)

    def _prompt_ids(self, full_prompt, ids=None):
        if ids is None:
            ids = self.tok.encode(full_prompt, add_special_tokens=True)
        elif not isinstance(ids, np.ndarray):
            ids = list(ids)
        limit = self.engine.max_model_len - self.params.max_new_tokens
        if len(ids) > limit:
            if self.cfg.truncate_prompt != "left":
                raise ValueError("prompt of %d tokens exceeds the model limit %d" % (len(ids), limit))
            ids = ids[len(ids) - limit:]  # keep the question and "Chatbot:" suffix
        return ids

    def generate(self, user_prompt, params=None, debug=False):
        """Synchronous /generate (thread-safe)."""
        tr = Trace("generate")
        results, rspans = self.retrieve(user_prompt)
        for k, v in rspans.items():
            tr.spans[k] = v
        log.debug("User query: %s", user_prompt)
        log.debug("Search results: %s", [(m.get("filename"), m.get("chunk_id"), d) for m, d in results])
        if not results:
            return {"generated_text": NO_RESULTS}
        context = build_context(results, self.cfg.context_k)
        log.debug("Context: %s...", context[:500])
        with tr.span("tokenize"):
            ids = self._prompt_ids(build_prompt(context, user_prompt))
        metrics.inc("prompt_tokens", len(ids))
        s = self.loop.submit(ids, params or self.params, seed=self._next_seed())
        if not s.done.wait(timeout=self.cfg.request_timeout_s):
            if self.loop.control is None:
                self.engine.abort(s)
            else:  # TP: every rank aborts it at the same step boundary
                self.loop.control.abort(s)
                with self.loop.cv:
                    self.loop.cv.notify()
            metrics.inc("timeouts")
            raise TimeoutError("generation timed out after %gs" % self.cfg.request_timeout_s)
        if s.finish_reason == "error":
            raise RuntimeError("generation engine failed: %r" % (self.loop.error,))
        tr.add("queue+prefill", (s.t_first or s.t_done) - s.t_arrive)
        tr.add("decode", s.t_done - (s.t_first or s.t_done))
        metrics.observe("ttft", (s.t_first or s.t_done) - s.t_arrive)
        with tr.span("detokenize"):
            text = postprocess(self._decode_answer(s.prompt, s.out))
        metrics.observe("request", tr.total())
        log.debug("Generated response: %s...", text[:200])
        out = {"generated_text": text, "context": context}
        if debug:
            out["timings_ms"] = tr.summary_ms()
            out["prompt_tokens"] = len(ids)
            out["generated_tokens"] = len(s.out)
        return out

    def generate_batch(self, prompts, params=None, seeds=None):
        """Many queries at once (benchmark / offline): one embed + one search + one engine run.
        Must not be mixed with the background loop (call with start_threads=False).

        Tensor parallel (every TP rank calls this with the same arguments): the TP leader embeds,
        searches, builds and tokenizes every prompt, broadcasts the token ids and seeds over the TP
        gloo group, and every rank queues ALL of them before its first step -- each rank's engine must
        see the same admissions at the same steps (TP has no per-step metadata exchange here)."""
        if self.loop.is_alive():  # two threads stepping one engine corrupt its running set
            raise RuntimeError("generate_batch needs exclusive use of the engine: build the service "
                               "with start_threads=False")
        t0 = time.perf_counter()
        eng = self.engine
        comm = getattr(eng, "comm", None)
        tp = eng.tp_size > 1 and comm is not None
        lead = (not tp) or comm.rank == 0
        n = len(prompts)
        ctxs, fulls = [None] * n, [None] * n
        if lead:
            q = self.embedder.embed(list(prompts))
            res = self.store.search(q, self.cfg.retrieve_k)
            for i, (p, r) in enumerate(zip(prompts, res)):
                if r:
                    ctxs[i] = build_context(r, self.cfg.context_k)
                    fulls[i] = build_prompt(ctxs[i], p)
        t_ret = time.perf_counter()
        rows = [i for i in range(n) if fulls[i] is not None]
        seqs = [None] * n
        seed_of = {i: (seeds[i] if seeds is not None else self._next_seed()) for i in rows}
        p_use = params or self.params
        queued = []

        def submit(idx, id_lists):
            for i, ids in zip(idx, id_lists):
                seqs[i] = eng.add_request(self._prompt_ids(None, ids=ids), p_use, seed=seed_of[i])
                queued.append(seqs[i])

        rest, err, t_rest = None, [], []
        if tp:
            flat, lens = (self.tok.encode_batch_flat([fulls[i] for i in rows], add_special_tokens=True)
                          if lead else (None, None))
            rows, id_lists, sd = _tp_bcast_prompts(comm, rows, flat, lens,
                                                   [seed_of[i] for i in rows] if lead else None)
            seed_of = dict(zip(rows, sd))
            submit(rows, id_lists)
        else:
            # Multi-threaded tokenizer calls (C++ workers, GIL released). The first few prompts -- about
            # one prefill step's worth -- are tokenized and submitted right away; the rest are tokenized
            # on a helper thread while the GPU runs that first prefill step, and join the queue in order.
            head = max(1, eng.max_prefill_tokens // max(1, 4 * self.cfg.chunk_words))  # ~1 step of prompts
            submit(rows[:head], self.tok.encode_batch([fulls[i] for i in rows[:head]], add_special_tokens=True))
            if len(rows) > head:
                def _rest():
                    try:
                        tail = rows[head:]
                        submit(tail, self.tok.encode_batch([fulls[i] for i in tail], add_special_tokens=True))
                        t_rest.append(time.perf_counter())
                    except Exception as e:  # surfaced below, after the engine drains
                        err.append(e)
                rest = threading.Thread(target=_rest, daemon=True)
                rest.start()
        t_prep = time.perf_counter()
        ok = False
        try:
            while True:
                if eng.has_work():
                    eng.step()
                elif rest is not None and rest.is_alive():
                    rest.join(0.001)
                elif not eng.has_work():  # re-check: the helper may have queued its last rows and exited
                    break
            ok = True
        finally:
            if rest is not None:
                rest.join()
            if not ok:  # a failed step: nothing this call queued may run in a later call
                for s in queued:
                    if s.status != 2:
                        eng.abort(s)
                try:
                    eng._apply_aborts()
                except Exception:
                    pass
        if err:
            raise err[0]
        st = eng.stats
        st["retrieve_s"] = st.get("retrieve_s", 0.0) + (t_ret - t0)
        st["prompt_build_s"] = st.get("prompt_build_s", 0.0) + (t_prep - t_ret)
        if t_rest:  # when the helper thread had queued the tail prompts (after the head's first step)
            st["tail_queued_s"] = st.get("tail_queued_s", 0.0) + (t_rest[0] - t_prep)
        outs = []
        for s, ctx in zip(seqs, ctxs):
            if s is None:
                outs.append({"generated_text": NO_RESULTS})
                continue
            text = postprocess(self._decode_answer(s.prompt, s.out))
            outs.append({"generated_text": text, "context": ctx, "_latency_s": s.t_done - t0,
                         "_ttft_s": (s.t_first or s.t_done) - t0, "_prompt_tokens": len(s.prompt),
                         "_gen_tokens": len(s.out)})
        return outs

    # ------------------------------------------------------------------ ingest
    def ingest_pdf_bytes(self, filename, data, persist=True):
        """Reference upload_pdf/process_pdf: extract -> chunk -> embed -> update_index."""
        text = pdfmod.extract_text(data)
        chunks = split_text(text, self.cfg.chunk_words, self.cfg.chunk_overlap)
        if chunks:
            args = (filename, chunks, not self.cfg.reingest_append, persist)
            if self.collective:  # tensor-parallel server: every rank embeds a share (data-parallel ingest)
                self.loop.run_job("ingest", args, timeout=self.cfg.request_timeout_s)
            else:
                self._job_ingest(args)
            metrics.set_gauge("index", self.store.index.ntotal)
        return len(chunks)

    def ingest_directory(self):
        """Reference process_pdf_directory(): every *.pdf in PDF_DIR (idempotent by default)."""
        d = self.cfg.pdf_dir
        if not os.path.isdir(d):
            log.warning("No PDF files found in %s", d)
            return 0
        files = sorted(f for f in os.listdir(d) if f.endswith(".pdf"))
        if not files:
            log.warning("No PDF files found in %s", d)
            return 0
        total = 0
        for fn in files:
            with open(os.path.join(d, fn), "rb") as f:
                # collective (TP) ingest: every rank snapshots what it holds, in the background
                total += self.ingest_pdf_bytes(fn, f.read(), persist=self.collective)
        if self.collective:
            self.store.flush()
        else:
            self.store.persist()
        log.info("Processed %d PDFs into %d chunks", len(files), total)
        return len(files)

    def index_info(self):
        self.store.maybe_reload()
        return self.store.info()

    def health(self):
        comm = getattr(self.engine, "comm", None)
        comm_ok = comm is None or getattr(comm, "broken", None) is None
        alive = self.loop.is_alive() and self.loop.error is None and not self.watchdog.hung and comm_ok
        return {"engine_alive": alive, "ready": self.ready, "engine_steps": self.loop.steps, "comm_ok": comm_ok,
                "engine_error": None if self.loop.error is None else repr(self.loop.error),
                "kv_free_blocks": self.engine.bm.free_blocks(), "index_vectors": int(self.store.index.ntotal),
                "hbm_bytes": torch.cuda.memory_allocated() if torch.cuda.is_available() else 0}

    def shutdown(self):
        self.watchdog.stop_flag = True
        self.loop.stop()
        try:
            self.store.flush()
        except Exception as e:
            log.error("index snapshot on shutdown failed: %s", e)
