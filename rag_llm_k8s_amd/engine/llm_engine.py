"""Continuous-batching generation engine (replaces transformers' generate loop, D2).

Reference loop ([dep] generation/utils.py _sample, driven from /root/reference/llm/rag.py:172):
one prompt at a time, DynamicCache, temperature -> top-k(50) -> top-p -> multinomial, stop on
EOS or max_new_tokens. The reference runs concurrent Flask requests as independent
generate() calls with no batching.

Here:
  * requests join a waiting queue; each engine step is either a PREFILL step (new prompts,
    packed varlen, chunked to `max_prefill_tokens`) or a DECODE step over every running
    sequence (continuous batching: sequences enter/leave between steps);
  * KV lives in a paged cache (64-token blocks, block manager); admission reserves the
    blocks for prompt + max_new_tokens, so a running sequence is never preempted;
  * decode steps replay a hipGraph per batch-size bucket (static input buffers, one H2D
    copy of a packed metadata block, sampling inside the graph); the host only reads back
    the sampled token ids;
  * tensor parallel: every TP rank runs the same deterministic schedule on the same inputs
    (rank 0 broadcasts new requests), so no per-step metadata broadcast is needed.
"""
from __future__ import annotations

import itertools
import logging
import os
import threading
import time
from collections import deque
from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np
import torch

from ..models.llama import StepInput
from ..ops.backend import AttnMeta
from ..utils import faults
from .kv_manager import BLOCK, make_block_manager

# decode batches up to this size split each row's top-k over ~31 chunks of ~4k logits (topk_wave_kernel,
# threshold-filtered lane networks, merged by the sampler's lane network); larger batches use 7
# radix-select chunks (topk_lds). tools/sampler_bench.py: top-k + sample 21.0 us at batch 1 (7 chunks:
# 40.1), 33.6 us at batch 32 (7 chunks: 41.2) -- profiles/sampler_bench_r3.log
SMALL_BATCH_TOPK_MAX_B = 64
SMALL_BATCH_TOPK_CHUNK = 4096

log = logging.getLogger(__name__)


@dataclass
class SamplingParams:
    max_new_tokens: int = 150
    temperature: float = 0.7
    top_p: float = 0.9
    top_k: int = 50
    do_sample: bool = True
    seed: Optional[int] = None
    stop_token_ids: tuple = ()
    ignore_eos: bool = False  # benchmark mode: always generate max_new_tokens


WAITING, RUNNING, FINISHED = 0, 1, 2


class Sequence:
    _ids = itertools.count()

    def __init__(self, prompt_ids, params: SamplingParams, seed: int):
        self.id = next(Sequence._ids)
        if isinstance(prompt_ids, np.ndarray):  # int32 buffers (TP admission broadcast)
            self.prompt_np = np.ascontiguousarray(prompt_ids, dtype=np.int32)
            self.prompt = self.prompt_np.tolist()
        else:
            self.prompt = list(prompt_ids)
            self.prompt_np = np.asarray(self.prompt, dtype=np.int32)  # vectorised prefill input building
        self.out: List[int] = []
        self.params = params
        self.seed = seed
        self.computed = 0  # tokens whose K/V is in the cache
        self.status = WAITING
        self.t_arrive = time.perf_counter()
        self.t_first = None
        self.t_done = None
        self.finish_reason = None
        self.done = threading.Event()
        self.user = None  # opaque payload for the caller

    @property
    def length(self):
        return len(self.prompt) + len(self.out)

    def token_at(self, i):
        n = len(self.prompt)
        return self.prompt[i] if i < n else self.out[i - n]


class LLMEngine:
    def __init__(self, model, num_blocks: int, max_batch: int = 64, max_prefill_tokens: int = 32768,
                 max_model_len: int = 16384, eos_ids=(), use_graphs: bool = True, tp_group=None, top_k_cap: int = 64,
                 graph_buckets=None, mixed_prefill_tokens: int = 0):
        self.model = model
        self.device = model.device
        self.max_batch = max_batch
        self.max_prefill_tokens = max_prefill_tokens
        # Decode-aware prefill budget (served path): a step that carries decoding rows takes at most this
        # many prompt tokens, so the rows' per-token latency (TPOT) is one short step, not a whole
        # max_prefill_tokens chunk; with nothing decoding the full budget applies (TTFT, throughput).
        # 0 = off (offline batch / the headline bench: its wave is throughput-bound).
        self.mixed_prefill_tokens = int(mixed_prefill_tokens or 0)
        self.max_model_len = max_model_len
        self.eos = set(int(e) for e in eos_ids)
        self.bm = make_block_manager(num_blocks)
        self.max_blocks = -(-max_model_len // BLOCK)
        model.allocate_kv_cache(num_blocks)
        self.waiting = deque()
        self.running: List[Sequence] = []
        self.lock = threading.Lock()
        self._aborts = []
        self.tp_group = tp_group
        self.comm = getattr(model, "comm", None)
        if self.comm is not None and self.comm.size > 1:
            self.tp_size = self.comm.size
        else:
            self.tp_size = 1 if tp_group is None else torch.distributed.get_world_size(tp_group)
        # candidate-list width of the native sampler (top-k <= K served inside the decode graph);
        # requests with a larger top_k, or top_k = 0 (HF: disabled), take the exact full-vocabulary path
        self.K = top_k_cap
        self._warned_topk = False
        # TP prefill steps of at least this many tokens run as 2 micro-batches with async all-reduces
        self.tp_overlap_min_tokens = 1024
        self.is_cuda = self.device.type == "cuda"
        self.use_graphs = use_graphs and self.is_cuda
        self.buckets = sorted(set(graph_buckets or [b for b in (1, 2, 4, 8, 16, 24, 32, 48, 64, 96, 128, 192, 256)
                                                    if b <= max_batch] + [max_batch]))
        self.graphs = {}
        # RAGK_DECODE_TIMING=1: (start, end) CUDA events around every async decode graph replay
        self._timing = [] if os.environ.get("RAGK_DECODE_TIMING") == "1" else None
        self.stats = dict(prefill_steps=0, decode_steps=0, prefill_tokens=0, decode_tokens=0, prefill_s=0.0,
                          decode_s=0.0)
        # two pinned staging buffers, alternated per step: with the asynchronous decode pipeline a
        # step's H2D copy may still be pending while the host stages the next one
        self._pins = [torch.empty(1 << 20 if self.is_cuda else 0, dtype=torch.int32, pin_memory=self.is_cuda)
                      for _ in range(2)]
        self._pin_idx = 0
        self._pin = self._pins[0]
        self._pin_off = 0
        # Asynchronous decode (hipGraph path): step t+1 is enqueued before step t's tokens are read
        # back; its input ids come from step t's sampled tokens on the device (D2D), so the GPU never
        # waits for the host round trip between decode steps. Tokens are accepted one step late; a
        # sequence that stops on EOS has computed one extra (discarded) row, and its KV blocks are
        # freed only after that step has completed. Under TP every rank samples the same token from
        # the same gathered candidates, so all ranks take the same decisions one step late.
        self.async_decode = self.use_graphs and os.environ.get("RAGK_ASYNC_DECODE", "1") == "1"
        # Mixed prefill + decode steps (chunked prefill): a step that admits prompt tokens
        # also advances every decoding sequence by one token through the same forward.
        self.mixed_steps = os.environ.get("RAGK_MIXED_STEPS", "1") == "1"
        self._inflight = None  # dict(seqs, rows, entry, event, host_out, n)
        self._free_after = []  # seq ids whose blocks are freed once the in-flight step has completed
        self._out_pins = [torch.empty(max(1, max_batch), dtype=torch.int32, pin_memory=self.is_cuda)
                          for _ in range(2)]
        self._out_idx = 0
        # sampled tokens of every decode graph land in this one device buffer: the next step's graph
        # (any bucket) reads its carried ids from it inside the embedding kernel (packed "carry" map)
        self._tok_out = torch.zeros(max(self.buckets + [max_batch, 1]), dtype=torch.int32,
                                    device=self.device) if self.is_cuda else None

    # ------------------------------------------------------------------ requests
    def add_request(self, prompt_ids, params: SamplingParams, seed: Optional[int] = None) -> Sequence:
        if len(prompt_ids) == 0:
            raise ValueError("empty prompt")
        if len(prompt_ids) + params.max_new_tokens > self.max_model_len:
            raise ValueError("prompt (%d) + max_new_tokens (%d) exceeds max_model_len %d"
                             % (len(prompt_ids), params.max_new_tokens, self.max_model_len))
        s = Sequence(prompt_ids, params, seed if seed is not None else (params.seed if params.seed is not None
                                                                        else int(time.time_ns() & 0xFFFFFFFF)))
        with self.lock:
            self.waiting.append(s)
        return s

    def make_sequence(self, prompt_ids, params: SamplingParams, seed: int) -> Sequence:
        if len(prompt_ids) == 0:
            raise ValueError("empty prompt")
        if len(prompt_ids) + params.max_new_tokens > self.max_model_len:
            raise ValueError("prompt (%d) + max_new_tokens (%d) exceeds max_model_len %d"
                             % (len(prompt_ids), params.max_new_tokens, self.max_model_len))
        return Sequence(prompt_ids, params, seed)

    def add_sequence(self, s: Sequence):
        with self.lock:
            self.waiting.append(s)
        return s

    def has_work(self):
        return bool(self.waiting) or bool(self.running) or self._inflight is not None

    # ------------------------------------------------------------------ scheduling
    def _admit(self, reserve=0):
        """Pick (seq, start, n) prefill chunks for this step (`reserve` tokens of the budget are taken
        by decode rows riding along in a mixed step)."""
        chunks = []
        budget = self.max_prefill_tokens
        if reserve and self.mixed_prefill_tokens > 0:
            budget = min(budget, self.mixed_prefill_tokens + reserve)
        budget -= reserve
        # continue partially-prefilled running sequences first
        for s in self.running:
            if s.computed < len(s.prompt) and budget > 0:
                n = min(len(s.prompt) - s.computed, budget)
                chunks.append((s, s.computed, n))
                budget -= n
        with self.lock:
            while self.waiting and budget > 0 and len(self.running) < self.max_batch:
                s = self.waiting[0]
                need = len(s.prompt) + s.params.max_new_tokens
                if not self.bm.can_allocate(s.id, need):
                    break
                self.waiting.popleft()
                self.bm.ensure(s.id, need)
                s.status = RUNNING
                self.running.append(s)
                n = min(len(s.prompt), budget)
                chunks.append((s, 0, n))
                budget -= n
        return chunks

    def abort(self, s: Sequence):
        """Cancel a sequence (request timeout / client gone); applied at the next step boundary."""
        with self.lock:
            self._aborts.append(s)

    def _apply_aborts(self):
        with self.lock:
            ab, self._aborts = self._aborts, []
            for s in ab:
                if s in self.waiting:
                    self.waiting.remove(s)
                    s.status, s.finish_reason, s.t_done = FINISHED, "abort", time.perf_counter()
                    s.done.set()
        for s in ab:
            if s in self.running:
                self._finish(s, "abort")

    def _fault_hooks(self):
        f = faults.faults()
        if not f:
            return
        if "engine_crash_at_step" in f and faults.tick("engine_crash_at_step") >= int(f["engine_crash_at_step"]):
            raise faults.FaultInjected("injected engine failure")
        if "step_delay_ms" in f:
            time.sleep(float(f["step_delay_ms"]) / 1000.0)

    def step(self):
        """One engine step. Returns the sequences that finished in it (with asynchronous decode:
        whose last token was read back in it). Under TP a failed collective raises CommError."""
        fin = self._step()
        if self.comm is not None and self.tp_size > 1:
            self.comm.check()
        return fin

    def _step(self):
        self._pin_idx ^= 1
        self._pin = self._pins[self._pin_idx]
        self._pin_off = 0
        fin = []
        if self._aborts:
            fin += self._drain()
            self._apply_aborts()
        self._fault_hooks()
        n_ready = sum(1 for s in self.running if s.computed >= len(s.prompt)) if self.mixed_steps else 0
        chunks = self._admit(reserve=n_ready)
        if chunks:
            fin += self._drain()
            rows = []
            if self.mixed_steps:
                # mixed step: every running sequence past its prompt rides along as a 1-token chunk (its
                # last sampled token), so a long prefill does not stall the decoding requests
                inchunk = set(id(c[0]) for c in chunks)
                rows = [(s, s.length - 1, 1) for s in self.running
                        if id(s) not in inchunk and s.computed >= len(s.prompt) and s.computed == s.length - 1]
            return fin + self._prefill(chunks + rows, n_decode=len(rows))
        ready = [s for s in self.running if s.computed >= len(s.prompt)]
        if ready and self._needs_full_vocab(ready):
            fin += self._drain()
            ready = [s for s in self.running if s.computed >= len(s.prompt)]
            return fin + self._decode(ready, full_vocab=True)
        if ready and self.async_decode:
            return fin + self._decode_async(ready)
        fin += self._drain()
        ready = [s for s in self.running if s.computed >= len(s.prompt)]
        if ready:
            return fin + self._decode(ready)
        return fin

    def run_until_done(self, callback=None):
        finished = []
        while self.has_work():
            f = self.step()
            finished.extend(f)
            if callback:
                for s in f:
                    callback(s)
        return finished

    def generate(self, prompts, params: SamplingParams, seeds=None):
        seqs = [self.add_request(p, params, seed=None if seeds is None else seeds[i]) for i, p in enumerate(prompts)]
        self.run_until_done()
        return [s.out for s in seqs]

    # ------------------------------------------------------------------ helpers
    def _h2d_i32(self, host_list):
        """Stage a host int list / int32 array through a pinned buffer. Two buffers alternate per step
        (step() flips _pin_idx and resets the offset). Invariant: pin[i] is reused by step t+2 only;
        every path that enqueues step t+1 first synchronises step t-1 (a synchronous step ends with a
        device->host sync; the asynchronous decode pipeline _collect()s step t-1 before returning from
        step t+1, and _drain()s before any prefill), so step t-1's H2D copies out of pin[i] have
        completed before step t+1 overwrites it. A third in-flight step would break this."""
        if isinstance(host_list, np.ndarray):
            t = torch.from_numpy(np.ascontiguousarray(host_list, dtype=np.int32))
        else:
            t = torch.tensor(host_list, dtype=torch.int32)
        if not self.is_cuda:
            return t
        n = t.numel()
        if self._pin_off + n > self._pin.numel():
            cap = max(1 << 20, 2 * (self._pin_off + n))
            torch.cuda.current_stream(self.device).synchronize()
            self._pin = torch.empty(cap, dtype=torch.int32, pin_memory=True)
            self._pins[self._pin_idx] = self._pin
            self._pin_off = 0
        buf = self._pin[self._pin_off:self._pin_off + n]
        self._pin_off += n
        buf.copy_(t.reshape(-1))
        return buf.to(self.device, non_blocking=True).reshape(t.shape)

    def _finish(self, s, reason, defer_free=False):
        s.status = FINISHED
        s.finish_reason = reason
        s.t_done = time.perf_counter()
        if defer_free:  # a step still in flight writes this sequence's KV row
            self._free_after.append(s.id)
        else:
            self.bm.free(s.id)
        self.running.remove(s)
        s.done.set()

    def _accept(self, s, tok):
        if s.t_first is None:
            s.t_first = time.perf_counter()
        s.out.append(int(tok))
        p = s.params
        if not p.ignore_eos and (int(tok) in self.eos or int(tok) in p.stop_token_ids):
            return "stop"
        if len(s.out) >= p.max_new_tokens:
            return "length"
        if s.length >= self.max_model_len:
            return "length"
        return None

    def _sampling_host(self, seqs, pad_to=None):
        """int32 [6n] = seeds (int64, n) | temps (f32) | top_p (f32) | top_k | steps -- one H2D copy."""
        n = pad_to or len(seqs)
        seeds = np.zeros(n, dtype=np.int64)
        temps = np.zeros(n, dtype=np.float32)
        ps = np.ones(n, dtype=np.float32)
        ks = np.ones(n, dtype=np.int32)
        steps = np.zeros(n, dtype=np.int32)
        for i, s in enumerate(seqs):
            p = s.params
            temps[i] = p.temperature if p.do_sample else 0.0
            ks[i] = p.top_k if 0 < p.top_k <= self.K else self.K  # wider top_k: see _needs_full_vocab
            ps[i] = p.top_p
            seeds[i] = int(s.seed) & 0x7FFFFFFFFFFFFFFF
            steps[i] = len(s.out)
        return np.concatenate([seeds.view(np.int32), temps.view(np.int32), ps.view(np.int32), ks, steps])

    @staticmethod
    def _sampling_views(buf, n):
        """(temps, ks, ps, seeds, steps) views of a packed int32 [6n] buffer (seeds first: 8-B aligned)."""
        return (buf[2 * n:3 * n].view(torch.float32), buf[4 * n:5 * n], buf[3 * n:4 * n].view(torch.float32),
                buf[0:2 * n].view(torch.int64), buf[5 * n:6 * n])

    def _sampling_tensors(self, seqs, pad_to=None):
        n = pad_to or len(seqs)
        buf = self._h2d_i32(self._sampling_host(seqs, pad_to))
        return self._sampling_views(buf, n)

    def _needs_full_vocab(self, seqs):
        """True if a sampled request's top_k does not fit the K-wide candidate lists (top_k = 0 means
        "disabled" as in transformers' TopKLogitsWarper, top_k > K): such a step samples from the full
        vocabulary (exact, slower, outside the decode graph) instead of silently clamping top_k."""
        bad = any(s.params.do_sample and s.params.temperature > 0 and not (0 < s.params.top_k <= self.K)
                  for s in seqs)
        if bad and not self._warned_topk:
            log.warning("top_k outside 1..%d requested: sampling those steps from the full vocabulary", self.K)
            self._warned_topk = True
        return bad

    def _sample_full_vocab(self, logits, seqs):
        """Exact temperature -> top-k (if 0 < top_k) -> top-p -> multinomial over the whole vocabulary
        (transformers' LogitsProcessor order, [dep] generation/utils.py:1311-1322). Under TP the vocab
        shards are all-gathered first. Uniforms come from torch.Generator(seed * 1000003 + step), as in
        the torch backend's sampler."""
        w = self.model.w
        lg = logits[:, :w.vocab_valid].float().contiguous()
        if self.tp_size > 1:
            import torch.distributed as dist

            # every rank contributes its FULL (padded) shard width -- the last shard is narrower when
            # vocab_size % tp != 0, and collectives need equal sizes -- with -inf in the pad columns;
            # the concatenation is then cut back to vocab_size
            lp = logits.float().clone()
            lp[:, w.vocab_valid:] = float("-inf")
            if lg.is_cuda and self.comm is not None and self.comm.ipc is None:
                parts = [torch.empty_like(lp) for _ in range(self.tp_size)]
                dist.all_gather(parts, lp.contiguous(), group=self.tp_group)
            else:  # host-side over the gloo group (CPU / peer-mapped ranks)
                grp = getattr(self.comm, "cpu_group", None) or self.tp_group
                lp = lp.cpu()
                parts = [torch.empty_like(lp) for _ in range(self.tp_size)]
                dist.all_gather(parts, lp, group=grp)
            lg = torch.cat([p.cpu() for p in parts], 1)[:, :self.model.cfg.vocab_size]
        lg = lg.cpu()
        toks = []
        for b, s in enumerate(seqs):
            p = s.params
            x = lg[b]
            if not p.do_sample or p.temperature <= 0:
                toks.append(int(torch.argmax(x)))
                continue
            x = x / p.temperature
            if p.top_k > 0:
                kth = torch.topk(x, min(p.top_k, x.numel())).values[-1]
                x = torch.where(x < kth, torch.full_like(x, float("-inf")), x)
            sv, order = torch.sort(x, descending=True)
            probs = torch.softmax(sv, 0)
            keep = (torch.cumsum(probs, 0) - probs) < p.top_p
            keep[0] = True
            q = torch.where(keep, probs, torch.zeros_like(probs))
            c = torch.cumsum(q, 0)
            g = torch.Generator().manual_seed((int(s.seed) * 1000003 + len(s.out)) & 0x7FFFFFFFFFFFFFFF)
            u = float(torch.rand(1, generator=g)) * float(c[-1])
            j = min(int(torch.searchsorted(c, torch.tensor([u]), right=True)[0]), int(keep.sum()) - 1)
            toks.append(int(order[j]))
        return toks

    def _sample_rows(self, logits, temps, ks, ps, seeds, steps, out=None):
        be = self.model.be
        w = self.model.w
        lg = logits[:, :w.vocab_valid] if w.vocab_valid < logits.shape[1] else logits
        # chunk count from the padded shard width so every TP rank gathers equal-sized lists,
        # and all ranks' candidates together fit the sampler's 2048-entry merge
        from ..ops.native import topk_chunks
        chunks = topk_chunks(logits.shape[1], self.K, min(512, 2048 // self.tp_size))
        if logits.shape[0] <= SMALL_BATCH_TOPK_MAX_B:
            # small decode batch: 7 workgroups of ~18k logits each left the top-k latency-bound (25 us
            # at batch 1); ~4k-entry chunks use ~31 CUs and the sampler merges up to 2048 candidates
            chunks = max(1, min(logits.shape[1] // SMALL_BATCH_TOPK_CHUNK, (2048 // self.tp_size) // self.K, 64))
        cv, ci = be.topk_candidates(lg.contiguous() if not lg.is_contiguous() else lg, self.K,
                                    vocab_offset=w.vocab_offset, chunks=chunks)
        if self.tp_size > 1:
            cv, ci = self._gather_candidates(cv, ci)
        tok = be.sample_candidates(cv, ci, temps, ks, ps, seeds, steps, list_len=self.K)
        if out is not None:
            out.copy_(tok)
            return out
        return tok

    def _gather_candidates(self, cv, ci):
        if self.comm is not None:
            return self.comm.gather_candidates(cv, ci)
        import torch.distributed as dist

        B, K = cv.shape
        if cv.is_cuda:
            gv = torch.empty((self.tp_size, B, K), dtype=cv.dtype, device=cv.device)
            gi = torch.empty((self.tp_size, B, K), dtype=ci.dtype, device=ci.device)
            dist.all_gather_into_tensor(gv, cv.contiguous(), group=self.tp_group)
            dist.all_gather_into_tensor(gi, ci.contiguous(), group=self.tp_group)
        else:  # gloo (CPU plumbing / tests)
            lv = [torch.empty_like(cv) for _ in range(self.tp_size)]
            li = [torch.empty_like(ci) for _ in range(self.tp_size)]
            dist.all_gather(lv, cv.contiguous(), group=self.tp_group)
            dist.all_gather(li, ci.contiguous(), group=self.tp_group)
            gv, gi = torch.stack(lv), torch.stack(li)
        return gv.permute(1, 0, 2).reshape(B, self.tp_size * K).contiguous(), \
            gi.permute(1, 0, 2).reshape(B, self.tp_size * K).contiguous()

    # ------------------------------------------------------------------ prefill
    def _prefill_input(self, chunks):
        """Packed StepInput for prefill chunks [(seq, start, n)] + the sequences whose prompt ends here.
        Built with numpy slices (a 32k-token step took ~20 ms of per-token Python before)."""
        ids, pos, slots, cu, kvl, qlens, out_rows, out_seqs = [], [], [], [0], [], [], [], []
        bts = np.zeros((len(chunks), self.max_blocks), dtype=np.int32)
        for ci, (s, start, n) in enumerate(chunks):
            table = np.asarray(self.bm.table(s.id), dtype=np.int32)
            p = np.arange(start, start + n, dtype=np.int32)
            if start + n <= len(s.prompt):
                ids.append(s.prompt_np[start:start + n])
            else:  # a decode row of a mixed step: the generated tokens past the prompt
                ids.append(np.asarray([s.token_at(i) for i in range(start, start + n)], dtype=np.int32))
            pos.append(p)
            slots.append(table[p // BLOCK] * BLOCK + p % BLOCK)
            cu.append(cu[-1] + n)
            kvl.append(start + n)
            qlens.append(n)
            nb = min(len(table), self.max_blocks)
            bts[ci, :nb] = table[:nb]
            if start + n == len(s.prompt) or (start + n == s.length and start >= len(s.prompt)):
                out_rows.append(cu[-1] - 1)
                out_seqs.append(s)
        from ..ops.native import build_prefill_tiles

        m = self.model
        tiles = build_prefill_tiles(qlens, m.Hq, m.Hkv)
        meta = AttnMeta("prefill", self._h2d_i32(kvl), self._h2d_i32(bts), cu_q=self._h2d_i32(cu),
                        tiles=tiles.to(self.device), host_kv_lens=kvl, host_q_lens=qlens)
        ntok = cu[-1]
        inp = StepInput(self._h2d_i32(np.concatenate(ids)), self._h2d_i32(np.concatenate(pos)),
                        self._h2d_i32(np.concatenate(slots)), meta,
                        self._h2d_i32(out_rows) if out_rows else self._h2d_i32([ntok - 1]))
        return inp, out_seqs, ntok

    @staticmethod
    def _split_chunks(chunks, parts):
        """Cut the packed token stream into `parts` nearly equal consecutive pieces (a chunk may be
        cut in two: its second piece continues the same sequence at a later position)."""
        total = sum(n for _, _, n in chunks)
        target = -(-total // parts)
        out, cur, room = [], [], target
        for s, start, n in chunks:
            while n > 0:
                k = min(n, room)
                cur.append((s, start, k))
                start, n, room = start + k, n - k, room - k
                if room == 0 and len(out) < parts - 1:
                    out.append(cur)
                    cur, room = [], target
        if cur:
            out.append(cur)
        return out

    def _prefill(self, chunks, n_decode=0):
        t0 = time.perf_counter()
        m = self.model
        ntok = sum(n for _, _, n in chunks)
        comm = getattr(m, "comm", None)
        overlap = (self.tp_size > 1 and comm is not None and hasattr(comm, "all_reduce_async")
                   and ntok >= self.tp_overlap_min_tokens and not getattr(m, "seq_parallel", False))
        if overlap:
            groups = self._split_chunks(chunks, 2)
            built = [self._prefill_input(g) for g in groups]
            hs = m.hidden_states_microbatched([b[0] for b in built])
            out_seqs = [s for b in built for s in b[1]]
            parts = [m.logits(h) for h, b in zip(hs, built) if b[1]]
            logits = torch.cat(parts, 0) if parts else None
        else:
            inp, out_seqs, _ = self._prefill_input(chunks)
            logits = m.forward(inp) if out_seqs else None
            if logits is None:
                m.hidden_states(inp)
        finished = []
        if out_seqs and self._needs_full_vocab(out_seqs):
            tok = self._sample_full_vocab(logits, out_seqs)
        elif out_seqs:
            tok = self._sample_rows(logits, *self._sampling_tensors(out_seqs)).cpu().tolist()
        else:
            tok = []
            if self.is_cuda:
                torch.cuda.current_stream(self.device).synchronize()
        for s, start, n in chunks:
            s.computed = start + n
        for s, t in zip(out_seqs, tok):
            r = self._accept(s, t)
            if r:
                self._finish(s, r)
                finished.append(s)
        self.stats["prefill_steps"] += 1
        self.stats["prefill_tokens"] += ntok - n_decode
        if n_decode:
            self.stats["mixed_decode_tokens"] = self.stats.get("mixed_decode_tokens", 0) + n_decode
        self.stats["prefill_s"] += time.perf_counter() - t0
        return finished

    # ------------------------------------------------------------------ decode
    def _bucket(self, n):
        for b in self.buckets:
            if b >= n:
                return b
        return n

    def _bt_row(self, s, need_blocks):
        """Cached, max_blocks-padded numpy block-table row of a sequence. Blocks for prompt +
        max_new_tokens are allocated at admission, so the row is built once per sequence (the
        per-step list -> array conversion was ~10 us per sequence)."""
        row = getattr(s, "_bt_np", None)
        if row is None or s._bt_nb < need_blocks:
            table = self.bm.table(s.id)
            nb = min(len(table), self.max_blocks)
            row = np.zeros(self.max_blocks, dtype=np.int32)
            row[:nb] = table[:nb]
            s._bt_np, s._bt_nb = row, nb
        return row

    def _decode_inputs_host(self, seqs, B):
        """Packed int32 metadata: ids[B] pos[B] slots[B] kv_lens[B] bt[B*maxb] (+ pad to even)."""
        mb = self.max_blocks
        n = len(seqs)
        out = np.zeros(4 * B + B * mb + (4 * B + B * mb) % 2, dtype=np.int32)
        ids, pos, slots, kvl = (out[i * B:(i + 1) * B] for i in range(4))
        bt = out[4 * B:4 * B + B * mb].reshape(B, mb)
        kvl[:] = 1  # padded rows: 1 scratch token in block 0
        if n:
            p = np.fromiter((s.length - 1 for s in seqs), dtype=np.int32, count=n)
            ids[:n] = np.fromiter((s.token_at(int(q)) for s, q in zip(seqs, p)), dtype=np.int32, count=n)
            bt[:n] = np.stack([self._bt_row(s, int(q) // BLOCK + 1) for s, q in zip(seqs, p)])
            pos[:n] = p
            slots[:n] = bt[np.arange(n), p // BLOCK] * BLOCK + p % BLOCK
            kvl[:n] = p + 1
        return out

    def _decode_graph(self, B):
        if B in self.graphs:
            return self.graphs[B]
        from ..ops.native import decode_partitions

        m = self.model
        dev = self.device
        mb = self.max_blocks
        meta_n = 4 * B + B * mb + (4 * B + B * mb) % 2  # even: the sampling block holds int64 seeds
        # ONE H2D copy per step: [decode metadata | sampling params (6B) | carry map (B)]
        packed = torch.zeros(meta_n + 7 * B, dtype=torch.int32, device=dev)
        ids, pos, slots, kvl = (packed[i * B:(i + 1) * B] for i in range(4))
        carry = packed[meta_n + 6 * B:meta_n + 7 * B]
        bt = packed[4 * B:4 * B + B * mb].view(B, mb)
        pt, mp = decode_partitions(self.max_model_len, B, m.Hkv)
        ws_o = torch.empty((B, m.Hq, mp, m.D), dtype=torch.float32, device=dev) if mp > 1 else None
        ws_ml = torch.empty((B, m.Hq, mp, 2), dtype=torch.float32, device=dev) if mp > 1 else None
        meta = AttnMeta("decode", kvl, bt, part_tiles=pt, max_parts=mp, ws_o=ws_o, ws_ml=ws_ml)
        temps, ks, ps, seeds, steps = self._sampling_views(packed[meta_n:meta_n + 6 * B], B)
        samp = dict(temps=temps, ks=ks, ps=ps, seeds=seeds, steps=steps)
        out_tok = self._tok_out[:B]
        inp = StepInput(ids, pos, slots, meta, None, carry=carry, carry_src=self._tok_out)

        def run():
            logits = m.forward(inp)
            self._sample_rows(logits, samp["temps"], samp["ks"], samp["ps"], samp["seeds"], samp["steps"],
                              out=out_tok)

        entry = dict(packed=packed, samp=samp, out=out_tok, run=run, graph=None, meta=meta, inp=inp)
        if self.use_graphs:
            kvl.fill_(1)  # scratch-only rows while capturing
            carry.fill_(-1)
            # the eager warm-up runs below sample into the shared _tok_out, which may hold the in-flight
            # step's tokens that the next step carries (a graph captured lazily mid-pipeline): restore it
            saved = self._tok_out.clone()
            s = torch.cuda.Stream(device=dev)
            s.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(s):
                for _ in range(2):
                    run()
            torch.cuda.current_stream(dev).wait_stream(s)
            g = torch.cuda.CUDAGraph()
            # captured on the warm-up stream: stream-keyed native state (the persistent decode MLP's
            # arrival counters, ops/native.py _me_workspace) was allocated by the warm-up runs above
            with torch.cuda.graph(g, stream=s):
                run()
            self._tok_out.copy_(saved)
            entry["graph"] = g
        self.graphs[B] = entry
        return entry

    def warmup_graphs(self, sizes=None):
        if not self.is_cuda:  # CPU plumbing: eager decode, nothing to capture
            return
        for b in sizes or self.buckets:
            self._decode_graph(b)
        # tensor parallel: leave warm-up together. A rank still capturing (host-bound, seconds on a loaded
        # host) would otherwise keep the others' first collectives spinning in their bounded peer waits.
        grp = getattr(self.comm, "cpu_group", None)
        if self.tp_size > 1 and grp is not None:
            import torch.distributed as dist

            torch.cuda.synchronize()
            dist.barrier(group=grp)

    # ------------------------------------------------------------------ asynchronous decode
    def _decode_inputs_async(self, seqs, B, carried):
        """As _decode_inputs_host, for a step whose rows with carried[i] feed the previous step's
        in-flight token (position = committed length; id patched on the device)."""
        mb = self.max_blocks
        n = len(seqs)
        out = np.zeros(4 * B + B * mb + (4 * B + B * mb) % 2, dtype=np.int32)
        ids, pos, slots, kvl = (out[i * B:(i + 1) * B] for i in range(4))
        bt = out[4 * B:4 * B + B * mb].reshape(B, mb)
        kvl[:] = 1
        if n:
            c = np.asarray(carried, dtype=np.int32)
            p = np.fromiter((s.length - 1 for s in seqs), dtype=np.int32, count=n) + c
            ids[:n] = np.fromiter((0 if ci else s.token_at(int(q)) for s, q, ci in zip(seqs, p, carried)),
                                  dtype=np.int32, count=n)
            bt[:n] = np.stack([self._bt_row(s, int(q) // BLOCK + 1) for s, q in zip(seqs, p)])
            pos[:n] = p
            slots[:n] = bt[np.arange(n), p // BLOCK] * BLOCK + p % BLOCK
            kvl[:n] = p + 1
        return out

    def _decode_async(self, ready):
        t0 = time.perf_counter()
        prev = self._inflight
        prev_row = {} if prev is None else {id(s): i for i, s in enumerate(prev["seqs"])}
        seqs = []
        for s in ready:
            if id(s) in prev_row:  # its in-flight token will be accepted: does it get another step?
                L = len(s.out) + 1
                if L >= s.params.max_new_tokens or s.length + 1 >= self.max_model_len:
                    continue
            seqs.append(s)
        if not seqs:
            return self._drain()
        n = len(seqs)
        carried = [id(s) in prev_row for s in seqs]
        B = self._bucket(n)
        e = self._decode_graph(B)
        samp = self._sampling_host(seqs, pad_to=B)
        steps = samp[5 * B:5 * B + n]
        steps += np.asarray(carried, dtype=np.int32)  # sampling step index of the token being produced
        # carried rows read their id from the previous step's sampled tokens (the shared device buffer
        # _tok_out, row = that step's row) inside the graph's embedding kernel: no extra copy / gather
        carry = np.full(B, -1, dtype=np.int32)
        carry[:n] = [prev_row[id(s)] if c else -1 for s, c in zip(seqs, carried)]
        host = np.concatenate([self._decode_inputs_async(seqs, B, carried), samp, carry])
        e["packed"].copy_(self._h2d_i32(host), non_blocking=True)
        forced = self._engine_fault_hook()
        if self._timing is not None:
            ea, eb = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ea.record()
            e["graph"].replay()
            eb.record()
            self._timing.append((ea, eb))
        else:
            e["graph"].replay()
        if forced:
            self._engine_fault_hook(release=True)
        self._out_idx ^= 1
        host_out = self._out_pins[self._out_idx]
        host_out[:n].copy_(e["out"][:n], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(self.device))
        for s in seqs:
            s.computed = s.length + (1 if id(s) in prev_row else 0)
        cur = dict(seqs=seqs, out=e["out"], event=ev, host_out=host_out, n=n)
        fin = self._collect(prev, in_flight=set(id(s) for s in seqs))
        if fin is None:  # prev failed in-kernel; cur consumed its tokens on the device
            self._recover_engine_fault([prev, cur])
            self.stats["decode_s"] += time.perf_counter() - t0
            return []
        self._inflight = cur
        self.stats["decode_steps"] += 1
        self._count_batch(n)
        self.stats["decode_s"] += time.perf_counter() - t0
        return fin

    def _count_batch(self, n):
        """Decode steps per batch size (stats["decode_batch_hist"]): how well the schedule keeps the
        weight stream of each decode step amortised over many sequences."""
        h = self.stats.setdefault("decode_batch_hist", {})
        h[n] = h.get(n, 0) + 1

    def _collect(self, step, in_flight=frozenset()):
        """Wait for an in-flight decode step, accept its tokens, free what it no longer touches."""
        if step is None:
            return []
        step["event"].synchronize()
        for sid in self._free_after:  # rows of the step before `step`: done with those blocks now
            self.bm.free(sid)
        self._free_after = []
        if self._kernel_fault():
            return None  # the caller discards this step (and the one in flight behind it)
        tok = step["host_out"][:step["n"]].tolist()
        finished = []
        for s, t in zip(step["seqs"], tok):
            if s.status == FINISHED:  # stopped (or aborted) before this step's token was read
                continue
            r = self._accept(s, t)
            self.stats["decode_tokens"] += 1
            if r:
                self._finish(s, r, defer_free=id(s) in in_flight)
                finished.append(s)
        return finished

    def _kernel_fault(self) -> int:
        """Error code a bounded in-kernel wait reported during the steps synchronised so far (the persistent
        decode MLP's hand-off, ops/native.py mlp_engine_fault): host-mapped words, read after the step's
        event sync at no extra cost. 0 = healthy."""
        if not self.is_cuda:
            return 0
        from ..ops import native
        return native.mlp_engine_fault(self.device)

    def _engine_fault_hook(self, release=False):
        """RAGK_FAULTS=mlp_engine_timeout_at_step=N: the N-th decode step's persistent MLP launches get a
        one-tick deadline (every wait gives up) -- the recovery path's test."""
        from ..ops import native
        if release:
            native.mlp_engine_force_timeout(0, self.device)
            return False
        at = faults.value("mlp_engine_timeout_at_step")
        if at is None or not self.is_cuda or faults.tick("mlp_engine_timeout_at_step") != int(at):
            return False
        native.mlp_engine_force_timeout(1, self.device)
        return True

    def _recover_engine_fault(self, steps):
        """A persistent decode MLP launch gave up a wait: its step's rows (and those of the step in flight
        behind it, which consumed its tokens) are garbage and are NOT accepted. Wait for the device, re-arm
        the counters, turn the engine off for this process (its graphs are recaptured on the separate
        kernels on demand) and rewind every affected sequence to its last accepted token, so the next decode
        step recomputes those rows; the KV rows they wrote are rewritten by the recomputation."""
        code = self._kernel_fault()
        if self.is_cuda:
            from ..ops import native
            torch.cuda.synchronize(self.device)
            native.mlp_engine_rearm(self.device)
            native.MLP_ENGINE = False
        self.graphs.clear()
        self._inflight = None
        for sid in self._free_after:
            self.bm.free(sid)
        self._free_after = []
        n = 0
        for step in steps:
            if step is None:
                continue
            for s in step["seqs"]:
                if s.status != FINISHED:
                    s.computed = s.length - 1
                    n += 1
        self.stats["engine_faults"] = self.stats.get("engine_faults", 0) + 1
        log.error("persistent decode MLP: a wait gave up (code %d); %d rows of the last decode steps discarded "
                  "and recomputed on the separate kernels (engine off for this process)", code, n)

    def _drain(self):
        """Complete the in-flight decode step (before a prefill, an abort, or when nothing is left)."""
        if self._inflight is None:
            return []
        t0 = time.perf_counter()
        step, self._inflight = self._inflight, None
        fin = self._collect(step)
        if fin is None:
            self._recover_engine_fault([step])
            self.stats["decode_s"] += time.perf_counter() - t0
            return []
        for sid in self._free_after:
            self.bm.free(sid)
        self._free_after = []
        self.stats["decode_s"] += time.perf_counter() - t0
        return fin

    def _decode(self, seqs, full_vocab=False):
        t0 = time.perf_counter()
        n = len(seqs)
        finished = []
        if not seqs:
            return finished
        if self.is_cuda:
            B = self._bucket(n)
            e = self._decode_graph(B)
            host = np.concatenate([self._decode_inputs_host(seqs, B), self._sampling_host(seqs, pad_to=B),
                                   np.full(B, -1, dtype=np.int32)])
            e["packed"].copy_(self._h2d_i32(host), non_blocking=True)
            if full_vocab:  # eager forward, exact sampler over the whole vocabulary
                tok = self._sample_full_vocab(self.model.forward(e["inp"])[:n], seqs)
            else:
                forced = self._engine_fault_hook()
                if e["graph"] is not None:
                    e["graph"].replay()
                else:
                    e["run"]()
                if forced:
                    self._engine_fault_hook(release=True)
                tok = e["out"][:n].cpu().tolist()
            if self._kernel_fault():  # synchronised by the token read-back above
                self._recover_engine_fault([dict(seqs=seqs)])
                self.stats["decode_s"] += time.perf_counter() - t0
                return finished
        else:
            host = self._decode_inputs_host(seqs, n)
            mb = self.max_blocks
            t = torch.from_numpy(host)
            kvl = t[3 * n:4 * n]
            meta = AttnMeta("decode", kvl, t[4 * n:4 * n + n * mb].view(n, mb), host_kv_lens=kvl.tolist())
            inp = StepInput(t[:n], t[n:2 * n], t[2 * n:3 * n], meta, None)
            logits = self.model.forward(inp)
            if full_vocab:
                tok = self._sample_full_vocab(logits, seqs)
            else:
                tok = self._sample_rows(logits, *self._sampling_tensors(seqs)).tolist()
            if self._kernel_fault():
                self._recover_engine_fault([dict(seqs=seqs)])
                self.stats["decode_s"] += time.perf_counter() - t0
                return finished
        for s in seqs:
            s.computed = s.length
        for s, t in zip(seqs, tok):
            r = self._accept(s, t)
            if r:
                self._finish(s, r)
                finished.append(s)
        self.stats["decode_steps"] += 1
        self._count_batch(n)
        self.stats["decode_tokens"] += n
        self.stats["decode_s"] += time.perf_counter() - t0
        return finished
