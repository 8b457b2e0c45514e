"""Document store = vector index + chunk metadata, with the reference's on-disk layout.

Reference behaviour and its fixes:
  ensure_index_exists / update_index / search_documents   /root/reference/llm/rag.py:57-86,114-120
  * index + metadata re-read from disk on every request    -> kept resident (HBM), reloaded
    only if the files on disk change (mtime check);
  * unlocked read-modify-write of both files               -> single writer lock + atomic
    os.replace snapshots, so readers never see torn files; an /upload_pdf append returns as soon
    as the vectors are in HBM and the snapshot is written by a background thread (the state is
    copied under the lock, the file I/O runs outside it; bursts of appends coalesce into one
    write), so a 1M x 1024 index (4 GB) is not rewritten on the request path;
  * faiss label -1 mapped to metadata[-1] (last chunk)     -> -1 results are dropped, making the
    "No relevant information found" branch reachable;
  * startup re-ingest duplicates chunks                    -> idempotent by (filename, chunk_id)
    unless reingest_append=True (legacy behaviour).
"""
from __future__ import annotations

import logging
import os
import threading
import time

import numpy as np

from ..utils import faults
from .faiss_io import load_metadata, read_index, save_metadata
from .flat import FlatL2Index

log = logging.getLogger(__name__)


class DocumentStore:
    def __init__(self, index_path, dim, device="cpu", index_type="flat", ivf_nlist=1024, ivf_nprobe=32,
                 recovery="rebuild", shard=None):
        """shard = (group, rank, world): INDEX_SHARDED tensor-parallel mode -- this rank keeps the rows
        g % world == rank of the index (parallel/dp.py ShardedFlatIndex) in `<index_path>.shard<r>of<W>`
        (a faiss IxF2 file of its rows); every rank keeps the full metadata list, rank 0 persists it.
        search() is then a collective (all ranks call it together, followers with no queries)."""
        self.sharded = shard is not None
        self.shard = shard
        self.index_path = index_path
        self.index_file = index_path if shard is None else "%s.shard%dof%d" % (index_path, shard[1], shard[2])
        self.persist_meta = shard is None or shard[1] == 0
        self.recovery = recovery  # rebuild: quarantine an unreadable index and start empty | fail
        self.meta_path = index_path + ".metadata"
        self.dim = dim
        self.device = device
        self.index_type = index_type
        self.ivf_nlist, self.ivf_nprobe = ivf_nlist, ivf_nprobe
        self.index = self._new_index()
        self.metadata = []
        self._keys = set()
        self._wlock = threading.RLock()
        self._mtimes = None
        self.recovered = None
        self._dirty = False
        self._writing = 0  # snapshot writes in flight (their file replacements are not "other writers")
        self._persister = None
        self._persist_error = None

    def _new_index(self):
        if self.sharded:
            if self.index_type != "flat":
                raise ValueError("INDEX_SHARDED supports the flat index only")
            from ..parallel.dp import ShardedFlatIndex

            return ShardedFlatIndex(self.dim, device=self.device, group=self.shard[0])
        if self.index_type == "ivf":
            from .ivf import IVFFlatIndex

            return IVFFlatIndex(self.dim, device=self.device, nlist=self.ivf_nlist, nprobe=self.ivf_nprobe)
        return FlatL2Index(self.dim, device=self.device)

    # ------------------------------------------------------------------ lifecycle
    def ensure_exists(self):
        """Reference ensure_index_exists(): create an empty index + [] metadata if missing."""
        if not os.path.exists(self.index_file):
            log.info("Faiss index not found. Creating a new one.")
            self.persist()
        else:
            log.info("Faiss index found.")
            try:
                self.load()
            except Exception as e:
                if self.recovery != "rebuild":
                    raise
                self._quarantine(e)
                self.persist()
        return self

    def _quarantine(self, err):
        """Move an unreadable index (+ metadata) aside and start empty; the startup directory
        ingest then rebuilds it from PDF_DIR. The reference would crash-loop instead."""
        tag = ".corrupt-%d" % int(time.time())
        for p in (self.index_file, self.meta_path) if self.persist_meta else (self.index_file,):
            if os.path.exists(p):
                os.replace(p, p + tag)
        log.error("index %s unreadable (%s); moved aside as *%s, starting empty", self.index_file, err, tag)
        self.index = self._new_index()
        self.metadata = []
        self._keys = set()
        self.recovered = tag

    def _disk_mtimes(self):
        try:
            return (os.path.getmtime(self.index_file), os.path.getmtime(self.meta_path))
        except OSError:
            return None

    def load(self):
        faults.check("index_read_error", self.index_file)
        r = read_index(self.index_file)
        meta = load_metadata(self.meta_path) if os.path.exists(self.meta_path) else []
        if r["d"] != self.dim:
            raise ValueError("index dimension %d != embedder dimension %d" % (r["d"], self.dim))
        idx = self._new_index()
        if self.sharded:  # this rank's rows only; the global count comes from the metadata
            world, rank = self.shard[2], self.shard[1]
            if r["ntotal"] != len(range(rank, len(meta), world)):
                raise ValueError("shard has %d vectors, metadata implies %d" % (r["ntotal"], len(range(rank, len(meta), world))))
            idx.load_local(r["xb"] if r["ntotal"] else None, len(meta))
            self.index, self.metadata = idx, list(meta)
            self._keys = {(m.get("filename"), m.get("chunk_id")) for m in self.metadata if isinstance(m, dict)}
            self._mtimes = self._disk_mtimes()
            return
        if len(meta) != r["ntotal"]:
            raise ValueError("index has %d vectors but metadata %d entries (torn write?)" % (r["ntotal"], len(meta)))
        if r["type"] == "flat":
            if r["ntotal"]:
                if self.index_type == "ivf":
                    idx.train(r["xb"])
                idx.add(r["xb"])
        else:
            from .ivf import IVFFlatIndex

            idx = IVFFlatIndex.from_lists(r, device=self.device)
        self.index = idx
        self.metadata = list(meta)
        self._keys = {(m.get("filename"), m.get("chunk_id")) for m in self.metadata if isinstance(m, dict)}
        self._mtimes = self._disk_mtimes()

    def maybe_reload(self):
        """Pick up index files replaced on disk by another writer (e.g. an offline ingest job)."""
        if self.sharded:  # a reload would have to be collective; shards change only through ingest jobs
            return
        m = self._disk_mtimes()
        if m is None or self._mtimes is None or m == self._mtimes:
            return
        with self._wlock:
            # Our own snapshot writer replaces the files outside the lock: while it runs (or while
            # appends are waiting for it) the disk lags HBM, and reloading would drop those appends.
            if self._writing or self._dirty:
                return
            m = self._disk_mtimes()  # re-check under the lock: a write may have finished meanwhile
            if m is None or m == self._mtimes:
                return
            try:
                self.load()
            except Exception as e:  # keep serving the resident snapshot; retry on the next change
                log.warning("index on disk changed but is unreadable (%s); keeping the resident copy", e)
                self._mtimes = m

    def _snapshot(self):
        """(index writer, metadata copy) of the current state; caller holds _wlock."""
        return self.index.snapshot_writer(), list(self.metadata)

    def _write(self, writer, meta):
        """Write a snapshot. The caller registered it in _writing under _wlock; the mtimes the store
        itself produced are recorded under the lock, so maybe_reload never mistakes them for another
        writer's files."""
        try:
            writer(self.index_file)
            if self.persist_meta:
                save_metadata(self.meta_path, meta)
        finally:
            with self._wlock:
                self._mtimes = self._disk_mtimes()
                self._writing -= 1

    def persist(self):
        """Synchronous snapshot (startup / directory ingest / shutdown)."""
        with self._wlock:
            writer, meta = self._snapshot()
            self._dirty = False
            self._writing += 1
            self._write(writer, meta)

    def persist_async(self):
        """Schedule a background snapshot; appends made meanwhile are folded into the same write."""
        with self._wlock:
            self._dirty = True
            if self._persister is None:  # cleared under the lock by the writer when it exits
                self._persister = threading.Thread(target=self._persist_loop, name="index-snapshot", daemon=True)
                self._persister.start()

    def _persist_loop(self):
        clean = False
        try:
            while True:
                with self._wlock:
                    if not self._dirty:
                        # deregister while still holding the lock: an add() after this point sees
                        # _persister None and starts a new writer (no lost wake-up)
                        self._persister = None
                        clean = True
                        return
                    # host copy under the lock (consistent vectors + metadata); a failure here (e.g. the
                    # device copy after a GPU fault) leaves _dirty set, so the next append retries
                    writer, meta = self._snapshot()
                    self._dirty = False
                    self._writing += 1
                try:
                    self._write(writer, meta)  # file I/O outside the lock: searches and appends continue
                except Exception as e:  # keep serving from HBM; the next append retries the snapshot
                    self._persist_error = e
                    log.error("index snapshot failed: %s", e)
        except Exception as e:
            self._persist_error = e
            log.error("index snapshot thread failed: %s", e)
        finally:
            if not clean:  # any abnormal exit deregisters too: the next persist_async starts a new writer
                with self._wlock:
                    if self._persister is threading.current_thread():
                        self._persister = None

    def flush(self):
        """Wait until every scheduled snapshot is on disk."""
        t = self._persister
        if t is not None:
            t.join()
        with self._wlock:
            if self._dirty:
                writer, meta = self._snapshot()
                self._dirty = False
                self._writing += 1
                self._write(writer, meta)

    # ------------------------------------------------------------------ writes
    def add(self, vectors, metadata, dedupe=True, persist=True):
        """Append vectors + metadata (reference update_index). Returns number added."""
        vecs = np.asarray(vectors.cpu() if hasattr(vectors, "cpu") else vectors, dtype=np.float32)
        if vecs.ndim == 1:
            vecs = vecs.reshape(1, -1)
        with self._wlock:
            keep = list(range(len(metadata)))
            if dedupe:
                keep = [i for i, m in enumerate(metadata) if (m["filename"], m["chunk_id"]) not in self._keys]
            if keep:
                if self.index_type == "ivf" and not self.index.is_trained:
                    self.index.train(vecs[keep])
                self.index.add(vecs[keep])
                for i in keep:
                    self.metadata.append(metadata[i])
                    self._keys.add((metadata[i]["filename"], metadata[i]["chunk_id"]))
                if persist:
                    self.persist_async()
            log.info("Index updated. Total vectors: %d, Dimension: %d", self.index.ntotal, self.dim)
            return len(keep)

    # ------------------------------------------------------------------ reads
    def search(self, qvecs, k):
        """Batched search -> list (per query) of [(metadata, squared_l2)] ascending, -1 dropped."""
        with self._wlock:  # consistent (index, metadata) pair: an append cannot land in between
            D, I = self.index.search(qvecs, k)
            meta = self.metadata
            n = len(meta)
        out = []
        for drow, irow in zip(D.tolist(), I.tolist()):
            res = []
            for d, i in zip(drow, irow):
                if 0 <= i < n:
                    res.append((meta[i], float(d)))
            out.append(res)
        return out

    def info(self):
        return {"total_vectors": int(self.index.ntotal), "dimension": int(self.dim),
                "total_chunks": len(self.metadata), "sample_chunks": self.metadata[:5] if self.metadata else []}
