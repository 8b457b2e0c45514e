"""Zero-copy safetensors reading (mmap) with TP-shard slicing, and a writer.

Replaces the reference's Rust `safetensors` dependency (D6) used by
AutoModelForCausalLM.from_pretrained (/root/reference/llm/rag.py:24). Prefers the native
C++ mmap reader from ``_ragk_rt`` when built; the pure-Python path parses the same
8-byte-length + JSON header + raw little-endian data layout.

Only the requested slice of a tensor is touched, so each TP rank reads just its shard
of the checkpoint from the PVC.
"""
from __future__ import annotations

import json
import mmap
import os
import struct
import warnings

import numpy as np
import torch

_DT = {
    "BF16": (np.uint16, torch.bfloat16, 2), "F16": (np.float16, torch.float16, 2),
    "F32": (np.float32, torch.float32, 4), "I64": (np.int64, torch.int64, 8), "I32": (np.int32, torch.int32, 4),
    "U8": (np.uint8, torch.uint8, 1), "I8": (np.int8, torch.int8, 1), "F64": (np.float64, torch.float64, 8),
    "F8_E4M3": (np.uint8, torch.float8_e4m3fn, 1), "BOOL": (np.bool_, torch.bool, 1),
}
_REV = {torch.bfloat16: "BF16", torch.float16: "F16", torch.float32: "F32", torch.int64: "I64",
        torch.int32: "I32", torch.uint8: "U8", torch.int8: "I8", torch.float64: "F64",
        torch.float8_e4m3fn: "F8_E4M3", torch.bool: "BOOL"}


class SafeFile:
    def __init__(self, path):
        self.path = path
        self._native = None
        try:
            from . import native_rt

            rt = native_rt()
            if rt is not None:
                self._native = rt.SafeTensors(path)
        except Exception:
            self._native = None
        self._f = open(path, "rb")
        self._mm = mmap.mmap(self._f.fileno(), 0, access=mmap.ACCESS_READ)
        (n,) = struct.unpack("<Q", self._mm[:8])
        self.header = json.loads(self._mm[8:8 + n].decode("utf-8"))
        self.metadata = self.header.pop("__metadata__", {}) or {}
        self.base = 8 + n

    def keys(self):
        return list(self.header.keys())

    def info(self, name):
        h = self.header[name]
        return h["dtype"], tuple(h["shape"]), h["data_offsets"]

    def get(self, name, rows=None, cols=None) -> torch.Tensor:
        """Tensor (CPU, zero-copy view of the mmap when unsliced). rows/cols: (start, stop)
        slices of the first / second dimension for TP sharding."""
        dt, shape, (a, b) = self.info(name)
        npdt, tdt, _ = _DT[dt]
        if self._native is not None and (rows is not None or cols is not None):
            # C++ row/col slice copy (GIL released): each TP rank touches only its shard's bytes
            r0, r1 = rows if rows is not None else (-1, -1)
            c0, c1 = cols if cols is not None else (-1, -1)
            t = torch.from_numpy(self._native.slice(name, r0, r1, c0, c1))
            if tdt in (torch.bfloat16, torch.float8_e4m3fn):
                t = t.view(tdt)
            return t
        arr = np.frombuffer(self._mm, dtype=npdt, count=(b - a) // np.dtype(npdt).itemsize, offset=self.base + a)
        arr = arr.reshape(shape) if shape else arr.reshape(())
        if rows is not None:
            arr = arr[rows[0]:rows[1]]
        if cols is not None:
            arr = arr[:, cols[0]:cols[1]]
        if rows or cols:
            t = torch.from_numpy(np.ascontiguousarray(arr))
        else:
            with warnings.catch_warnings():  # read-only mmap view; consumers copy to the device
                warnings.simplefilter("ignore", UserWarning)
                t = torch.from_numpy(arr)
        if tdt in (torch.bfloat16, torch.float8_e4m3fn):
            t = t.view(tdt)
        return t

    def close(self):
        try:
            self._mm.close()
            self._f.close()
        except Exception:
            pass


class CheckpointReader:
    """HF checkpoint directory: model.safetensors or sharded with model.safetensors.index.json."""

    def __init__(self, path):
        self.path = path
        idx = os.path.join(path, "model.safetensors.index.json")
        self.files = {}
        self.where = {}
        if os.path.exists(idx):
            with open(idx) as f:
                wm = json.load(f)["weight_map"]
            for name, fn in wm.items():
                self.where[name] = fn
            # fail fast, naming every absent shard (the reference's downloader swallowed errors,
            # /root/reference/llm/download_model.py:32-33, and the load failed later, opaquely)
            shards = sorted(set(wm.values()))
            from ..utils import faults

            drop = faults.value("missing_shard")
            missing = [fn for i, fn in enumerate(shards)
                       if not os.path.exists(os.path.join(path, fn)) or (drop is not None and int(drop) == i + 1)]
            if missing:
                raise FileNotFoundError("checkpoint %s is incomplete: missing shard(s) %s of %d listed in "
                                        "model.safetensors.index.json (re-run llm/download_model.py)"
                                        % (path, ", ".join(missing), len(shards)))
        else:
            single = os.path.join(path, "model.safetensors")
            if not os.path.exists(single):
                cands = sorted(x for x in os.listdir(path) if x.endswith(".safetensors"))
                if not cands:
                    raise FileNotFoundError("no safetensors checkpoint in %s" % path)
                single = os.path.join(path, cands[0])
            sf = SafeFile(single)
            self.files[os.path.basename(single)] = sf
            for k in sf.keys():
                self.where[k] = os.path.basename(single)

    def _file(self, fn):
        if fn not in self.files:
            self.files[fn] = SafeFile(os.path.join(self.path, fn))
        return self.files[fn]

    def has(self, name):
        return name in self.where

    def keys(self):
        return list(self.where.keys())

    def get(self, name, rows=None, cols=None):
        return self._file(self.where[name]).get(name, rows=rows, cols=cols)

    def shape(self, name):
        return self._file(self.where[name]).info(name)[1]

    def close(self):
        for f in self.files.values():
            f.close()


def save_file(tensors: dict, path: str, metadata=None):
    header = {}
    off = 0
    blobs = []
    for k, t in tensors.items():
        t = t.detach().contiguous().cpu()
        raw = t.view(torch.uint16).numpy().tobytes() if t.dtype == torch.bfloat16 else (
            t.view(torch.uint8).numpy().tobytes() if t.dtype == torch.float8_e4m3fn else t.numpy().tobytes())
        header[k] = {"dtype": _REV[t.dtype], "shape": list(t.shape), "data_offsets": [off, off + len(raw)]}
        blobs.append(raw)
        off += len(raw)
    if metadata:
        header["__metadata__"] = metadata
    hb = json.dumps(header, separators=(",", ":")).encode()
    hb += b" " * ((8 - len(hb) % 8) % 8)
    with open(path, "wb") as f:
        f.write(struct.pack("<Q", len(hb)))
        f.write(hb)
        for b in blobs:
            f.write(b)


def save_sharded(tensors: dict, directory: str, n_shards: int, prefix="model"):
    """HF sharded layout: model-0000i-of-0000N.safetensors + model.safetensors.index.json."""
    os.makedirs(directory, exist_ok=True)
    names = list(tensors.keys())
    per = -(-len(names) // n_shards)
    weight_map = {}
    total = 0
    for i in range(n_shards):
        part = names[i * per:(i + 1) * per]
        fn = "%s-%05d-of-%05d.safetensors" % (prefix, i + 1, n_shards)
        save_file({k: tensors[k] for k in part}, os.path.join(directory, fn), metadata={"format": "pt"})
        for k in part:
            weight_map[k] = fn
            total += tensors[k].numel() * tensors[k].element_size()
    with open(os.path.join(directory, "%s.safetensors.index.json" % prefix), "w") as f:
        json.dump({"metadata": {"total_size": total}, "weight_map": weight_map}, f, indent=2)
