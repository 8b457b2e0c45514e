"""faiss-compatible index files (D4's read_index / write_index) and the metadata pickle (D12).

IndexFlatL2 ("IxF2"), [ext] faiss impl/index_write.cpp:
  u32 fourcc 'IxF2' | i32 d | i64 ntotal | i64 dummy(1<<20) | i64 dummy(1<<20) |
  u8 is_trained | i32 metric_type (1 = L2) | u64 n_floats | f32[n_floats] row-major
IndexIVFFlat ("IwFl"): index header | u64 nlist | u64 nprobe | quantizer (IxF2) |
  direct map (u8 type, u64 n, i64[n]) | inverted lists 'ilar' (u64 nlist, u64 code_size,
  'full' + u64 n + u64 sizes[nlist]  or  'sprs' + u64 n + (list, size) pairs, then per
  non-empty list: codes (size*code_size bytes) + ids (i64[size])).
faiss is not installed on this box: the layout is pinned by golden-byte tests built from
this spec; byte-level parity with a real faiss build is "parity unpinned".

Metadata: the reference pickles a list of {'filename','chunk_id','text'} dicts
(/root/reference/llm/rag.py:63-64,83-84). We write the same protocol-4 pickle, and read
with a restricted Unpickler that only materialises builtin containers/scalars, so a
tampered file cannot execute code.
"""
from __future__ import annotations

import io
import os
import pickle
import struct
import tempfile

import numpy as np

METRIC_INNER_PRODUCT, METRIC_L2 = 0, 1


def _hdr(f, d, ntotal, metric=METRIC_L2, is_trained=True):
    f.write(struct.pack("<iqqqBi", d, ntotal, 1 << 20, 1 << 20, 1 if is_trained else 0, metric))


def write_flat_l2(f, xb: np.ndarray):
    xb = np.ascontiguousarray(xb, dtype=np.float32)
    n, d = xb.shape
    f.write(b"IxF2")
    _hdr(f, d, n)
    f.write(struct.pack("<Q", n * d))
    f.write(xb.tobytes())


def _read_exact(f, n):
    b = f.read(n)
    if len(b) != n:
        raise ValueError("truncated faiss index file")
    return b


def _read_hdr(f):
    d, ntotal, _, _, is_trained, metric = struct.unpack("<iqqqBi", _read_exact(f, 4 + 8 * 3 + 1 + 4))
    if metric > 1:
        _read_exact(f, 4)  # metric_arg
    return d, ntotal, bool(is_trained), metric


def read_index_stream(f):
    h = _read_exact(f, 4)
    if h in (b"IxF2", b"IxFI", b"IxFl"):
        d, n, _, metric = _read_hdr(f)
        (nf,) = struct.unpack("<Q", _read_exact(f, 8))
        if nf != n * d:
            raise ValueError("corrupt IndexFlat: %d floats for ntotal=%d d=%d" % (nf, n, d))
        xb = np.frombuffer(_read_exact(f, nf * 4), dtype=np.float32).reshape(n, d).copy()
        return {"type": "flat", "d": d, "ntotal": n, "metric": metric, "xb": xb}
    if h == b"IwFl":
        d, n, _, metric = _read_hdr(f)
        nlist, nprobe = struct.unpack("<QQ", _read_exact(f, 16))
        quant = read_index_stream(f)
        (dm_type,) = struct.unpack("<B", _read_exact(f, 1))
        (dm_n,) = struct.unpack("<Q", _read_exact(f, 8))
        _read_exact(f, 8 * dm_n)
        if dm_type == 2:  # hashtable direct map
            (hn,) = struct.unpack("<Q", _read_exact(f, 8))
            _read_exact(f, 16 * hn)
        if _read_exact(f, 4) != b"ilar":
            raise ValueError("unsupported inverted-list type")
        il_n, code_size = struct.unpack("<QQ", _read_exact(f, 16))
        kind = _read_exact(f, 4)
        (vn,) = struct.unpack("<Q", _read_exact(f, 8))
        v = np.frombuffer(_read_exact(f, 8 * vn), dtype=np.uint64)
        sizes = np.zeros(il_n, dtype=np.int64)
        if kind == b"full":
            sizes[:] = v
        else:
            for i in range(0, len(v), 2):
                sizes[int(v[i])] = int(v[i + 1])
        codes, ids = [], []
        for li in range(il_n):
            s = int(sizes[li])
            if s:
                codes.append(np.frombuffer(_read_exact(f, s * code_size), dtype=np.float32).reshape(s, d))
                ids.append(np.frombuffer(_read_exact(f, 8 * s), dtype=np.int64))
            else:
                codes.append(np.zeros((0, d), np.float32))
                ids.append(np.zeros(0, np.int64))
        return {"type": "ivf_flat", "d": d, "ntotal": n, "metric": metric, "nlist": nlist, "nprobe": nprobe,
                "centroids": quant["xb"], "lists": codes, "ids": ids}
    raise ValueError("unsupported faiss index fourcc %r" % h)


def write_ivf_flat(f, d, centroids, lists, ids, nprobe=1):
    nlist = len(lists)
    n = int(sum(len(x) for x in ids))
    f.write(b"IwFl")
    _hdr(f, d, n)
    f.write(struct.pack("<QQ", nlist, nprobe))
    write_flat_l2(f, centroids)
    f.write(struct.pack("<BQ", 0, 0))  # no direct map
    f.write(b"ilar")
    f.write(struct.pack("<QQ", nlist, d * 4))
    sizes = [len(x) for x in ids]
    n_non0 = sum(1 for s in sizes if s)
    if n_non0 > nlist // 2:
        f.write(b"full")
        f.write(struct.pack("<Q", nlist))
        f.write(np.asarray(sizes, dtype=np.uint64).tobytes())
    else:
        f.write(b"sprs")
        pairs = [v for i, s in enumerate(sizes) if s for v in (i, s)]
        f.write(struct.pack("<Q", len(pairs)))
        f.write(np.asarray(pairs, dtype=np.uint64).tobytes())
    for c, i in zip(lists, ids):
        if len(i):
            f.write(np.ascontiguousarray(c, dtype=np.float32).tobytes())
            f.write(np.ascontiguousarray(i, dtype=np.int64).tobytes())


def read_index(path):
    with open(path, "rb") as f:
        return read_index_stream(f)


def atomic_write(path, writer):
    """Write via a temp file in the same directory + os.replace (readers never see a torn file)."""
    d = os.path.dirname(os.path.abspath(path)) or "."
    os.makedirs(d, exist_ok=True)
    fd, tmp = tempfile.mkstemp(prefix=".tmp-", dir=d)
    try:
        with os.fdopen(fd, "wb") as f:
            writer(f)
            f.flush()
            os.fsync(f.fileno())
        os.replace(tmp, path)
    except BaseException:
        try:
            os.unlink(tmp)
        except OSError:
            pass
        raise


# ---------------------------------------------------------------------------- metadata
class _SafeUnpickler(pickle.Unpickler):
    _ALLOWED = {("builtins", n) for n in ("dict", "list", "tuple", "set", "frozenset", "str", "int", "float",
                                          "bool", "bytes", "NoneType")}

    def find_class(self, module, name):
        if (module, name) in self._ALLOWED:
            import builtins

            return getattr(builtins, name)
        raise pickle.UnpicklingError("metadata pickle references forbidden global %s.%s" % (module, name))


def load_metadata(path):
    with open(path, "rb") as f:
        obj = _SafeUnpickler(io.BytesIO(f.read())).load()
    if not isinstance(obj, list):
        raise ValueError("metadata pickle must hold a list")
    return obj


def save_metadata(path, metadata):
    atomic_write(path, lambda f: pickle.dump(list(metadata), f, protocol=4))
