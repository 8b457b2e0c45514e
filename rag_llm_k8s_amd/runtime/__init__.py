"""Host runtime: safetensors I/O, tokenizers, faiss-format index I/O, native C++ helpers."""
from __future__ import annotations

import importlib.util
import os

_rt = None
_tried = False


def native_rt():
    """The pybind11 C++ runtime module (``_lib/_ragk_rt*.so``) or None if not built."""
    global _rt, _tried
    if _tried:
        return _rt
    _tried = True
    from .._build import runtime_ext_path

    p = runtime_ext_path()
    if os.path.exists(p):
        spec = importlib.util.spec_from_file_location("_ragk_rt", p)
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        check_rt_stamp(mod, p)
        _rt = mod
    return _rt


class StaleRuntimeError(RuntimeError):
    pass


def check_rt_stamp(mod, path="_ragk_rt"):
    """The runtime must have been built from csrc/runtime in this tree (content hash compiled in by
    _build.build_runtime). RAGK_ALLOW_STALE_LIB=1 skips the check."""
    from .. import _build

    if os.environ.get("RAGK_ALLOW_STALE_LIB") == "1" or not _build.runtime_sources()[0]:
        return
    got = mod.build_stamp() if hasattr(mod, "build_stamp") else None
    want = _build.runtime_source_hash()
    if got != want:
        raise StaleRuntimeError("%s was built from other runtime sources (stamp %s, tree %s): rebuild it "
                                "(python -m rag_llm_k8s_amd._build)" % (path, got, want))
