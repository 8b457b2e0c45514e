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
        _rt = mod
    return _rt
