"""Build reuse is checked, not assumed: the kernel library carries the content hash of the kernel
sources it was built from, and the loader refuses a library that does not match the tree."""
import ctypes
import os

import pytest

from rag_llm_k8s_amd import _build
from rag_llm_k8s_amd.ops import _lib


def test_source_hash_is_content_based(tmp_path, monkeypatch):
    h = _build.source_hash()
    assert len(h) == 32 and h == _build.source_hash()
    srcs, _ = _build.hip_sources()
    assert any(s.endswith("search.hip") for s in srcs)
    monkeypatch.setattr(_build, "EXTRA_FLAGS", dict(_build.EXTRA_FLAGS, **{"x.hip": ["-DX"]}))
    assert _build.source_hash() != h  # flags are part of the stamp


@pytest.mark.skipif(not _lib.available(), reason="kernel library not built")
def test_library_stamp_matches_tree_and_stale_is_refused(monkeypatch):
    h = ctypes.CDLL(_lib.LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    _lib._check_stamp(h)  # the in-tree library was built from these sources
    monkeypatch.setattr(_build, "source_hash", lambda: "0" * 32)
    monkeypatch.delenv("RAGK_ALLOW_STALE_LIB", raising=False)
    with pytest.raises(_lib.NativeLibraryError, match="other kernel sources"):
        _lib._check_stamp(h)
    monkeypatch.setenv("RAGK_ALLOW_STALE_LIB", "1")
    _lib._check_stamp(h)
    assert os.path.exists(os.path.join(_build.OBJ_DIR, "ragk_stamp.txt"))


def test_runtime_hash_is_content_based(monkeypatch):
    h = _build.runtime_source_hash()
    assert len(h) == 32 and h == _build.runtime_source_hash()
    monkeypatch.setattr(_build, "RT_FLAGS", _build.RT_FLAGS + ["-DX"])
    assert _build.runtime_source_hash() != h


@pytest.mark.skipif(not os.path.exists(_build.runtime_ext_path()), reason="runtime not built")
def test_runtime_stamp_matches_tree_and_stale_is_refused(monkeypatch):
    from rag_llm_k8s_amd import runtime

    mod = runtime.native_rt()
    assert mod is not None and mod.build_stamp() == _build.runtime_source_hash()
    monkeypatch.delenv("RAGK_ALLOW_STALE_LIB", raising=False)
    monkeypatch.setattr(_build, "runtime_source_hash", lambda: "0" * 32)
    with pytest.raises(runtime.StaleRuntimeError, match="other runtime sources"):
        runtime.check_rt_stamp(mod)
    monkeypatch.setenv("RAGK_ALLOW_STALE_LIB", "1")
    runtime.check_rt_stamp(mod)
