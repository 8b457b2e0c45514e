"""ctypes binding of the gfx950 kernel library (``_lib/libragk_hip.so``).

Dispatch policy of the whole ``ops`` package: tensors on a GPU go to the native HIP
kernels -- if the library is missing or fails to load on a GPU box, we raise
(no silent eager fallback); tensors on the CPU go to the pure-torch reference
implementations in :mod:`rag_llm_k8s_amd.ops.reference` (the CPU plumbing
configuration of BASELINE.json config 1).
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(os.path.dirname(_HERE), "_lib", "libragk_hip.so")

P, I, F, S, U64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_float, ctypes.c_void_p, ctypes.c_uint64

_SIGS = {
    "ragk_gemm": [P, I, P, I, P, I, P, P, I, I, I, I, I, I, S],
    "ragk_gemm_path": [I, P, I, P, I, P, I, P, P, I, I, I, I, I, S],
    "ragk_gemm_pp": [P, I, P, I, P, I, P, P, I, I, I, I, I, I, S],
    "ragk_gemm_w4_set_grid": [I],
    "ragk_gemm_stream_set_nt": [I],
    "ragk_gemm_stream_set_diag": [I],
    "ragk_gemm_stream_set_pair_rows": [I],
    "ragk_gemm_w4": [P, I, P, I, P, I, P, P, I, I, I, I, I, I, S],
    "ragk_gemm_w4_rope_kv": [P, I, P, I, P, I, I, I, P, P, P, P, P, P, I, I, I, S],
    "ragk_gemm_w4_splitk": [P, I, P, I, P, I, I, I, I, S],
    "ragk_gemm_part": [P, I, P, I, P, I, I, I, I, S],
    "ragk_gemm_part_norm": [P, I, P, F, P, I, P, I, I, I, I, S],
    "ragk_gemm_part_fp8": [P, I, P, I, P, P, I, I, I, I, S],
    "ragk_attn_decode_set_nt": [I],
    "ragk_attn_decode_set_nw8": [I],
    "ragk_attn_decode_set_defer": [I],
    "ragk_attn_decode_set_diag": [I],
    "ragk_attn_decode_set_kl": [I],
    "ragk_gemm_part_merge": [P, P, P, I, P, I, I, I, P, I, P, P, I, I, I, I, S],
    "ragk_gemm_part_merge_ok": [I, I, I, I, I],
    "ragk_gemm_stream_part": [P, I, P, I, P, I, I, I, I, I, S],
    "ragk_gemm_part_silu": [P, I, P, I, P, I, I, I, I, S],
    "ragk_gemm_part_silu_ok": [I, I, I, I],
    "ragk_mlp_engine_ok": [I, I, I, I],
    "ragk_mlp_engine_set_nt": [I],
    "ragk_mlp_engine_set_stamps": [P],
    "ragk_mlp_engine_set_xcd_weights": [I, I],
    "ragk_mlp_engine": [P, P, I, P, F, P, P, P, P, P, P, P, P, I, I, I, I, S],
    "ragk_host_word_alloc": [],
    "ragk_host_word_dev": [P],
    "ragk_host_word_free": [P],
    "ragk_mlp_engine_ctr_bytes": [],
    "ragk_mlp_engine_split": [I, I, I, I, P],
    "ragk_gemm_part_ksteps": [I, I, I],
    "ragk_gemm_part_set_min_blocks": [I],
    "ragk_add_partials_rmsnorm": [P, I, I, P, I, P, P, I, I, F, S],
    "ragk_rope_kv_partials": [P, I, I, I, P, I, P, P, P, P, P, P, I, I, I, I, S],
    "ragk_gemm_dec": [P, I, P, I, P, I, P, P, I, I, I, I, I, I, I, P, P, S],
    "ragk_gemm_dec_splits": [I, I, I],
    "ragk_rmsnorm": [P, I, P, I, P, P, I, I, I, F, S],
    "ragk_layernorm": [P, I, P, I, P, P, P, I, I, I, F, S],
    "ragk_embed": [P, P, P, I, I, I, S],
    "ragk_embed_carry": [P, P, P, P, P, I, I, I, S],
    "ragk_embed_ln": [P, P, P, P, P, P, P, P, I, I, F, I, S],
    "ragk_rope_kv": [P, I, P, P, P, P, P, P, I, I, I, I, I, I, S],
    "ragk_pool_l2norm": [P, I, P, P, I, I, I, I, S],
    "ragk_silu_mul": [P, I, P, I, I, I, S],
    "ragk_gather_rows": [P, I, P, P, I, I, I, S],
    "ragk_attn_prefill_qtile": [I, I],
    "ragk_attn_prefill": [P, I, P, P, I, P, I, P, P, P, P, I, P, I, I, I, I, I, I, F, S],
    "ragk_attn_decode": [P, I, P, P, P, I, P, P, P, P, I, I, I, I, I, I, I, F, S],
    "ragk_attn_decode_rope": [P, I, I, P, P, P, P, P, P, P, I, P, P, P, P, I, I, I, I, I, I, I, F, S],
    "ragk_topk_candidates": [P, I, I, I, I, I, I, P, P, S],
    "ragk_sample_candidates": [P, P, I, I, P, P, P, P, P, P, P, S],
    "ragk_sample_candidates_lists": [P, P, I, I, I, P, P, P, P, P, P, P, S],
    "ragk_l2_scan_groups": [I, I, I],
    "ragk_l2_search_groups": [I, I, I, I, I],
    "ragk_l2_search_set_mfma_min_nq": [I],
    "ragk_l2_search": [P, I, I, I, I, P, I, I, P, P, P, P, P, S],
    "ragk_ivf_search": [P, I, I, P, I, P, I, P, P, P, I, P, P, P, P, S],
    "ragk_kmeans_assign": [P, I, I, P, P, I, P, P, P, S],
    "ragk_l2_scatter": [P, I, I, P, P, I, S],
    "ragk_l2_append": [P, I, I, I, P, I, S],
    "ragk_l2_gather": [P, I, I, P, I, P, S],
    "ragk_gemm_stream": [P, I, P, I, P, P, I, P, P, I, I, I, I, I, I, I, P, P, S],
    "ragk_gemm_stream_splits": [I, I, I, I],
    "ragk_quant_fp8_rows": [P, I, P, I, P, I, I, S],
    "ragk_gemm_fp8": [P, I, P, I, P, P, I, P, P, I, P, P, I, I, I, I, I, I, S],
    # csrc/comm/allreduce.hip (xGMI peer-mapped all-reduce)
    "ragk_ar_create": [I, I, ctypes.c_long, I, I, I],
    "ragk_ar_add_rmsnorm": [P, P, I, I, P, I, P, P, I, I, F, I, S],
    "ragk_ar_fused_rows": [P],
    "ragk_ar_ipc_handle": [P, P],
    "ragk_ar_handle_size": [],
    "ragk_ar_open_peers": [P, P],
    "ragk_ar_max_bytes": [P],
    "ragk_ar_allreduce": [P, P, P, ctypes.c_long, I, S],
    "ragk_ar_error": [P],
    "ragk_ar_set_spin_limit": [P, ctypes.c_uint],
    "ragk_ar_error_host_ptr": [P],
    "ragk_ar_allgather": [P, P, P, ctypes.c_long, S],
    "ragk_ar_destroy": [P],
    "ragk_ar_set_fences": [P, I],
    "ragk_ar_get_fences": [P],
}
_RESTYPES = {"ragk_host_word_alloc": ctypes.c_void_p, "ragk_host_word_dev": ctypes.c_void_p,
             "ragk_ar_create": ctypes.c_void_p, "ragk_ar_error_host_ptr": ctypes.c_void_p, "ragk_ar_max_bytes": ctypes.c_long, "ragk_ar_destroy": None}

_lib = None
_lock = threading.Lock()


class NativeLibraryError(RuntimeError):
    pass


def available() -> bool:
    return os.path.exists(LIB_PATH)


def lib():
    """Load (once) and return the kernel library. Raises if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise NativeLibraryError(
                "gfx950 kernel library not built (%s). Run `python -m rag_llm_k8s_amd._build` "
                "or __graft_entry__.build()." % LIB_PATH)
        h = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        _check_stamp(h)
        for name, args in _SIGS.items():
            fn = getattr(h, name)
            fn.argtypes = args
            fn.restype = _RESTYPES.get(name, ctypes.c_int)
        _lib = h
        return h


def _check_stamp(h):
    """The library must have been built from the kernel sources in this tree (content hash compiled in
    by _build.build_hip). RAGK_ALLOW_STALE_LIB=1 skips the check (kernel A/B work only)."""
    if os.environ.get("RAGK_ALLOW_STALE_LIB") == "1":
        return
    from .. import _build

    srcs, _ = _build.hip_sources()
    if not srcs:  # installed without sources: nothing to compare against
        return
    if not hasattr(h, "ragk_build_stamp"):
        raise NativeLibraryError("%s has no build stamp: rebuild it (python -m rag_llm_k8s_amd._build)" % LIB_PATH)
    f = h.ragk_build_stamp
    f.restype = ctypes.c_char_p
    f.argtypes = []
    got, want = f().decode(), _build.source_hash()
    if got != want:
        raise NativeLibraryError("%s was built from other kernel sources (stamp %s, tree %s): rebuild it "
                                 "(python -m rag_llm_k8s_amd._build)" % (LIB_PATH, got, want))


def build_stamp():
    h = lib()
    f = h.ragk_build_stamp
    f.restype = ctypes.c_char_p
    return f().decode()


def has_symbol(name: str) -> bool:
    try:
        return hasattr(lib(), name)
    except NativeLibraryError:
        return False


def stream_ptr(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def check(rc: int, what: str):
    if rc != 0:
        raise NativeLibraryError("%s failed with hipError %d" % (what, rc))


def ptr(t):
    return None if t is None else t.data_ptr()
