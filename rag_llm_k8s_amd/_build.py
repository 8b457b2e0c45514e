"""In-tree native build for the framework.

Two artefacts, both written into ``rag_llm_k8s_amd/_lib/`` so they travel with the
repository snapshot to the GPU box:

* ``libragk_hip.so``  -- every gfx950 HIP kernel in ``csrc/kernels/*.hip``
  (hipcc --offload-arch=gfx950), C ABI, loaded with ctypes after ``import torch``
  so it binds to torch's HIP runtime (same ``libamdhip64.so.7`` SONAME).
* ``_ragk_rt*.so``    -- the C++ host runtime in ``csrc/runtime/*.cpp`` (pybind11):
  safetensors mmap reader, faiss-format index I/O, tokenizers, KV block manager.

Incremental: an object is rebuilt only when its source or a header is newer -- and everything is
rebuilt when the content hash of the kernel sources (+ flags) differs from the one recorded at the
last build. That hash is compiled into the library (``ragk_build_stamp()``); ``ops/_lib.py`` checks
it against the sources at load, so a library that does not match the tree is never used silently.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import hashlib
import os
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_DIR = os.path.join(ROOT, "rag_llm_k8s_amd", "_lib")
OBJ_DIR = os.path.join(ROOT, "build", "obj")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
HIP_LIB = os.path.join(LIB_DIR, "libragk_hip.so")


# per-file flags: gemm_w4.hip is written in its final instruction order (see its header)
EXTRA_FLAGS = {"gemm_w4.hip": ["-mllvm", "-disable-post-ra"]}


HIP_FLAGS = ["-O3", "--offload-arch=" + ARCH, "-fPIC", "-std=c++17", "-Wno-unused-result", "-munsafe-fp-atomics"]


def hip_sources():
    kdir = os.path.join(ROOT, "csrc", "kernels")
    cdir = os.path.join(ROOT, "csrc", "comm")
    srcs = sorted(glob.glob(os.path.join(kdir, "*.hip")) + glob.glob(os.path.join(cdir, "*.hip")))
    headers = sorted(glob.glob(os.path.join(kdir, "*.h")) + glob.glob(os.path.join(cdir, "*.h")))
    return srcs, headers


def source_hash():
    """Content hash of every kernel source and header plus the compile flags (no mtimes)."""
    srcs, headers = hip_sources()
    h = hashlib.sha256()
    h.update(repr((HIP_FLAGS, sorted(EXTRA_FLAGS.items()))).encode())
    for f in srcs + headers:
        h.update(os.path.relpath(f, ROOT).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
        h.update(b"\0")
    return h.hexdigest()[:32]


def _newer(src_files, target):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(s) > t for s in src_files)


def _run(cmd):
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError("build failed: %s\n%s" % (" ".join(cmd), r.stdout))
    return r.stdout


def check_lds_waits(objs, jobs=4):
    """Build step: every freshly compiled kernel object passes tools/isa_lds_hazard.py (no instruction touches
    an LDS read's registers before the lgkmcnt that retires it -- the hand-placed asm waits of gemm_w4 and
    the attention kernels). A hazard fails the build; a tree without the tool or llvm-objdump skips it."""
    tool = os.path.join(ROOT, "tools", "isa_lds_hazard.py")
    if not os.path.exists(tool):
        return
    import importlib.util

    spec = importlib.util.spec_from_file_location("isa_lds_hazard", tool)
    H = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(H)
    if not os.path.exists(os.path.join(H.LLVM, "llvm-objdump")):
        return
    with cf.ThreadPoolExecutor(jobs) as ex:
        bad = [(o, b) for o, b in zip(objs, ex.map(H.check_object, objs)) if b]
    if bad:
        for o in {o for o, _ in bad}:
            os.remove(o)  # recompiled (and re-checked) by the next build
        raise RuntimeError("LDS-wait hazards in %s" % "; ".join(
            "%s: %s at %#x" % (os.path.basename(o), k, h[0][0]) for o, b in bad for k, h in b[:2]))


def build_hip(verbose=False, jobs=None):
    os.makedirs(OBJ_DIR, exist_ok=True)
    os.makedirs(LIB_DIR, exist_ok=True)
    kdir = os.path.join(ROOT, "csrc", "kernels")
    srcs, headers = hip_sources()
    flags = HIP_FLAGS + ["-I" + kdir]
    stamp = source_hash()
    stamp_txt = os.path.join(OBJ_DIR, "ragk_stamp.txt")
    prev = open(stamp_txt).read().strip() if os.path.exists(stamp_txt) else None
    objs, todo = [], []
    for s in srcs:
        o = os.path.join(OBJ_DIR, os.path.basename(s) + ".o")
        objs.append(o)
        if prev != stamp or _newer([s] + headers + [os.path.abspath(__file__)], o):
            todo.append((s, o))
    stamp_src = os.path.join(OBJ_DIR, "ragk_stamp.cpp")
    stamp_obj = stamp_src + ".o"
    if prev != stamp or not os.path.exists(stamp_obj):
        with open(stamp_src, "w") as f:
            f.write('extern "C" __attribute__((visibility("default"))) const char* ragk_build_stamp() '
                    '{ return "%s"; }\n' % stamp)
        _run(["g++", "-O2", "-fPIC", "-c", stamp_src, "-o", stamp_obj])
    objs.append(stamp_obj)
    jobs = jobs or min(8, os.cpu_count() or 4)
    with cf.ThreadPoolExecutor(jobs) as ex:
        futs = [ex.submit(_run, [HIPCC] + flags + EXTRA_FLAGS.get(os.path.basename(s), []) + ["-c", s, "-o", o])
                for s, o in todo]
        for f in futs:
            out = f.result()
            if verbose and out.strip():
                print(out)
    if todo:
        check_lds_waits([o for _, o in todo], jobs)
    if todo or prev != stamp or _newer(objs, HIP_LIB):
        _run([HIPCC, "-shared", "-fPIC", "--offload-arch=" + ARCH] + objs + ["-o", HIP_LIB])
        with open(stamp_txt, "w") as f:
            f.write(stamp + "\n")
    return HIP_LIB


def runtime_ext_path():
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    return os.path.join(LIB_DIR, "_ragk_rt" + suffix)


RT_FLAGS = ["-O2", "-fPIC", "-std=c++17", "-fvisibility=hidden", "-Wall", "-Wno-unused-function"]


def runtime_sources():
    rdir = os.path.join(ROOT, "csrc", "runtime")
    return sorted(glob.glob(os.path.join(rdir, "*.cpp"))), sorted(glob.glob(os.path.join(rdir, "*.h")))


def runtime_source_hash():
    """Content hash of the host-runtime sources + flags, compiled into _ragk_rt (build_stamp()) and
    checked by runtime.native_rt() at import: a stale runtime (tokenizer, block manager) never loads
    silently -- the same contract as libragk_hip.so's stamp."""
    srcs, headers = runtime_sources()
    h = hashlib.sha256()
    h.update(repr(RT_FLAGS).encode())
    for f in srcs + headers:
        h.update(os.path.relpath(f, ROOT).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
        h.update(b"\0")
    return h.hexdigest()[:32]


def build_runtime(verbose=False):
    import pybind11

    os.makedirs(LIB_DIR, exist_ok=True)
    rdir = os.path.join(ROOT, "csrc", "runtime")
    srcs, headers = runtime_sources()
    if not srcs:
        return None
    target = runtime_ext_path()
    os.makedirs(OBJ_DIR, exist_ok=True)
    inc = ["-I" + pybind11.get_include(), "-I" + sysconfig.get_paths()["include"], "-I" + rdir]
    stamp = runtime_source_hash()
    stamp_txt = os.path.join(OBJ_DIR, "rt_stamp.txt")
    prev = open(stamp_txt).read().strip() if os.path.exists(stamp_txt) else None
    flags = RT_FLAGS + ['-DRAGK_RT_STAMP="%s"' % stamp]
    objs, todo = [], []
    for s in srcs:
        o = os.path.join(OBJ_DIR, "rt_" + os.path.basename(s) + ".o")
        objs.append(o)
        if prev != stamp or _newer([s] + headers, o):
            todo.append((s, o))
    with cf.ThreadPoolExecutor(min(8, os.cpu_count() or 4)) as ex:
        for f in [ex.submit(_run, ["g++"] + flags + inc + ["-c", s, "-o", o]) for s, o in todo]:
            out = f.result()
            if verbose and out.strip():
                print(out)
    if todo or prev != stamp or _newer(objs, target):
        _run(["g++", "-shared", "-fPIC"] + objs + ["-o", target])
        with open(stamp_txt, "w") as f:
            f.write(stamp + "\n")
    return target


def build_all(verbose=False):
    paths = [build_hip(verbose=verbose), build_runtime(verbose=verbose)]
    return [p for p in paths if p]


if __name__ == "__main__":
    for p in build_all(verbose="-v" in sys.argv):
        print(p)
