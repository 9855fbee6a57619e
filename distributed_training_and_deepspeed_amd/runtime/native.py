"""Build + ctypes binding of the native host runtime (``runtime/_dtd_runtime.so``).

``runtime/csrc/*.cpp`` is plain C++17 host code (g++, no HIP): the gradient-readiness tracker at
the core of the DDP reducer and the ZeRO engine (``reducer.cpp``) and the worker-pool batch
producer of the data path (``loader.cpp``).  The library is built in-tree (it ships to the GPU
box with the tree) and is REQUIRED: the reducers and loaders call into it on CPU and GPU alike,
and an import fails loudly if it cannot be built or loaded.
"""
from __future__ import annotations

import ctypes
import os
import shutil
import subprocess
import sys
import threading
from pathlib import Path

HERE = Path(__file__).resolve().parent
CSRC = HERE / "csrc"
LIB_PATH = HERE / "_dtd_runtime.so"

_LIB = None
_LOCK = threading.Lock()

P, I, LL, U8 = ctypes.c_void_p, ctypes.c_int, ctypes.c_longlong, ctypes.c_uint8
IP = ctypes.POINTER(ctypes.c_int)
LLP = ctypes.POINTER(ctypes.c_longlong)


class SynthSpec(ctypes.Structure):
    _fields_ = [("seed", ctypes.c_uint64), ("row0", ctypes.c_int64), ("nrows", ctypes.c_int64),
                ("seq", ctypes.c_int32), ("vocab", ctypes.c_int32), ("lo", ctypes.c_int32),
                ("cls", ctypes.c_int32), ("sep", ctypes.c_int32), ("mask_id", ctypes.c_int32),
                ("mlm", ctypes.c_int32), ("mlm_p", ctypes.c_float), ("nspecial", ctypes.c_int32),
                ("special", ctypes.c_int32 * 8)]


_SIGS = {
    "dtd_tracker_create": (P, [I, IP, I, P]),
    "dtd_tracker_destroy": (None, [P]),
    "dtd_tracker_reset": (None, [P]),
    "dtd_tracker_expect": (I, [P, I]),
    "dtd_tracker_contribute": (I, [P, I, I, I, IP, I]),
    "dtd_tracker_drain": (I, [P, IP, I]),
    "dtd_tracker_is_ready": (I, [P, I]),
    "dtd_tracker_is_launched": (I, [P, I]),
    "dtd_tracker_ready_count": (I, [P, I]),
    "dtd_tracker_stat": (LL, [P, I]),
    "dtd_bucket_assign": (I, [I, LLP, LLP, LL, LL, IP, LLP, LLP, I]),
    "dtd_loader_create": (P, [I]),
    "dtd_loader_destroy": (None, [P]),
    "dtd_loader_threads": (I, [P]),
    "dtd_loader_wait": (None, [P, I]),
    "dtd_loader_gather": (I, [P, P, LL, LL, P, LL, P]),
    "dtd_loader_synth": (I, [P, ctypes.POINTER(SynthSpec), P, P]),
}


def _sources():
    return sorted(CSRC.glob("*.cpp")) + sorted(CSRC.glob("*.h"))


def needs_build() -> bool:
    if not LIB_PATH.exists():
        return True
    t = LIB_PATH.stat().st_mtime
    return any(p.stat().st_mtime > t for p in _sources() + [Path(__file__)])


def build(force: bool = False, verbose: bool = True) -> Path:
    """Compile in-tree.  Concurrent callers (every rank of a spawned job importing a stale
    library) serialise on a lock file and write through private temporaries, so no process
    ever loads a half-written library."""
    import fcntl
    if not force and not needs_build():
        return LIB_PATH
    with open(HERE / ".build.lock", "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        try:
            if not force and not needs_build():   # another process built it meanwhile
                return LIB_PATH
            return _build_locked(verbose)
        finally:
            fcntl.flock(lk, fcntl.LOCK_UN)


def _build_locked(verbose: bool) -> Path:
    cxx = os.environ.get("CXX") or shutil.which("g++") or shutil.which("c++")
    if not cxx:
        raise RuntimeError("no C++ compiler (g++) found for the native runtime")
    tmp = LIB_PATH.with_suffix(f".so.tmp{os.getpid()}")
    cmd = [cxx, "-O2", "-std=c++17", "-shared", "-fPIC", "-pthread", "-fvisibility=hidden",
           *map(str, sorted(CSRC.glob("*.cpp"))), "-o", str(tmp)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"native runtime build failed:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, LIB_PATH)
    if verbose:
        print(f"[dtd.build] wrote {LIB_PATH}", file=sys.stderr)
    return LIB_PATH


def lib():
    global _LIB
    if _LIB is not None:
        return _LIB
    with _LOCK:
        if _LIB is None:
            if os.environ.get("DTD_NO_BUILD") != "1" and needs_build():
                build()
            # PyDLL: the calls keep the GIL (they are sub-microsecond bookkeeping, made from
            # autograd hooks); only the blocking loader wait goes through a GIL-releasing handle
            so = ctypes.PyDLL(str(LIB_PATH))
            for name, (res, args) in _SIGS.items():
                fn = getattr(so, name)
                fn.restype = res
                fn.argtypes = args
            nogil = ctypes.CDLL(str(LIB_PATH))
            so.wait_nogil = nogil.dtd_loader_wait
            so.wait_nogil.restype = None
            so.wait_nogil.argtypes = [P, I]
            _LIB = so
    return _LIB


def int_array(vals):
    return (ctypes.c_int * len(vals))(*vals)


def ll_array(vals):
    return (ctypes.c_longlong * len(vals))(*vals)
