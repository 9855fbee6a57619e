"""In-tree build of the gfx950 HIP kernel library (``ops/_dtd_kernels.so``).

Every ``ops/csrc/*.hip`` and ``comm/csrc/*.hip`` file is compiled with ``hipcc --offload-arch=gfx950`` into an object
and linked into one shared library that exports a plain C ABI (``extern "C" dtd_*``).
Python binds it with ctypes (``ops/_lib.py``) after ``import torch`` so the library resolves
``libamdhip64.so.7`` to the HIP runtime torch already loaded (one HIP runtime per process).

The library is rebuilt only when a source or header is newer than it.  Run directly:
``python -m distributed_training_and_deepspeed_amd.ops.build [--force] [-j N]``.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
CSRC = HERE / "csrc"
SRC_DIRS = (CSRC, HERE.parent / "comm" / "csrc")   # kernels + the native xGMI collectives
LIB_NAME = "_dtd_kernels.so"
LIB_PATH = HERE / LIB_NAME
OBJ_DIR = HERE / "build"
ARCH = os.environ.get("DTD_OFFLOAD_ARCH", "gfx950")


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found (set HIPCC or install ROCm)")


def sources() -> list[Path]:
    return sorted(p for d in SRC_DIRS for p in d.glob("*.hip"))


def _headers() -> list[Path]:
    return sorted(p for d in SRC_DIRS for p in d.glob("*.h"))


def needs_build() -> bool:
    if not LIB_PATH.exists():
        return True
    t = LIB_PATH.stat().st_mtime
    return any(p.stat().st_mtime > t for p in sources() + _headers() + [Path(__file__)])


def _file_flags(src: Path) -> list[str]:
    """Per-source hipcc flags: a ``// hipcc-flags: ...`` line among the first 80 of the file."""
    with open(src) as f:
        for i, line in enumerate(f):
            if i >= 80:
                break
            if line.startswith("// hipcc-flags:"):
                return line.split(":", 1)[1].split()
    return []


# DTD_BUILD_EXPERIMENTAL=1 also compiles the kernels that lost their A/B against the default path
# (the one-kernel attention backward, the fused projection + LayerNorm GEMM); they stay opt-in at
# run time as well.
EXPERIMENTAL_FLAGS = ["-DDTD_ATTN_FUSED_BWD=1", "-DDTD_GEMM_LN_BUILD=1"]


def _compile(src: Path, hipcc: str, extra: list[str]) -> Path:
    OBJ_DIR.mkdir(exist_ok=True)
    extra = [*_file_flags(src), *extra]
    if os.environ.get("DTD_BUILD_EXPERIMENTAL") == "1":
        extra += EXPERIMENTAL_FLAGS
    obj = OBJ_DIR / (src.stem + ".o")
    hdr_t = max((p.stat().st_mtime for p in _headers()), default=0)
    if obj.exists() and obj.stat().st_mtime > max(src.stat().st_mtime, hdr_t, Path(__file__).stat().st_mtime):
        return obj
    cmd = [hipcc, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-c", str(src), "-o", str(obj),
           "-I", str(CSRC), "-Wno-unused-command-line-argument", "-fvisibility=hidden", *extra]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src.name}:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return obj


def _check_kernel_stubs(lib: Path) -> None:
    """Refuse a library with unresolved kernel launch stubs: hipcc can drop a ``__global__``
    template's host stub without an error (e.g. a lambda inside the kernel body), which only
    surfaces as an ``undefined symbol`` when the library is loaded on the GPU box."""
    nm = shutil.which("nm") or "/opt/rocm/lib/llvm/bin/llvm-nm"
    if not Path(nm).exists():
        return
    r = subprocess.run([nm, "-D", "--undefined-only", str(lib)], capture_output=True, text=True)
    bad = [ln.split()[-1] for ln in r.stdout.splitlines() if "__device_stub__" in ln]
    if bad:
        raise RuntimeError(f"{lib.name}: unresolved kernel stubs (host side of a kernel was not emitted): {bad}")


def build(force: bool = False, jobs: int | None = None, verbose: bool = True) -> Path:
    """Compile all kernels for gfx950 and link ``_dtd_kernels.so`` in-tree; return its path.
    Concurrent callers (every rank of a job importing a stale library) serialise on a lock file
    (the objects in ``build/`` are shared) and the library is replaced atomically, so no process
    loads a half-written one."""
    import fcntl
    if not force and not needs_build():
        return LIB_PATH
    with open(HERE / ".build.lock", "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        try:
            if not force and not needs_build():   # another process built it meanwhile
                return LIB_PATH
            return _build_locked(force, jobs, verbose)
        finally:
            fcntl.flock(lk, fcntl.LOCK_UN)


def _build_locked(force: bool, jobs: int | None, verbose: bool) -> Path:
    hipcc = _hipcc()
    extra = os.environ.get("DTD_HIPCC_FLAGS", "").split()
    srcs = sources()
    if force and OBJ_DIR.exists():
        shutil.rmtree(OBJ_DIR)
    jobs = jobs or min(len(srcs), int(os.environ.get("MAX_JOBS", os.cpu_count() or 4)), 16)
    if verbose:
        print(f"[dtd.build] compiling {len(srcs)} HIP sources for {ARCH} with {jobs} jobs", file=sys.stderr)
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, hipcc, extra), srcs))
    tmp = LIB_PATH.with_suffix(f".so.tmp{os.getpid()}")
    cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(tmp), *map(str, objs)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    _check_kernel_stubs(tmp)
    os.replace(tmp, LIB_PATH)
    if verbose:
        print(f"[dtd.build] wrote {LIB_PATH}", file=sys.stderr)
    return LIB_PATH


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", "--jobs", type=int, default=None)
    a = ap.parse_args()
    build(force=a.force, jobs=a.jobs)
