"""ctypes binding of the in-tree gfx950 kernel library ``ops/_dtd_kernels.so``.

The library exposes a C ABI (``extern "C" int dtd_*(..., hipStream_t)``); every launch goes
onto torch's *current* HIP stream, so kernels interleave correctly with hipBLASLt GEMMs and
RCCL collectives issued by torch, and are captured by ``torch.cuda.graph`` like any ATen op.

On a machine with a GPU the library is REQUIRED: ``lib()`` raises if it cannot be built or
loaded (no silent fallback to eager PyTorch on the GPU path).  On CPU-only hosts the pure
PyTorch reference branches of ``ops/functional.py`` are used instead.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path
import threading

import torch  # noqa: F401  (must be imported first: binds libamdhip64 to torch's runtime)

from . import build as _build

_LIB = None
_LOCK = threading.Lock()

P = ctypes.c_void_p
I = ctypes.c_int
F = ctypes.c_float
SZ = ctypes.c_size_t
U32 = ctypes.c_uint32

_SIGS = {
    # norm.hip
    "dtd_ln_bwd_num_partials": (I, [I, I]),
    "dtd_ln_fwd": (I, [I, P, P, P, P, P, P, P, P, I, I, F, F, P, U32, P]),
    "dtd_ln_bwd": (I, [I, P, P, P, P, P, P, P, P, P, P, P, P, I, I, F, P, U32, P]),
    "dtd_ln_bwd_fo": (I, [I, P, P, P, P, P, P, P, P, P, P, P, P, I, I, F, P, U32, P]),
    # act.hip
    "dtd_act_fwd": (I, [I, P, P, SZ, I, P]),
    "dtd_act_bwd_num_partials": (I, [I, I]),
    "dtd_act_bwd": (I, [I, P, P, P, P, P, I, I, I, P]),
    "dtd_colsum_finalize": (I, [P, I, I, P, I, I, F, P]),
    "dtd_colsum_finalize_multi": (I, [I, P, I, I, P, I, I, P, I, I, P, I, I, P]),
    "dtd_colsum_finalize_batch": (I, [I, P, P]),
    "dtd_embed_word_bwd_chunked": (I, [I, I, P, P, P, P, P, P, P, I, I, I, I, P]),
    # xent.hip
    "dtd_xent_fwd": (I, [I, P, P, P, P, P, I, I, I, P]),
    "dtd_xent_bwd": (I, [I, P, P, P, P, P, P, I, I, I, P]),
    "dtd_xent_bwd_colsum_parts": (I, [I]),
    "dtd_xent_bwd_colsum_supported": (I, [I]),
    "dtd_xent_bwd_colsum": (I, [P, P, P, P, P, P, P, I, I, I, P]),
    "dtd_xent_fwd_train": (I, [P, P, P, P, P, P, P, I, I, I, P]),
    "dtd_xent_grad_scale": (I, [P, SZ, P, P]),
    # embed.hip
    "dtd_embed_fwd": (I, [I, P, P, P, P, P, P, I, I, I, I, P]),
    "dtd_embed_word_bwd": (I, [I, I, P, P, P, P, I, I, I, I, P]),
    "dtd_embed_pos_bwd": (I, [I, I, P, P, I, I, I, I, I, P]),
    "dtd_scatter_rows": (I, [P, P, P, I, P, I, I, P]),
    "dtd_dropout": (I, [I, P, P, P, SZ, F, P, U32, P]),
    "dtd_embed_ln_fwd": (I, [P, P, P, P, P, P, P, P, P, P, P, I, I, I, I, F, F, P, U32, P]),
    # adam.hip
    "dtd_adam_step": (I, [P, P, P, P, I, P, SZ, P, I, P]),
    "dtd_scale_cast": (I, [P, I, P, I, SZ, F, P, P]),
    "dtd_sqnorm_num_partials": (I, [SZ]),
    "dtd_sqnorm_partials": (I, [P, I, SZ, P, P]),
    # attention.hip
    "dtd_attn_fwd": (I, [P, P, P, P, P, P, P, I, I, I, I, I, I, I, F, F, P, U32, P]),
    "dtd_attn_bwd": (I, [P, P, P, P, P, P, P, P, P, P, P, P, I, I, I, I, I, I, I, F, F, P, P]),
    "dtd_attn_masks": (I, [P, I, I, I, F, P, U32, P]),
    "dtd_attn_set_bwd_form": (I, [I]),
    "dtd_attn_fused_bwd_built": (I, []),
    # attention_f32.hip
    "dtd_attn_fwd_f32": (I, [P, P, P, P, P, P, P, I, I, I, I, I, I, I, F, F, P]),
    "dtd_attn_bwd_f32": (I, [P, P, P, P, P, P, P, P, P, P, P, P, I, I, I, I, I, I, I, F, F, P]),
    # softmax.hip
    "dtd_softmax_fwd": (I, [I, P, P, I, I, P]),
    "dtd_softmax_bwd": (I, [I, P, P, P, I, I, P]),
    # gemm.hip
    "dtd_gemm_bt_supported": (I, [I, I, I]),
    # gemm_w4.hip
    "dtd_gemm_w4_supported": (I, [I, I, I]),
    "dtd_gemm_w4_set_sched": (I, [I]),
    "dtd_gemm_w4": (I, [I, P, I, P, I, P, I, P, I, I, I, P]),
    "dtd_gemm_bt_part_rows": (I, [I]),
    "dtd_gemm_bt": (I, [I, P, I, P, I, P, I, P, P, I, P, P, I, I, I, P, P]),
    "dtd_spin_occupy": (I, [I, ctypes.c_double, P]),
    "dtd_gemm_set_stagger": (I, [ctypes.c_double]),
    "dtd_transpose_bf16": (I, [P, P, I, I, P]),
    "dtd_transpose_many": (I, [P, P, P, P, I, P]),
    "dtd_gemm_set_stamps": (I, [P]),
    # wgrad.hip
    "dtd_wgrad_tn_supported": (I, [I, I, I]),
    "dtd_wgrad_tn_splits": (I, [I, I, I]),
    "dtd_wgrad_tn": (I, [I, P, I, P, I, P, I, I, I, I, P]),
    # gemm_f32.hip
    "dtd_gemm_f32_supported": (I, [I, I, I]),
    "dtd_gemm_f32_set_kernel": (I, [I]),
    "dtd_gemm_f32_nt": (I, [P, I, P, I, P, I, P, I, I, I, I, P]),
    "dtd_gemm_f32_nn": (I, [P, I, P, I, P, I, I, I, I, I, P]),
    "dtd_transpose_many_f32": (I, [P, P, P, P, I, P]),
    "dtd_gemm_f32_tn_splits": (I, [I, I, I]),
    "dtd_gemm_f32_tn": (I, [P, I, P, I, P, I, I, I, I, P]),
    # gemm_ln.hip
    "dtd_gemm_ln_supported": (I, [I, I, I, I, I, I, I]),
    "dtd_gemm_ln": (I, [P, P, P, P, P, P, P, P, P, P, I, I, I, I, I, I, I, F, F, P, U32, P]),
    # reduce.hip
    "dtd_splitk_reduce": (I, [P, I, I, ctypes.c_longlong, P, I, I, P]),
}


class KernelError(RuntimeError):
    pass


def available() -> bool:
    """True when a GPU is present (the HIP library is then mandatory)."""
    return torch.cuda.is_available()


def lib():
    """Load (building first if stale) the kernel library. Raises on failure."""
    global _LIB
    if _LIB is not None:
        return _LIB
    with _LOCK:
        if _LIB is not None:
            return _LIB
        path = _build.LIB_PATH
        override = os.environ.get("DTD_KERNELS_SO")   # A/B runs: an alternative build of the library
        if override:
            path = Path(override)
        elif os.environ.get("DTD_NO_BUILD") != "1" and _build.needs_build():
            _build.build(verbose=True)
        if not path.exists():
            raise KernelError(f"HIP kernel library missing: {path} (run ops/build.py)")
        so = ctypes.CDLL(str(path), mode=ctypes.RTLD_GLOBAL)
        for name, (res, args) in _SIGS.items():
            fn = getattr(so, name, None)
            if fn is None:
                continue  # optional kernels (e.g. attention while under development)
            fn.restype = res
            fn.argtypes = args
        _LIB = so
        return _LIB


def has(name: str) -> bool:
    return hasattr(lib(), name)


DEBUG_SYNC = os.environ.get("DTD_DEBUG_SYNC", "0") == "1"


def call(name: str, *args) -> None:
    """Launch ``name``; raise on a launch error.  With ``DTD_DEBUG_SYNC=1`` (the framework's
    HIP_LAUNCH_BLOCKING-style debug mode) every kernel is followed by a device
    synchronisation, so an asynchronous fault is reported at the kernel that caused it."""
    rc = getattr(lib(), name)(*args)
    if rc != 0:
        raise KernelError(f"{name} failed with hipError {rc}")
    if DEBUG_SYNC:
        try:
            torch.cuda.synchronize()
        except RuntimeError as e:  # noqa: PERF203
            raise KernelError(f"{name}: device error after launch: {e}") from e


def stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def ptr(t) -> int | None:
    return None if t is None else t.data_ptr()


DT_F32, DT_BF16 = 0, 1


def dt(t: torch.Tensor) -> int:
    if t.dtype == torch.bfloat16:
        return DT_BF16
    if t.dtype == torch.float32:
        return DT_F32
    raise TypeError(f"unsupported dtype {t.dtype} (kernels take bf16 or fp32)")
