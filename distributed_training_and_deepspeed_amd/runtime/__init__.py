"""Native host runtime (C++, ``runtime/csrc``): gradient-readiness tracking for the reducers and
a worker-pool batch producer for the data path.  See ``runtime/native.py``."""
from __future__ import annotations

import ctypes

import torch

from . import native as _n


class ReadyTracker:
    """Per-window gradient-contribution counting and bucket launch decisions (reducer.cpp).

    ``bucket_of[i]`` is the bucket of parameter ``i``; ``ordered[b]`` False marks a bucket that
    launches as soon as it is complete (ZeRO-3 units) instead of in bucket order."""

    def __init__(self, bucket_of, nbuckets: int, ordered=None):
        L = _n.lib()
        self._lib = L
        self.nparams, self.nbuckets = len(bucket_of), int(nbuckets)
        ob = None
        if ordered is not None:
            ob = (ctypes.c_uint8 * self.nbuckets)(*[1 if o else 0 for o in ordered])
        self._h = L.dtd_tracker_create(self.nparams, _n.int_array(list(bucket_of)), self.nbuckets,
                                       ctypes.cast(ob, ctypes.c_void_p) if ob is not None else None)
        if not self._h:
            raise ValueError("invalid bucket assignment for the readiness tracker")
        self._out = (ctypes.c_int * max(self.nbuckets, 1))()

    def close(self) -> None:
        """Free the native state (otherwise it lives as long as the process: a few bytes per
        parameter; no finaliser runs at interpreter shutdown)."""
        h, self._h = getattr(self, "_h", None), None
        if h:
            self._lib.dtd_tracker_destroy(h)

    def reset(self) -> None:
        self._lib.dtd_tracker_reset(self._h)

    def expect(self, i: int) -> None:
        self._lib.dtd_tracker_expect(self._h, i)

    def contribute(self, i: int, autograd: bool = False, allow_launch: bool = True):
        """-> (ready, buckets to launch now)"""
        r = self._lib.dtd_tracker_contribute(self._h, i, int(autograd), int(allow_launch), self._out, self.nbuckets)
        if r < 0:
            raise IndexError(i)
        if r <= 1:
            return r == 1, []
        return True, [self._out[k] for k in range(r - 1)]

    def drain(self) -> list[int]:
        n = self._lib.dtd_tracker_drain(self._h, self._out, self.nbuckets)
        return [self._out[k] for k in range(n)]

    def is_ready(self, i: int) -> bool:
        return self._lib.dtd_tracker_is_ready(self._h, i) == 1

    def is_launched(self, b: int) -> bool:
        return self._lib.dtd_tracker_is_launched(self._h, b) == 1

    def ready_count(self, b: int) -> int:
        return self._lib.dtd_tracker_ready_count(self._h, b)

    def stats(self) -> dict:
        return {"windows": self._lib.dtd_tracker_stat(self._h, 0), "launches": self._lib.dtd_tracker_stat(self._h, 1)}


def assign_buckets(offsets, numels, total: int, cap_elems: int):
    """Greedy consecutive bucketing (reducer.cpp): -> (bucket_of list, [(start, end), ...])."""
    n = len(offsets)
    if n == 0:
        return [], []
    bo = (ctypes.c_int * n)()
    st = (ctypes.c_longlong * n)()
    en = (ctypes.c_longlong * n)()
    nb = _n.lib().dtd_bucket_assign(n, _n.ll_array(list(offsets)), _n.ll_array(list(numels)), int(total),
                                    int(cap_elems), bo, st, en, n)
    if nb < 0:
        raise RuntimeError("bucket assignment overflow")
    return list(bo), [(st[k], en[k]) for k in range(nb)]


class BatchProducer:
    """Worker pool that fills (pinned) host batches asynchronously (loader.cpp)."""

    def __init__(self, threads: int = 0):
        self._lib = _n.lib()
        self._h = self._lib.dtd_loader_create(int(threads))

    def __del__(self):
        h, self._h = getattr(self, "_h", None), None
        if h:
            self._lib.dtd_loader_destroy(h)

    @property
    def threads(self) -> int:
        return self._lib.dtd_loader_threads(self._h)

    def wait(self, job: int) -> None:
        self._lib.wait_nogil(self._h, job)   # releases the GIL while the workers finish

    def gather(self, src: torch.Tensor, idx: torch.Tensor, dst: torch.Tensor, wait: bool = True) -> int:
        """dst[i] = src[idx[i]] (rows), CPU tensors, contiguous; returns the job id."""
        assert src.is_contiguous() and dst.is_contiguous() and not src.is_cuda and not dst.is_cuda
        idx = idx.to(torch.int64).contiguous()
        n = idx.numel()
        row = src[0].numel() * src.element_size() if src.dim() > 0 and src.shape[0] else 0
        assert dst.shape[0] >= n and dst.dtype == src.dtype and dst[0].numel() == src[0].numel()
        job = self._lib.dtd_loader_gather(self._h, src.data_ptr(), src.shape[0], row, idx.data_ptr(), n,
                                          dst.data_ptr())
        if job < 0:
            raise IndexError("gather index out of range")
        if wait:
            self.wait(job)
        return job

    def synthesize(self, cfg, seed: int, row0: int, ids: torch.Tensor, labels: torch.Tensor, mlm: bool = True,
                   mlm_probability: float = 0.15, wait: bool = True) -> int:
        """Synthetic rows row0 .. row0+n-1 of the (seed) stream into int64 [n, seq] tensors."""
        assert ids.dtype == torch.int64 and labels.dtype == torch.int64 and ids.is_contiguous()
        assert labels.is_contiguous() and ids.shape == labels.shape and not ids.is_cuda
        specials = sorted(set(cfg.special_token_ids))[:8]
        bert = cfg.family == "bert"
        lo = min(max(specials) + 1, cfg.vocab_size - 1) if bert and specials else 0
        sp = _n.SynthSpec(seed=int(seed) & (2 ** 64 - 1), row0=int(row0), nrows=ids.shape[0], seq=ids.shape[1],
                          vocab=cfg.vocab_size, lo=lo, cls=101 if bert else -1, sep=102 if bert else -1,
                          mask_id=cfg.mask_token_id if mlm else -1, mlm=int(mlm), mlm_p=float(mlm_probability),
                          nspecial=len(specials))
        for k, s in enumerate(specials):
            sp.special[k] = s
        job = self._lib.dtd_loader_synth(self._h, ctypes.byref(sp), ids.data_ptr(), labels.data_ptr())
        if job < 0:
            raise ValueError("invalid synthetic batch spec")
        if wait:
            self.wait(job)
        return job
