"""Distributed sampling and batch loading.

``DistributedSampler`` reproduces torch's semantics used by the reference
(data_parallel_training.py:41, zero_dp_training.py:66): a permutation seeded
with ``seed + epoch`` (shuffle=True default), padded by repetition to a multiple of the world
size (drop_last=False), then ``indices[rank::world]``.

``DeviceBatchLoader`` replaces the DataLoader hot path: the native worker pool
(``runtime/csrc/loader.cpp``) gathers a whole batch's rows straight into one of two reused
pinned host slots, and a single non-blocking H2D copy per tensor runs on a side stream, one
batch ahead, so the input copy overlaps the previous step's compute.  Datasets that produce rows
on demand (``NativeSyntheticLM``) are generated into the slot by the same workers instead.
"""
from __future__ import annotations

import math

import torch


class DistributedSampler(torch.utils.data.Sampler):
    def __init__(self, dataset, num_replicas: int | None = None, rank: int | None = None, shuffle: bool = True,
                 seed: int = 0, drop_last: bool = False):
        if num_replicas is None or rank is None:
            import torch.distributed as dist
            ws = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
            rk = dist.get_rank() if dist.is_available() and dist.is_initialized() else 0
            num_replicas = ws if num_replicas is None else num_replicas
            rank = rk if rank is None else rank
        self.dataset, self.num_replicas, self.rank = dataset, num_replicas, rank
        self.shuffle, self.seed, self.drop_last, self.epoch = shuffle, seed, drop_last, 0
        n = len(dataset)
        if drop_last and n % num_replicas:
            self.num_samples = math.ceil((n - num_replicas) / num_replicas)
        else:
            self.num_samples = math.ceil(n / num_replicas)
        self.total_size = self.num_samples * num_replicas

    def __iter__(self):
        n = len(self.dataset)
        if self.shuffle:
            g = torch.Generator()
            g.manual_seed(self.seed + self.epoch)
            indices = torch.randperm(n, generator=g).tolist()
        else:
            indices = list(range(n))
        if not self.drop_last:
            pad = self.total_size - len(indices)
            if pad <= len(indices):
                indices += indices[:pad]
            else:
                indices += (indices * math.ceil(pad / len(indices)))[:pad]
        else:
            indices = indices[: self.total_size]
        return iter(indices[self.rank:self.total_size:self.num_replicas])

    def __len__(self):
        return self.num_samples

    def set_epoch(self, epoch: int) -> None:
        self.epoch = epoch


class DeviceBatchLoader:
    """Iterate fixed-size batches of a tensor dataset directly onto a device."""

    SLOTS = 2

    def __init__(self, dataset, batch_size: int, sampler=None, device="cpu", drop_last: bool = False,
                 keys=("input_ids", "labels"), threads: int = 0):
        from ..runtime import BatchProducer
        self.dataset, self.batch_size, self.device = dataset, batch_size, torch.device(device)
        self.sampler = sampler if sampler is not None else range(len(dataset))
        self.drop_last, self.keys = drop_last, keys
        self._pin = self.device.type == "cuda"
        self._generate = hasattr(dataset, "fill_rows")           # on-demand rows (NativeSyntheticLM)
        self._host = {} if self._generate else {k: getattr(dataset, k).contiguous() for k in keys}
        self._producer = BatchProducer(threads)
        self._stream = torch.cuda.Stream(self.device) if self._pin else None
        self._slots: list = []        # per slot: {key: pinned [batch, ...] tensor}
        self._slot_ev: list = []      # per slot: event of the H2D copy that last read it
        self._next_slot = 0

    def __len__(self):
        n = len(self.sampler)
        return n // self.batch_size if self.drop_last else math.ceil(n / self.batch_size)

    def _batches(self):
        idx = list(iter(self.sampler))
        for i in range(0, len(idx), self.batch_size):
            chunk = idx[i:i + self.batch_size]
            if self.drop_last and len(chunk) < self.batch_size:
                return
            yield torch.as_tensor(chunk, dtype=torch.int64)

    def _host_slot(self, n: int):
        """A pinned slot for an n-row batch whose previous H2D copy has finished."""
        k = self._next_slot
        self._next_slot = (k + 1) % self.SLOTS
        if len(self._slots) <= k:
            self._slots.append({})
            self._slot_ev.append(None)
        if self._slot_ev[k] is not None:
            self._slot_ev[k].synchronize()
            self._slot_ev[k] = None
        slot = self._slots[k]
        for key in self.keys:
            t = slot.get(key)
            shape = (n,) + self._row_shape(key)
            if t is None or t.shape != shape:
                t = torch.empty(shape, dtype=self._dtype(key), pin_memory=self._pin)
                slot[key] = t
        return k, slot

    def _row_shape(self, key):
        return tuple(self.dataset.row_shape(key)) if self._generate else tuple(self._host[key].shape[1:])

    def _dtype(self, key):
        return self.dataset.row_dtype(key) if self._generate else self._host[key].dtype

    def _load(self, ix):
        n = ix.numel()
        if self._pin:
            k, host = self._host_slot(n)
        else:
            k, host = None, {key: torch.empty((n,) + self._row_shape(key), dtype=self._dtype(key)) for key in self.keys}
        if self._generate:
            self.dataset.fill_rows(ix, host, self._producer)
        else:
            jobs = [self._producer.gather(self._host[key], ix, host[key][:n], wait=False) for key in self.keys]
            for j in jobs:
                self._producer.wait(j)
        if not self._pin:
            return {key: v.to(self.device) for key, v in host.items()}
        out = {}
        with torch.cuda.stream(self._stream):
            for key, v in host.items():
                out[key] = v.to(self.device, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(self._stream)
        self._slot_ev[k] = ev     # the slot is reused only after this copy has read it
        return out

    def __iter__(self):
        # one batch ahead: batch i+1's gather + H2D copy is issued on the side stream before
        # batch i is handed out, so it overlaps batch i's compute; the compute stream waits
        # only on the event recorded after the copy of the batch it is about to consume
        it = self._batches()
        ix = next(it, None)
        if ix is None:
            return
        cur, ev = self._load(ix), self._record()
        for ix in it:
            nxt = self._load(ix)
            nev = self._record()
            yield self._handoff(cur, ev)
            cur, ev = nxt, nev
        yield self._handoff(cur, ev)

    def _record(self):
        if self._stream is None:
            return None
        ev = torch.cuda.Event()
        ev.record(self._stream)
        return ev

    def _handoff(self, batch, ev):
        if ev is not None:
            cs = torch.cuda.current_stream(self.device)
            cs.wait_event(ev)
            for t in batch.values():
                t.record_stream(cs)   # the side-stream allocation is not recycled under compute
        return batch
