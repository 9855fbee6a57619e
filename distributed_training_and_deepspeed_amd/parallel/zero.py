"""ZeRO data parallelism, stages 0-3, with a DeepSpeed-style engine API.

Reference: ``deepspeed.initialize(model, model_parameters, config)`` -> (engine, optimizer, _, _),
``engine(input_ids, labels=...)``, ``engine.backward(loss)``, ``engine.step()``,
``engine.zero_optimization_stage()`` and ``optimizer.param_groups[0]`` printing the *local*
partition size (/root/reference/zero_dp_training.py:26-57,81-94).

MI355X-first design (flat buffers, RCCL collectives on contiguous slices, no flatten copies):

* Parameters are grouped into *segments*.  A segment is a contiguous range of a flat buffer
  whose length is a multiple of world*64; rank r owns chunk r of EVERY segment, so gradient
  reduction is one ``reduce_scatter_tensor`` per segment and the parameter refresh one
  ``all_gather_into_tensor`` per segment -- no per-parameter "reduce to owner" calls.
  Each rank's chunks are packed into one shard buffer (fp32 master, Adam moments, gradient
  shard, low-precision copy), so the optimizer step is ONE fused-Adam launch per rank.
* stage 0: segments = ``allreduce_bucket_size`` buckets, gradients all-reduced (replicated
  optimizer state, DeepSpeed's "stage 0").
* stage 1: optimizer states partitioned; full gradient buffer, reduce-scatter after backward.
* stage 2: + gradients partitioned: a bucket's gradient landing region is taken from a
  persistent ring arena (``_Arena``) on its first write, reduce-scattered on the comm stream as
  soon as the bucket is complete (overlapping the rest of backward) and handed back with an
  event -- only the local gradient shard persists, and no buffer is allocated per step (the
  whole step is hipGraph-capturable).
* stage 3: + parameters partitioned: every model unit (embeddings, each transformer layer,
  head) keeps only its parameter shard; the unit is all-gathered into a gather arena on a
  SEPARATE communicator (``gather_group``: its RCCL stream runs beside the reduce-scatters
  instead of queueing behind them) before its forward/backward, with prefetch up to
  ``stage3_prefetch_bucket_size`` elements ahead, released after use, and its gradients are
  reduce-scattered as soon as its backward finishes.  Parameters shared between units (tied
  word embeddings) stay replicated with stage-2 treatment.
* After ``step()`` (stages >= 1) the updated shards are all-gathered back into the replicated
  buckets in FORWARD order, ``allgather_bucket_size`` elements per coalesced RCCL launch, each
  group recording an event; the next forward's per-unit pre-hooks wait only for the events of
  the buckets holding that unit's parameters, so the refresh of later layers overlaps the
  forward of earlier ones (DeepSpeed waits for the whole all-gather inside ``step()``).
* Collectives go through ``comm.logger`` (the DeepSpeed comms-logger equivalent).
"""
from __future__ import annotations

import contextlib
import math
import os

import torch
import torch.distributed as dist
from torch import nn

from .. import comm
from ..comm import logger as clog
from ..ops.functional import flush_finalizes
from ..optim.fused_adam import FusedAdam
from ..runtime import ReadyTracker
from .flat import ALIGN, unique_params

DEFAULTS = {
    "train_micro_batch_size_per_gpu": 1,
    "gradient_accumulation_steps": 1,
    "gradient_clipping": 0.0,
    "optimizer": {"type": "Adam", "params": {"lr": 1e-3}},
    "comms_logger": {"enabled": False},
    "zero_optimization": {"stage": 0, "reduce_bucket_size": 5e8, "allgather_bucket_size": 5e8,
                          "overlap_comm": None, "stage3_prefetch_bucket_size": 5e7,
                          "overlap_param_refresh": True, "world1_replicated": True,
                          "force_collectives": False, "stage3_gather_communicator": False,
                          "overlap_optimizer_step": False},
}


class ZeroConfig:
    def __init__(self, cfg: dict | None):
        cfg = dict(cfg or {})
        self.raw = cfg
        self.micro_batch = int(cfg.get("train_micro_batch_size_per_gpu", 1))
        self.gas = int(cfg.get("gradient_accumulation_steps", 1))
        self.clip = float(cfg.get("gradient_clipping", 0.0) or 0.0)
        opt = dict(DEFAULTS["optimizer"])
        opt.update(cfg.get("optimizer", {}))
        self.opt_type = str(opt.get("type", "Adam"))
        self.opt_params = dict(opt.get("params", {}))
        self.comms_logger = dict(cfg.get("comms_logger", {}))
        z = dict(DEFAULTS["zero_optimization"])
        z.update(cfg.get("zero_optimization", {}))
        self.stage = int(z.get("stage", 0))
        if self.stage not in (0, 1, 2, 3):
            raise ValueError(f"ZeRO stage must be 0-3, got {self.stage}")
        self.reduce_bucket = int(float(z.get("reduce_bucket_size", 5e8)))
        self.allreduce_bucket = int(float(cfg.get("allreduce_bucket_size", z.get("allreduce_bucket_size", 5e8))))
        self.allgather_bucket = max(1, int(float(z.get("allgather_bucket_size", 5e8))))
        self.prefetch_bucket = max(0, int(float(z.get("stage3_prefetch_bucket_size", 5e7))))
        self.overlap_refresh = bool(z.get("overlap_param_refresh", True))
        self.world1_replicated = bool(z.get("world1_replicated", True))
        # issue every collective even on a one-rank group (one-GPU rehearsal of the N > 1 path)
        self.force_collectives = (bool(z.get("force_collectives", False))
                                  or os.environ.get("DTD_FORCE_COLLECTIVES", "0") == "1")
        # stage 3 gathers on a second communicator beside the reduce-scatters: off by default --
        # RCCL documents that concurrent communicators on one device can deadlock when their
        # kernels cannot all be resident; the gathers then share the main group and its stream
        # order (they still run on their own HIP stream, fenced by events)
        self.gather_communicator = bool(z.get("stage3_gather_communicator", False))
        # race / stale-reference detector: fill every released stage-3 gather region
        # with NaN, so a read through a stale view of released weights poisons the result
        self.poison_released = (bool(z.get("debug_poison_released", False))
                                or os.environ.get("DTD_ZERO_POISON", "0") == "1")
        oc = z.get("overlap_comm")
        self.overlap = (self.stage >= 2) if oc is None else bool(oc)
        # Adam on each segment's shard as soon as the backward is past it (a side stream), instead
        # of one launch after the backward.  Opt-in: the update then starts inside backward(), so
        # the weights change before step() returns -- a loop must pair every backward() with a
        # step() (the reference scripts do) and not read weights in between.  Needs no gradient
        # clipping (the global norm is known only after the backward); env DTD_ZERO_OPT_OVERLAP=1/0
        # overrides the config key.
        env = os.environ.get("DTD_ZERO_OPT_OVERLAP")
        self.overlap_opt = bool(z.get("overlap_optimizer_step", False)) if env is None else env == "1"
        bf = cfg.get("bf16", {})
        self.bf16 = bool(bf.get("enabled", False)) if isinstance(bf, dict) else bool(bf)


class _Segment:
    __slots__ = ("index", "params", "shapes", "offsets", "numel", "chunk", "shard_off", "full", "gbuf", "ready",
                 "launched", "unit", "gather_event", "module", "pending_release", "first_use", "hold")

    def __init__(self, index, params, world):
        self.index = index
        self.params = params
        self.shapes = [tuple(p.shape) for p in params]  # kept: stage-3 params are emptied between uses
        self.offsets, off = [], 0
        for p in params:
            self.offsets.append(off)
            off += -(-p.numel() // ALIGN) * ALIGN
        q = world * ALIGN
        self.numel = max(q, -(-off // q) * q)
        self.chunk = self.numel // world
        self.shard_off = 0
        self.full = None      # full param buffer (persistent: view into flat; unit: gathered region)
        self.gbuf = None      # full gradient landing region
        self.ready = 0
        self.launched = False
        self.unit = False
        self.gather_event = None
        self.module = None
        self.pending_release = False
        self.hold = False     # stage 3: kept gathered from its forward until its own backward reduced
        self.first_use = 0    # forward position of the first unit that reads this segment

    def view(self, flat: torch.Tensor, i: int) -> torch.Tensor:
        shape = self.shapes[i]
        n = math.prod(shape)
        return flat[self.offsets[i]:self.offsets[i] + n].view(shape)


def _split_buckets(params, cap_elems: int):
    buckets, cur, size = [], [], 0
    for p in params:
        n = -(-p.numel() // ALIGN) * ALIGN
        if cur and size + n > cap_elems:
            buckets.append(cur)
            cur, size = [], 0
        cur.append(p)
        size += n
    if cur:
        buckets.append(cur)
    return buckets


class _WorkFence:
    """A collective still in flight, used where the eager path records a HIP event on the comm
    stream: a landing region's release fence, a ZeRO-3 unit's gather fence.  Inside a hipGraph
    capture the collectives are issued on the capturing stream (a collective issued on a side
    stream forked from the capture crashes hipStreamEndCapture: RCCL's internal stream then forks
    from a non-origin stream -- scripts/diag/capture_collectives.py, profiles/r5_capture_results.jsonl)
    and their ``Work.wait()`` -- the capturing stream waiting for the collective's end -- is
    deferred to the first reader of the bytes: in the graph each collective is a branch parallel
    to the backward / forward work issued after it."""

    __slots__ = ("work",)

    def __init__(self, work):
        self.work = work


def _fence_wait(fence, stream=None) -> None:
    """Make the current stream (``stream``) wait for a HIP event or a pending collective."""
    if fence is None:
        return
    if isinstance(fence, _WorkFence):
        fence.work.wait()           # ProcessGroupNCCL: the current stream waits for the end event
    else:
        (stream or torch.cuda.current_stream()).wait_event(fence)


class _Arena:
    """Ring sub-allocator over ONE persistent buffer (ZeRO-2/3 gradient landing regions and
    ZeRO-3 gathered-parameter regions).

    ``acquire(n, key)`` returns a region at the ring head (wrapping to 0 when it does not fit),
    skipping past regions still live; ``release(t, event)`` hands a region back together with
    the event after which it may be overwritten, and the next acquirer of overlapping bytes makes
    its stream wait for that event.  Requests larger than half the arena get a dedicated
    persistent buffer per ``key`` (a BLOOM word-embedding gradient), and a request that finds no
    free range falls back to the caching allocator.  The sequence of requests is the same every
    step, so after the first step the addresses are too: nothing is allocated per step and the
    step can be captured in a hipGraph.  ``new_window()`` drops the previous step's events
    (callers order the new step behind the old one with a stream wait)."""

    def __init__(self, numel: int, dtype, device):
        self.numel = max(int(numel), 0)
        self.dtype, self.device = dtype, device
        self.buf = torch.empty(self.numel, dtype=dtype, device=device) if self.numel else None
        self.head = 0
        self.live = {}       # start -> end of regions handed out and not released
        self.done = []       # (start, end, event or None) released regions
        self.dedicated = {}  # key -> [tensor, event, live]
        self.heap_fallbacks = 0

    def _base(self) -> int:
        return self.buf.data_ptr() if self.buf is not None else 0

    def new_window(self) -> None:
        self.done = [(a, b, None) for a, b, _ in self.done]
        for d in self.dedicated.values():
            d[1] = None

    def acquire(self, n: int, key, waiter=None) -> torch.Tensor:
        """A region of ``n`` elements; ``waiter(event)`` is called for every release event that
        guards the returned bytes (the caller makes its stream wait)."""
        if n > self.numel // 2:
            d = self.dedicated.get(key)
            if d is None:
                d = self.dedicated[key] = [torch.empty(n, dtype=self.dtype, device=self.device), None, False]
            if d[1] is not None and waiter is not None:
                waiter(d[1])
            d[1], d[2] = None, True
            return d[0]
        a = self.head if self.head + n <= self.numel else 0
        for _ in range(len(self.live) + 2):
            hit = [e for st, e in self.live.items() if st < a + n and a < e]
            if not hit:
                break
            a = max(hit)
            if a + n > self.numel:
                a = 0
        else:
            hit = True
        if hit or a + n > self.numel:
            self.heap_fallbacks += 1
            return torch.empty(n, dtype=self.dtype, device=self.device)
        keep = []
        for st, e, ev in self.done:
            if st < a + n and a < e:
                if ev is not None and waiter is not None:
                    waiter(ev)
            else:
                keep.append((st, e, ev))
        self.done = keep
        self.live[a] = a + n
        self.head = a + n
        return self.buf[a:a + n]

    def drop_work_fences(self) -> None:
        """Forget the pending-collective fences (a captured step joined them all on the capturing
        stream, so later acquirers on that stream are already ordered behind them); no RCCL Work
        object may outlive the capture that created it (one freed after its process group is
        destroyed crashed the next test's replay)."""
        self.done = [(a, b, None if isinstance(ev, _WorkFence) else ev) for a, b, ev in self.done]
        for d in self.dedicated.values():
            if isinstance(d[1], _WorkFence):
                d[1] = None

    def release(self, t: torch.Tensor, event=None, stream=None) -> None:
        for d in self.dedicated.values():
            if d[0].data_ptr() == t.data_ptr() and d[2]:
                d[1], d[2] = event, False
                return
        if self.buf is not None:
            es = t.element_size()
            a = (t.data_ptr() - self._base()) // es
            if 0 <= a < self.numel and a in self.live:
                self.done.append((a, self.live.pop(a), event))
                return
        if stream is not None and t.is_cuda:   # a caching-allocator fallback region
            t.record_stream(stream)


class ZeroEngine(nn.Module):
    def __init__(self, model: nn.Module, config: dict | None = None, model_parameters=None, process_group=None):
        super().__init__()
        self.module = model
        self.config = ZeroConfig(config)
        if not dist.is_initialized():
            comm.init()
        self.group = process_group
        self.world = dist.get_world_size(process_group)
        self.rank = dist.get_rank(process_group)
        self.backend = dist.get_backend(process_group)
        clog.comms_logger.configure(self.config.comms_logger)
        self.stage = self.config.stage
        params = unique_params(model_parameters if model_parameters is not None else model.parameters())
        p0 = params[0]
        self.device, self.dtype = p0.device, p0.dtype
        self.grad_dtype = p0.dtype
        self.cuda = self.device.type == "cuda"
        self.comm_stream = torch.cuda.Stream(self.device) if self.cuda else None
        # stage 3 gathers: their own stream AND their own communicator (one RCCL stream per
        # process group), so a prefetch gather does not queue behind a reduce-scatter
        self.gather_stream = torch.cuda.Stream(self.device) if (self.cuda and self.stage == 3) else None
        self.gather_group = process_group
        if self.stage == 3 and self.world > 1 and self.config.gather_communicator:
            ranks = dist.get_process_group_ranks(process_group) if process_group is not None \
                else list(range(self.world))
            self.gather_group = dist.new_group(ranks=ranks)
        self.shard_world = 1 if self.stage == 0 else self.world
        self.shard_rank = 0 if self.stage == 0 else self.rank
        # replicated layout (stage 0's): the stage-0 engine, and stages 1/2 on ONE rank, where the
        # partition is the whole buffer -- reduce-scatter and all-gather are identities, so the
        # gradient / parameter "shards" alias the flat buffers instead of being copied each step.
        # `zero_optimization.world1_replicated: false` keeps the partitioned code path at world 1
        # (bench.py does, so the 1-GPU bench runs the N > 1 data flow).
        self.replicated = self.stage == 0 or (self.world == 1 and self.stage in (1, 2)
                                              and self.config.world1_replicated)
        # stage 3 on one rank: a unit's "gathered" parameters and its gradient landing region are
        # views of its (whole) shard, so nothing is copied per use (one micro-batch per step)
        self.alias_units = (self.stage == 3 and self.world == 1 and self.config.world1_replicated
                            and self.config.gas == 1)
        # collectives run with a peer, or always when forced (world-1 rehearsal of the RCCL path)
        self.collect = self.world > 1 or self.config.force_collectives
        if self.collect and self.world == 1:
            # the partitioned data flow (stage 0 keeps its all-reduce), so the reduce-scatters and
            # all-gathers of stages 1-3 actually run
            self.replicated = self.stage == 0
            self.alias_units = False
        self.micro_step = 0
        self.global_steps = 0
        self._callback_queued = False
        self._need_reset = True
        self._refresh_events = {}   # segment index -> event of its last refresh all-gather
        self._cap_pending = []      # _WorkFence of collectives issued inside a capture, not yet joined
        # DTD_ZERO_CAPTURE_DEFER=0: inside a capture every collective is waited where it is issued
        self._defer_capture = os.environ.get("DTD_ZERO_CAPTURE_DEFER", "1") == "1"
        self._refresh_waits = {}    # id(module) -> segment indices its forward reads

        # ---- partition parameters into persistent buckets and (stage 3) units
        units, persistent = [], params
        if self.stage == 3:
            units, persistent = self._plan_units(model, params)
        cap = self.config.reduce_bucket if self.stage > 0 else self.config.allreduce_bucket
        order = list(reversed(persistent))  # ~ gradient-ready order
        self.buckets = [_Segment(i, b, self.shard_world) for i, b in enumerate(_split_buckets(order, max(cap, ALIGN)))]
        self.units = []
        for i, (mod, ps) in enumerate(units):
            s = _Segment(len(self.buckets) + i, ps, self.world)
            s.unit, s.module = True, mod
            self.units.append(s)
        self.segments = self.buckets + self.units
        off = 0
        for s in self.segments:
            s.shard_off = off
            off += s.chunk
        self.shard_numel = off
        self._seg_of = {}
        self._pindex = {}
        bucket_of = []
        for s in self.segments:
            for i, p in enumerate(s.params):
                self._seg_of[id(p)] = (s, i)
                self._pindex[id(p)] = len(bucket_of)
                bucket_of.append(s.index)
        # native readiness tracker (runtime/csrc/reducer.cpp): expected-contribution counts per
        # parameter, segment completeness, in-order launch of the reduce buckets; stage-3 units
        # reduce as soon as they are complete
        self.tracker = ReadyTracker(bucket_of, len(self.segments), ordered=[not s.unit for s in self.segments])

        self._broadcast_initial(params)
        self._build_storage()
        self._install_grad_hooks()
        self._plan_refresh(model)
        if self.stage == 3:
            self._install_unit_hooks()
        self.optimizer = self._build_optimizer()
        self.overlap_opt = self.config.overlap_opt
        self._opt_stream = torch.cuda.Stream(self.device) if self.cuda else None
        self._opt_started = False    # this step's update began during the backward
        self._opt_pending = []       # segments reduced, their update not launched yet
        self._opt_done = set()       # segment indices updated this step

    # ================================================================== planning
    def _plan_units(self, model, params):
        mods = model.zero3_units() if hasattr(model, "zero3_units") else list(model.children())
        shared = {id(p) for p in (model.zero3_persistent() if hasattr(model, "zero3_persistent") else [])}
        owner, units = {}, []
        for m in mods:
            ps = [p for p in unique_params(m.parameters()) if id(p) not in shared]
            for p in ps:
                owner.setdefault(id(p), []).append(m)
        multi = {k for k, v in owner.items() if len(v) > 1}
        shared |= multi
        placed = set()
        for m in mods:
            ps = [p for p in unique_params(m.parameters()) if id(p) not in shared and id(p) not in placed]
            placed.update(id(p) for p in ps)
            if ps:
                units.append((m, ps))
        persistent = [p for p in params if id(p) not in placed]
        return units, persistent

    def _plan_refresh(self, model) -> None:
        """Forward order of the replicated buckets and the per-unit waits of the overlapped
        parameter refresh (stages >= 1).  A bucket's forward position is that of the first unit
        (``model.zero3_units()``, forward order) reading one of its parameters; buckets no unit
        reads are waited for before the forward starts."""
        mods = list(model.zero3_units()) if hasattr(model, "zero3_units") else []
        first = {}
        for k, m in enumerate(mods):
            seen = set()
            for p in m.parameters():
                hit = self._seg_of.get(id(p))
                if hit is None or hit[0].unit:
                    continue
                s = hit[0]
                first.setdefault(s.index, k)
                seen.add(s.index)
            if seen:
                self._refresh_waits[id(m)] = sorted(seen)
        for s in self.buckets:
            s.first_use = first.get(s.index, -1)
        # forward order; ties (and buckets no unit reads, first_use -1, first) by reverse bucket
        # order = registration order
        fwd = sorted(self.buckets, key=lambda s: (s.first_use, -s.index))
        cap = self.config.allgather_bucket
        self._refresh_groups, cur, size = [], [], 0
        for s in fwd:
            if cur and size + s.numel > cap:
                self._refresh_groups.append(cur)
                cur, size = [], 0
            cur.append(s)
            size += s.numel
        if cur:
            self._refresh_groups.append(cur)
        self._overlap_refresh = (self.config.overlap_refresh and self.cuda and self.stage >= 1 and bool(mods))
        if self._overlap_refresh:
            for m in mods:
                if id(m) in self._refresh_waits:
                    m.register_forward_pre_hook(self._make_refresh_wait(self._refresh_waits[id(m)]))

    def _make_refresh_wait(self, idx):
        def hook(mod, args):
            self._wait_refresh(idx)
        return hook

    def _wait_refresh(self, idx=None) -> None:
        """Make the compute stream wait for the refresh all-gathers of segments ``idx`` (all when
        None).  Each event is waited for once."""
        if not self._refresh_events:
            return
        cur = torch.cuda.current_stream(self.device)
        for k in (list(self._refresh_events) if idx is None else idx):
            ev = self._refresh_events.pop(k, None)
            if ev is not None:
                cur.wait_event(ev)

    @torch.no_grad()
    def _broadcast_initial(self, params) -> None:
        """C6: every rank starts from rank 0's weights -- one broadcast per <= 256 MiB flat chunk
        of each dtype (DDP's 250 MiB coalescing), not one per parameter."""
        if self.world <= 1:
            return
        by_dtype = {}
        for p in params:
            by_dtype.setdefault(p.dtype, []).append(p)
        for dt, ps in by_dtype.items():
            es = torch.empty(0, dtype=dt).element_size()
            cap = max(1, (256 << 20) // es)
            chunk, n = [], 0
            for p in ps + [None]:
                if p is None or (chunk and n + p.numel() > cap):
                    flat = torch.cat([q.data.reshape(-1) for q in chunk])
                    clog.broadcast(flat, src=0, group=self.group)
                    off = 0
                    for q in chunk:
                        q.data.copy_(flat[off:off + q.numel()].view_as(q))
                        off += q.numel()
                    chunk, n = [], 0
                if p is not None:
                    chunk.append(p)
                    n += p.numel()

    # ================================================================== storage
    @torch.no_grad()
    def _build_storage(self) -> None:
        dev, dt = self.device, self.dtype
        P = self.shard_numel
        self.master = torch.zeros(P, dtype=torch.float32, device=dev)
        self.lowp = torch.zeros(P, dtype=dt, device=dev) if dt != torch.float32 else None
        self.gshard = torch.zeros(P, dtype=self.grad_dtype, device=dev)
        self._gtmp = None
        # persistent buckets: one flat replicated param buffer
        total = sum(s.numel for s in self.buckets)
        self.param_flat = torch.zeros(total, dtype=dt, device=dev)
        off = 0
        for s in self.buckets:
            s.full = self.param_flat[off:off + s.numel]
            for i, p in enumerate(s.params):
                v = s.view(s.full, i)
                v.copy_(p.data)
                p.data = v
            off += s.numel
        self.grad_flat = None
        if self.stage <= 1 or self.replicated:
            self.grad_flat = torch.zeros(total, dtype=self.grad_dtype, device=dev)
            off = 0
            for s in self.buckets:
                s.gbuf = self.grad_flat[off:off + s.numel]
                for i, p in enumerate(s.params):
                    p.main_grad = s.view(s.gbuf, i)
                off += s.numel
        # ring arenas: gradient landing regions (stages 2/3) and gathered units (stage 3)
        # (aliased stage-3 segments land in their own shard and gather nothing: no arena for them).
        # The landing arena never exceeds the regions it can hold at once -- the whole gradient
        # -- so a large reduce_bucket_size on a small model does not pin more than that.
        reg = [s.numel for s in self.segments
               if not self.alias_units and (s.unit or (self.stage >= 2 and not self.replicated))]
        big_unit = 0 if self.alias_units else max([s.numel for s in self.units], default=0)
        want = max(4 * max(self.config.reduce_bucket, ALIGN), 3 * big_unit)
        self.landing = _Arena(min(want, sum(reg)) if reg else 0, self.grad_dtype, dev)
        self.gather_arena = _Arena(max(self.config.prefetch_bucket + 2 * big_unit, 4 * big_unit)
                                   if self.units and not self.alias_units else 0, dt, dev)
        # master shard: chunk `shard_rank` of every segment
        for s in self.buckets:
            lo = self.shard_rank * s.chunk
            self.master[s.shard_off:s.shard_off + s.chunk].copy_(s.full[lo:lo + s.chunk])
            if self.lowp is not None:
                self.lowp[s.shard_off:s.shard_off + s.chunk].copy_(s.full[lo:lo + s.chunk])
        for s in self.units:
            full = torch.zeros(s.numel, dtype=dt, device=dev)
            for i, p in enumerate(s.params):
                s.view(full, i).copy_(p.data)
            lo = self.rank * s.chunk
            self.master[s.shard_off:s.shard_off + s.chunk].copy_(full[lo:lo + s.chunk])
            if self.lowp is not None:
                self.lowp[s.shard_off:s.shard_off + s.chunk].copy_(full[lo:lo + s.chunk])
            for p in s.params:
                p.data = torch.empty(0, dtype=self.dtype, device=self.device)
        if self.replicated:
            # replicated optimizer: the shard IS the whole flat buffer -- alias instead of copying
            self.gshard = self.grad_flat
            if self.lowp is not None:
                self.lowp = self.param_flat
            else:
                self.master = self.param_flat
        if self.lowp is None:  # fp32 model: the master shard is the parameter shard
            self.lowp_view = self.master
        else:
            self.lowp_view = self.lowp
        if self.alias_units:
            # one rank, stage 3: the persistent buckets alias their (whole) shard as the units do, so
            # their gradients land in place and the refresh copies nothing.  bloom-560m's tied
            # 257 M-parameter embedding paid a landing copy + a refresh copy, 0.4 ms of a 12.4 ms
            # step (profiles/r6_bloom_z3_b1_kernels.txt)
            for s in self.buckets:
                s.full = self.lowp_view[s.shard_off:s.shard_off + s.numel]
                for i, p in enumerate(s.params):
                    p.data = s.view(s.full, i)
            self.param_flat = torch.empty(0, dtype=dt, device=dev)

    def _set_released(self, s: _Segment) -> None:
        for p in s.params:
            p.data = torch.empty(0, dtype=self.dtype, device=self.device)
        s.full = None

    def _build_optimizer(self) -> FusedAdam:
        op = dict(self.config.opt_params)
        t = self.config.opt_type.lower()
        kw = dict(lr=float(op.get("lr", 1e-3)), betas=tuple(op.get("betas", (0.9, 0.999))),
                  eps=float(op.get("eps", 1e-8)), weight_decay=float(op.get("weight_decay", 0.0)),
                  adam_w_mode=(t in ("adamw",) or bool(op.get("adam_w_mode", True))),
                  bias_correction=bool(op.get("bias_correction", True)))
        if self.config.clip > 0:
            kw["max_grad_norm"] = self.config.clip
        opt = FusedAdam.from_flat(self.master, self.gshard, self.lowp, **kw)
        if self.stage > 0 and self.world > 1:
            def _red(sq):
                clog.all_reduce(sq, op=dist.ReduceOp.SUM, group=self.group)
                return sq
            opt._reduce_sqnorm = _red
        return opt

    # ================================================================== gradient flow
    def _install_grad_hooks(self) -> None:
        self._hooks = []
        for s in self.segments:
            for p in s.params:
                p._dtd_ready_hook = self._on_ready
                p._dtd_expect = self._expect
                p._dtd_touched = False
                p._dtd_pending = 0
                if (self.stage >= 2 and not self.replicated) or s.unit:
                    p._dtd_pre_write_hook = self._pre_write
                self._hooks.append(p.register_post_accumulate_grad_hook(self._from_autograd))

    def _from_autograd(self, p) -> None:
        g = p.grad
        if g is None:
            return
        dst_pre = getattr(p, "_dtd_pre_write_hook", None)
        if dst_pre is not None:
            dst_pre(p)
        if p._dtd_touched:
            p.main_grad.add_(g.to(p.main_grad.dtype))
        else:
            p.main_grad.copy_(g)
        p.grad = None
        p._dtd_touched = True
        self._on_ready(p, autograd=True)

    def _pre_write(self, p) -> None:
        s, _ = self._seg_of[id(p)]
        if s.gbuf is None:
            self._alloc_landing(s)

    def _alloc_landing(self, s: _Segment) -> None:
        if self.alias_units:   # the segment's gradient shard itself (padding stays zero)
            s.gbuf = self.gshard[s.shard_off:s.shard_off + s.numel]
            for i, p in enumerate(s.params):
                p.main_grad = s.view(s.gbuf, i)
                p._dtd_touched = False
            return
        cur = torch.cuda.current_stream(self.device) if self.cuda else None
        s.gbuf = self.landing.acquire(s.numel, s.index,
                                      waiter=(lambda f: _fence_wait(f, cur)) if cur is not None else None)
        # padding (alignment gaps, segment tail) must reduce as zeros: the region is recycled.  Only
        # the padding is cleared (one index_fill_ launch): every parameter's own range is written
        # in full by its first contribution (grad_dst: accumulate=False) or zeroed in
        # _reduce_segment when the parameter got no gradient
        pad = self._pad_index(s)
        if pad is not None:
            s.gbuf.index_fill_(0, pad, 0)
        for i, p in enumerate(s.params):
            p.main_grad = s.view(s.gbuf, i)
            p._dtd_touched = False

    def _pad_index(self, s: _Segment):
        """Positions of segment ``s`` outside every parameter (alignment gaps and the tail),
        cached on the device; None when there are none."""
        cache = self.__dict__.setdefault("_pads", {})
        if s.index not in cache:
            idx, off = [], 0
            for i, shape in enumerate(s.shapes):
                n = math.prod(shape)
                end = s.offsets[i + 1] if i + 1 < len(s.shapes) else s.numel
                idx.extend(range(s.offsets[i] + n, end))
            cache[s.index] = torch.tensor(idx, dtype=torch.long, device=self.device) if idx else None
        return cache[s.index]

    def _expect(self, p) -> None:
        self.tracker.expect(self._pindex[id(p)])

    def _on_ready(self, p, autograd: bool = False) -> None:
        if not self._callback_queued:
            self._callback_queued = True
            torch.autograd.Variable._execution_engine.queue_callback(self._end_of_backward)
        full = self.stage <= 1 or self.replicated   # one full gradient buffer, reduced once per step
        allow = self.config.overlap and not (full and not self.is_gradient_accumulation_boundary())
        _, launch = self.tracker.contribute(self._pindex[id(p)], autograd, allow_launch=allow)
        for k in launch:
            s = self.segments[k]
            if s.unit:
                self._reduce_unit(s)
            elif not s.launched:
                self._reduce_segment(s)

    def _capturing(self) -> bool:
        return self.cuda and torch.cuda.is_current_stream_capturing()

    def _cs(self):
        """The comm stream, or None while a hipGraph capture is in progress: a collective issued on
        a side stream joined to the capture crashed hipStreamEndCapture on the box (RCCL
        reduce-scatter, scripts/diag/capture_collectives.py side_stream_rs) while the same
        collective on the capturing stream itself captures and replays -- inside a graph the
        collectives run on the capture stream (RCCL still launches them on its own stream)."""
        return None if self._capturing() else self.comm_stream

    def _comm_ctx(self, stream=None):
        stream = stream if stream is not None else self.comm_stream
        if stream is None or self._capturing():
            return contextlib.nullcontext()
        stream.wait_stream(torch.cuda.current_stream(self.device))
        return torch.cuda.stream(stream)

    def _reduce_segment(self, s: _Segment) -> None:
        """Reduce one segment's gradients: all-reduce (stage 0) or reduce-scatter into the
        local gradient shard (stages 1-3); stage 2/3 landing regions go back to the arena."""
        flush_finalizes()   # queued bias / LayerNorm finalizes may write into this segment
        s.launched = True
        if s.gbuf is None:   # no parameter of this segment got a gradient yet: land it now
            self._alloc_landing(s)
        for p in s.params:  # parameters without a gradient this step contribute zeros (the
            if not p._dtd_touched:   # recycled landing region holds an earlier segment's bytes)
                p.main_grad.zero_()
        buf = s.gbuf
        # stages 0/1 accumulate micro-batches in the full gradient buffer and reduce once;
        # stages 2/3 reduce every micro-batch and accumulate the shards
        first = self.micro_step == 0 or self.stage <= 1 or self.replicated
        out = self.gshard[s.shard_off:s.shard_off + s.chunk]
        # inside a capture an RCCL collective is left in flight (its wait deferred to the readers:
        # the landing region's next acquirer, the end of the backward); what reads the result right
        # away (gloo's division, the accumulation add) waits here
        defer = self._defer_capture and self._capturing() and self.backend == "nccl"
        fence = None
        with self._comm_ctx():
            if self.replicated:  # buf aliases the gradient "shard" (the full buffer)
                if self.collect:
                    op = dist.ReduceOp.AVG if self.backend == "nccl" else dist.ReduceOp.SUM
                    w = clog.all_reduce(buf, op=op, group=self.group, async_op=True)
                    if defer:
                        fence = _WorkFence(w)
                    else:
                        w.wait()
                    if self.backend != "nccl":
                        buf.div_(self.world)
            else:
                dst = out if first else self._tmp()[s.shard_off:s.shard_off + s.chunk]
                if self.collect:
                    op = dist.ReduceOp.AVG if self.backend == "nccl" else dist.ReduceOp.SUM
                    w = clog.reduce_scatter_tensor(dst, buf, op=op, group=self.group, async_op=True)
                    if defer and first:
                        fence = _WorkFence(w)
                    else:
                        w.wait()
                    if self.backend != "nccl":
                        dst.div_(self.world)
                elif dst.data_ptr() != buf.data_ptr():   # aliased stage-3 segment: already in place
                    dst.copy_(buf)
                if not first:
                    out.add_(dst)
            ev = None
            landed = (self.stage >= 2 and not self.replicated) or s.unit
            cs = self._cs()
            if fence is not None:
                self._cap_pending.append(fence)
                ev = fence
            elif cs is not None and landed:
                ev = torch.cuda.Event()
                ev.record(cs)
        if landed:
            if not self.alias_units:
                self.landing.release(buf, ev, cs)
            s.gbuf = None
            for p in s.params:
                p.main_grad = None
        self._opt_after_reduce(s)

    # ================================================================== optimizer under the backward
    def _opt_overlap_active(self) -> bool:
        return (self.overlap_opt and self.cuda and self.optimizer.max_grad_norm is None
                and self.optimizer._chunks is None and not self._capturing()
                and self.is_gradient_accumulation_boundary())

    def _opt_after_reduce(self, s: _Segment) -> None:
        """Segment ``s`` holds its final gradient shard.  Its Adam update is launched at the NEXT
        segment's reduce (or in ``step``), not now: the backward call that reported the segment's
        last gradient may still read its weights (a layer emits its weight gradient before its
        input-gradient GEMM), and with the world-1 aliases the update writes those weights.  By the
        next reduce -- the next unit's backward, in reverse layer order -- everything that reads
        them has been enqueued, so the side stream's update runs beside the rest of the backward."""
        if not hasattr(self, "_opt_stream") or not self._opt_overlap_active():
            return
        if not self._opt_started:
            self.optimizer.begin_ranged_step()
            self._opt_started = True
        self._opt_launch(self._opt_pending)
        self._opt_pending = [s]

    def _opt_launch(self, segs) -> None:
        segs = [s for s in segs if s.index not in self._opt_done]
        if not segs:
            return
        side = self._opt_stream
        side.wait_stream(torch.cuda.current_stream(self.device))   # grads written, weights read
        if self.comm_stream is not None:
            side.wait_stream(self.comm_stream)                     # reduce-scatters landed
        for s in segs:
            self.optimizer.step_range(s.shard_off, s.shard_off + s.chunk, side)
            self._opt_done.add(s.index)

    def _opt_finish(self) -> None:
        """step(): update every segment not yet updated and join the side stream."""
        self._opt_launch(self.segments)
        torch.cuda.current_stream(self.device).wait_stream(self._opt_stream)
        self._opt_started = False
        self._opt_pending = []
        self._opt_done = set()

    def _tmp(self) -> torch.Tensor:
        if self._gtmp is None:
            self._gtmp = torch.zeros_like(self.gshard)
        return self._gtmp

    def _end_of_backward(self) -> None:
        self._callback_queued = False
        flush_finalizes()
        if (self.stage <= 1 or self.replicated) and not self.is_gradient_accumulation_boundary():
            return
        for s in self.buckets:
            if not s.launched:
                self._reduce_segment(s)
        for s in self.units:
            if not s.launched:
                self._reduce_unit(s)
        self._release_pending()
        self._join_captured()
        if self._cs() is not None:
            torch.cuda.current_stream(self.device).wait_stream(self.comm_stream)

    def _join_captured(self) -> None:
        """Join every collective a capture left in flight (the optimizer reads the shards next)."""
        if not self._cap_pending:
            return
        for f in self._cap_pending:
            f.work.wait()
        self._cap_pending.clear()
        self.landing.drop_work_fences()
        for u in self.units:
            if isinstance(u.gather_event, _WorkFence):
                u.gather_event = None

    # ================================================================== stage 3 units
    def _install_unit_hooks(self) -> None:
        for k, s in enumerate(self.units):
            s.module.register_forward_pre_hook(self._make_pre_fwd(k))
            s.module.register_forward_hook(self._make_post_fwd(k))

    def _gather(self, s: _Segment) -> None:
        if s.full is not None:
            return
        if self.alias_units:   # one rank: the shard is the whole unit
            s.full = self.lowp_view[s.shard_off:s.shard_off + s.numel]
            for i, p in enumerate(s.params):
                p.data = s.view(s.full, i)
            return
        full = self.gather_arena.acquire(s.numel, s.index)
        src = self.lowp_view[s.shard_off:s.shard_off + s.chunk]
        with self._comm_ctx(self.gather_stream):   # the stream wait orders it behind earlier reads
            if self.collect:
                w = clog.all_gather_into_tensor(full, src, group=self.gather_group, async_op=True)
                if self._defer_capture and self._capturing() and self.backend == "nccl":
                    s.gather_event = _WorkFence(w)     # waited by the unit's first reader (_ensure)
                    self._cap_pending.append(s.gather_event)
                else:
                    w.wait()
            else:
                full.copy_(src)
            if self.gather_stream is not None and not self._capturing():
                ev = torch.cuda.Event()
                ev.record(self.gather_stream)
                s.gather_event = ev
        s.full = full
        for i, p in enumerate(s.params):
            p.data = s.view(full, i)

    def _ensure(self, s: _Segment) -> None:
        self._gather(s)
        if s.gather_event is not None:
            _fence_wait(s.gather_event, torch.cuda.current_stream(self.device))
            s.gather_event = None

    def _release(self, s: _Segment) -> None:
        if s.full is None:
            return
        if s.gather_event is not None:   # gathered (prefetched) but never used: still order it
            _fence_wait(s.gather_event, torch.cuda.current_stream(self.device))
            s.gather_event = None
        if not self.alias_units:
            if self.config.poison_released and s.full.is_floating_point():
                s.full.fill_(float("nan"))
            self.gather_arena.release(s.full, None,
                                      torch.cuda.current_stream(self.device) if self.cuda else None)
        self._set_released(s)

    def _prefetch(self, order) -> None:
        """Gather the units of ``order`` (the next ones to run) while the elements gathered
        ahead stay within ``stage3_prefetch_bucket_size`` -- at least one unit ahead."""
        ahead = 0
        for j, u in enumerate(order):
            if j > 0 and ahead + u.numel > self.config.prefetch_bucket:
                break
            if u.full is None:
                self._gather(u)
            ahead += u.numel

    def _make_pre_fwd(self, k: int):
        def hook(mod, args):
            if self._need_reset:
                self._reset()
            self._ensure(self.units[k])
            self._prefetch(self.units[k + 1:])
        return hook

    def _make_post_fwd(self, k: int):
        def hook(mod, args, out):
            s = self.units[k]
            if torch.is_grad_enabled() and self.module.training:
                t = out if torch.is_tensor(out) else None
                if t is not None and t.requires_grad:
                    t.register_hook(self._make_bwd_start(k))
                if not getattr(mod, "_dtd_weightless_bwd", False):
                    # plain autograd ops saved VIEWS of the gathered weights for the backward
                    # (F.linear keeps weight.t()); those views do not follow a re-gather, and the
                    # arena would hand their bytes to the next unit.  Keep the unit gathered until
                    # its own backward has reduced (pending release).  The fused modules' backward
                    # re-reads the parameters themselves and declares _dtd_weightless_bwd.
                    s.hold = True
                    return
            self._release(s)
        return hook

    def _make_bwd_start(self, k: int):
        def hook(grad):
            s = self.units[k]
            self._release_pending(keep=(s,))
            self._ensure(s)
            if s.gbuf is None:
                self._alloc_landing(s)
            self._prefetch(self.units[:k][::-1])
            return grad
        return hook

    def _reduce_unit(self, s: _Segment) -> None:
        """Reduce-scatter a unit's gradients as soon as they are complete.  The gathered
        parameters are released LATER (next unit's backward start / end of backward): the
        backward that reported the last gradient may still read the weights for its dgrad."""
        if s.launched:
            return
        self._reduce_segment(s)
        s.pending_release = True
        s.hold = False

    def _release_pending(self, keep=()) -> None:
        for u in self.units:
            if u.pending_release and not u.hold and u not in keep:
                u.pending_release = False
                self._release(u)

    # ================================================================== engine API
    def _reset(self) -> None:
        accumulate_full = (self.stage <= 1 or self.replicated) and self.micro_step > 0  # keep accumulating in place
        self.tracker.reset()
        # a unit kept gathered by a training forward that had no backward (hold set in its
        # post-forward hook, cleared only by its own reduce) would otherwise stay gathered into
        # this step and skip the re-gather of the updated weights
        for u in self.units:
            if u.hold or u.pending_release:
                u.hold = False
                u.pending_release = False
                self._release(u)
        self.landing.new_window()
        self.gather_arena.new_window()
        for s in self.segments:
            s.launched = False
            for p in s.params:
                if not accumulate_full:
                    p._dtd_touched = False
                p._dtd_pending = 0
                p.grad = None
        self._need_reset = False

    def forward(self, *args, **kwargs):
        if self._need_reset:
            self._reset()
        if self._refresh_events and self.cuda and torch.cuda.is_current_stream_capturing():
            self._refresh_events.clear()   # recorded before the capture (which starts synchronised)
        if self._refresh_events:
            # buckets no unit reads (and every bucket when the model has no units) first; the
            # units' pre-hooks wait for their own buckets while the later refreshes land
            self._wait_refresh([s.index for s in self.buckets if s.first_use < 0])
        out = self.module(*args, **kwargs)
        self._wait_refresh()   # the backward reads every weight
        return out

    def backward(self, loss: torch.Tensor) -> None:
        if self.config.gas > 1:
            loss = loss / self.config.gas
        loss.backward()

    def is_gradient_accumulation_boundary(self) -> bool:
        return (self.micro_step + 1) % self.config.gas == 0

    def step(self) -> None:
        if not self.is_gradient_accumulation_boundary():
            self.micro_step += 1
            self._need_reset = True
            return
        self._join_captured()
        if self._cs() is not None:
            torch.cuda.current_stream(self.device).wait_stream(self.comm_stream)
        if self._opt_started:
            self._opt_finish()
        else:
            self.optimizer.step()
        self._refresh_params()
        self.micro_step = 0
        self.global_steps += 1
        self._need_reset = True
        rt = getattr(self.module, "rt", None)
        if rt is not None:
            rt.rng.advance()

    @torch.no_grad()
    def _refresh_params(self, wait: bool | None = None) -> None:
        """Stage 0: the kernel wrote the replicated params; stages 1-2 (and stage 3's replicated
        buckets): all-gather the updated shards into the buckets in forward order, one coalesced
        RCCL launch per ``allgather_bucket_size`` group on the comm stream.  With the overlapped
        refresh each group records an event and the next forward's unit pre-hooks wait for their
        own buckets only; otherwise the compute stream waits for everything here.  Stage 3 units
        stay sharded until their next use."""
        if self.replicated or self.alias_units:
            for s in self.buckets:
                src = self.lowp_view[s.shard_off:s.shard_off + s.chunk]
                if src.data_ptr() != s.full.data_ptr():   # aliased (the usual case): nothing to copy
                    s.full.copy_(src)
            return
        wait = (not self._overlap_refresh) if wait is None else wait
        if self.cuda and torch.cuda.is_current_stream_capturing():
            wait = True   # a captured step must join its side-stream work before it ends
        for grp in self._refresh_groups:
            with self._comm_ctx():
                outs = [s.full for s in grp]
                ins = [self.lowp_view[s.shard_off:s.shard_off + s.chunk] for s in grp]
                if self.collect:
                    w = clog.all_gather_coalesced(outs, ins, group=self.group, async_op=True)
                    w.wait()
                else:
                    for o, i in zip(outs, ins):
                        o.copy_(i)
                if self._cs() is not None and not wait:
                    ev = torch.cuda.Event()
                    ev.record(self.comm_stream)
                    for s in grp:
                        self._refresh_events[s.index] = ev
        if self._cs() is not None and wait:
            torch.cuda.current_stream(self.device).wait_stream(self.comm_stream)

    def zero_optimization_stage(self) -> int:
        return self.stage

    # ================================================================== checkpointing
    # DeepSpeed-compatible layout: <dir>/<tag>/mp_rank_00_model_states.pt holds the
    # full module state (rank 0), <dir>/<tag>/zero_pp_rank_<r>_mp_rank_00_optim_states.pt holds rank
    # r's flat shard (fp32 master, Adam moments, step), <dir>/latest names the newest tag.  Loading
    # with the same world size / stage restores the shards exactly; otherwise the parameters are
    # re-sharded from the full module state and the optimizer moments start fresh.
    def _pid_names(self) -> dict:
        names: dict = {}
        for n, p in self.module.named_parameters(remove_duplicate=False):
            names.setdefault(id(p), []).append(n)
        return names

    @torch.no_grad()
    def full_state_dict(self) -> dict:
        """Module state dict on CPU with every parameter materialised; stage 3 gathers one unit
        at a time (collective: call on every rank)."""
        self._wait_refresh()
        names = self._pid_names()
        sd = {}
        in_units = set()
        for s in self.units:
            was = s.full is not None
            self._ensure(s)
            for p in s.params:
                in_units.add(id(p))
                t = p.detach().to("cpu", copy=True)
                for n in names[id(p)]:
                    sd[n] = t
            if not was:
                self._release(s)
        for n, p in self.module.named_parameters(remove_duplicate=False):
            if id(p) not in in_units:
                sd[n] = p.detach().to("cpu", copy=True)
        for n, b in self.module.named_buffers():
            sd[n] = b.detach().to("cpu", copy=True)
        return sd

    def _ckpt_barrier(self):
        if self.world > 1:
            dist.barrier(group=self.group)

    def _shard_file(self, path: str) -> str:
        return os.path.join(path, f"zero_pp_rank_{self.shard_rank}_mp_rank_00_optim_states.pt")

    @torch.no_grad()
    def save_checkpoint(self, save_dir: str, tag=None, client_state: dict | None = None,
                        save_latest: bool = True) -> str:
        # under hipGraph replay (zero_dp_training.py --graph) the host counters stop advancing
        # after capture; the optimizer's device step count (hp[5]) is the truth for both the
        # Adam bias correction and the engine's global step
        opt_step = int(self.optimizer.state_dict()["step"])
        self.global_steps = max(self.global_steps, opt_step)
        tag = str(tag) if tag is not None else f"global_step{self.global_steps}"
        path = os.path.join(save_dir, tag)
        if self.rank == 0:
            os.makedirs(path, exist_ok=True)
        self._ckpt_barrier()
        if self.comm_stream is not None:
            torch.cuda.current_stream(self.device).wait_stream(self.comm_stream)
        opt = self.optimizer
        if self.stage > 0 or self.rank == 0:      # stage 0: the state is replicated
            torch.save({"master": self.master.detach().cpu(), "exp_avg": opt.exp_avg.detach().cpu(),
                        "exp_avg_sq": opt.exp_avg_sq.detach().cpu(), "step": opt_step,
                        "param_groups": [{k: v for k, v in g.items() if k != "params"} for g in opt.param_groups],
                        "stage": self.stage, "world": self.world, "shard_numel": self.shard_numel,
                        "global_steps": self.global_steps}, self._shard_file(path))
        full = self.full_state_dict()
        if self.rank == 0:
            rt = getattr(self.module, "rt", None)
            torch.save({"module": full, "global_steps": self.global_steps, "zero_stage": self.stage,
                        "world_size": self.world, "client_state": client_state or {},
                        "dropout_rng": rt.rng.state.detach().cpu() if rt is not None else None},
                       os.path.join(path, "mp_rank_00_model_states.pt"))
            if save_latest:
                with open(os.path.join(save_dir, "latest"), "w") as f:
                    f.write(tag)
        self._ckpt_barrier()
        return path

    @torch.no_grad()
    def load_checkpoint(self, load_dir: str, tag=None, load_optimizer_states: bool = True,
                        load_module_only: bool = False):
        """Returns (checkpoint path, client_state)."""
        if tag is None:
            with open(os.path.join(load_dir, "latest")) as f:
                tag = f.read().strip()
        path = os.path.join(load_dir, str(tag))
        ms = torch.load(os.path.join(path, "mp_rank_00_model_states.pt"), map_location="cpu", weights_only=True)
        shard_path = self._shard_file(path)
        shard = None
        if load_optimizer_states and not load_module_only and os.path.exists(shard_path):
            shard = torch.load(shard_path, map_location="cpu", weights_only=True)
            if (shard["stage"], shard["world"], shard["shard_numel"]) != (self.stage, self.world, self.shard_numel):
                shard = None                       # different layout: re-shard from the module state
        if shard is not None:
            opt = self.optimizer
            opt.load_state_dict({"step": shard["step"], "exp_avg": shard["exp_avg"], "exp_avg_sq": shard["exp_avg_sq"],
                                 "master": shard["master"], "param_groups": shard["param_groups"]})
            self._refresh_params(wait=True)
        else:
            self._load_full(ms["module"])
        self.global_steps = int(ms.get("global_steps", 0))
        rt = getattr(self.module, "rt", None)
        if rt is not None and ms.get("dropout_rng") is not None:   # dropout masks continue at the saved step;
            rt.rng.state[1:2].copy_(ms["dropout_rng"][1:2])         # each rank keeps its own seed
        self._need_reset = True
        self._ckpt_barrier()
        return path, ms.get("client_state", {})

    @torch.no_grad()
    def _load_full(self, sd: dict) -> None:
        self._wait_refresh()
        names = self._pid_names()
        for s in self.buckets:
            for p in s.params:
                p.data.copy_(sd[names[id(p)][0]])
            lo = self.shard_rank * s.chunk
            self.master[s.shard_off:s.shard_off + s.chunk].copy_(s.full[lo:lo + s.chunk])
            if self.lowp is not None and not self.replicated:
                self.lowp[s.shard_off:s.shard_off + s.chunk].copy_(s.full[lo:lo + s.chunk])
        for s in self.units:
            full = torch.zeros(s.numel, dtype=self.dtype, device=self.device)
            for i, p in enumerate(s.params):
                s.view(full, i).copy_(sd[names[id(p)][0]])
            lo = self.rank * s.chunk
            self.master[s.shard_off:s.shard_off + s.chunk].copy_(full[lo:lo + s.chunk])
            if self.lowp is not None:
                self.lowp[s.shard_off:s.shard_off + s.chunk].copy_(full[lo:lo + s.chunk])
            if s.full is not None:
                s.full.copy_(full)
        for n, b in self.module.named_buffers():
            if n in sd:
                b.copy_(sd[n])
        opt = self.optimizer
        opt.exp_avg.zero_()
        opt.exp_avg_sq.zero_()
        opt.step_count = 0
        opt.hp[5] = 0.0

    def train(self, mode: bool = True):
        self.module.train(mode)
        return self

    def eval(self):
        return self.train(False)

    # ------------------------------------------------------------------ introspection
    def partition_numel(self) -> int:
        return self.shard_numel

    def state_bytes_per_rank(self) -> dict:
        es = self.dtype.itemsize if hasattr(self.dtype, "itemsize") else torch.empty(0, dtype=self.dtype).element_size()
        out = {"master_fp32": self.master.numel() * 4, "adam_moments": 2 * self.master.numel() * 4,
               "grad_shard": self.gshard.numel() * self.gshard.element_size(),
               "replicated_params": self.param_flat.numel() * es}
        if self.grad_flat is not None:
            out["full_grads"] = self.grad_flat.numel() * self.grad_flat.element_size()
        return out


def initialize(model: nn.Module, model_parameters=None, config: dict | None = None, optimizer=None, **_):
    """DeepSpeed-compatible entry point: returns (engine, optimizer, None, None)."""
    if optimizer is not None:
        raise NotImplementedError("pass the optimizer through the config dict (type Adam/AdamW)")
    engine = ZeroEngine(model, config, model_parameters)
    return engine, engine.optimizer, None, None
