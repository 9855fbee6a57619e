"""Pipeline parallelism with one stage per process (one rank per GPU).

Reference: ``BertModelWithMP`` places contiguous module groups on the GPUs of ONE process and
``to_pipeline(chunks)`` wraps them in torch's GPipe ``Pipe`` (/root/reference/model/bert_mp.py:39-47,
73-99; /root/reference/model_parallel_training.py:43-44,65-78).  The single-process form stays
(``parallel/pipeline.py``, the reference's behaviour); this module is the MI355X-native
multi-process form: rank ``s`` of an ``S``-rank group owns stage ``s`` (the same ``np.array_split``
module groups), activations travel forward and their gradients backward as point-to-point
messages (RCCL send/recv over xGMI on GPUs; staged through host memory on gloo), and every rank
issues only its own stage's kernels -- no host thread drives several GPUs, so the step is not
host-issue-bound, and each rank's step is a fixed kernel + message sequence that can be
captured as one hipGraph per stage (``utils/graphs.CapturedStep`` around ``train_step`` + the
optimizer: ``model_parallel_training.py --graph on`` under torchrun with RCCL; gloo stages
messages through host memory and is not capturable).

Schedules (``schedule``):
  * ``gpipe``: fill-drain (torch Pipe's): all micro-batch forwards, then all backwards;
  * ``1f1b``: S - s - 1 warm-up forwards on stage s, then one forward / one backward
    alternating, then the cool-down backwards -- at most S micro-batches hold activations.
    The steady-state exchanges pair a send with the opposite receive in one
    ``batch_isend_irecv`` (both neighbours send at the same time there).

The loss of micro-batch m is ``loss_fn(out_m, target_m)`` weighted by m's share of the batch's
labelled (non-ignored) tokens, so the step's loss and gradients are those of ONE loss over the
concatenated output, as the reference computes it (``loss_weighting="mean"``: the mean of the
micro-batch means).  Receives are posted a micro-batch ahead and sends do not block; the
``checkpoint`` option recomputes micro-batch forwards in the backward as torch Pipe does.
"""
from __future__ import annotations

import torch
import torch.distributed as dist
from torch import nn
from torch.utils.checkpoint import checkpoint as _ckpt

from ..comm import logger as clog


class _Recv:
    """A posted receive: ``wait()`` returns the received activation on the stage's device."""

    def __init__(self, work, buf, device, host: bool):
        self.work, self.buf, self.device, self.host = work, buf, device, host

    def wait(self) -> torch.Tensor:
        if self.work is not None:
            self.work.wait()
            self.work = None
        return self.buf.to(self.device, non_blocking=True) if self.host else self.buf


class _Link:
    """Point-to-point messages between neighbouring stages.  RCCL sends device tensors directly;
    gloo (CPU tests, or several ranks sharing one GPU) stages device tensors through host memory.
    Sends are non-blocking (``isend``; the handles are kept until ``drain``) and receives are
    posted ahead of their consumer (``irecv``), so a stage computes while its next input is in
    flight instead of blocking in ``recv``."""

    def __init__(self, group=None):
        self.group = group
        self.backend = dist.get_backend(group)
        self.rank = dist.get_rank(group)
        self.inflight = []      # (work, tensor kept alive until the send completes)

    def _host(self, t: torch.Tensor) -> bool:
        return self.backend != "nccl" and t.is_cuda

    def isend(self, t: torch.Tensor, dst: int) -> None:
        t = t.detach()
        t = t.cpu() if self._host(t) else t.contiguous()
        self.inflight.append((clog.isend(t, dst, group=self.group), t))

    def irecv(self, like: torch.Tensor, src: int) -> _Recv:
        host = self._host(like)
        buf = torch.empty(like.shape, dtype=like.dtype) if host else torch.empty_like(like)
        return _Recv(clog.irecv(buf, src, group=self.group), buf, like.device, host)

    def send_recv(self, t: torch.Tensor, peer: int, like: torch.Tensor) -> _Recv:
        """Send ``t`` to ``peer`` and post the receive of a ``like``-shaped tensor from it in one
        ``batch_isend_irecv`` (the peer does the same at the same time: two blocking sends would
        wait for each other).  Only the receive is waited for, by its consumer."""
        host = self._host(t)
        src = t.detach()
        src = src.cpu() if host else src.contiguous()
        out = torch.empty(like.shape, dtype=like.dtype) if host else torch.empty_like(like)
        ops = [dist.P2POp(dist.isend, src, peer, self.group), dist.P2POp(dist.irecv, out, peer, self.group)]
        ws = dist.batch_isend_irecv(ops)
        self.inflight.append((ws[0], src))
        return _Recv(ws[1], out, like.device, host)

    def drain(self) -> None:
        for w, _ in self.inflight:
            if w is not None:
                w.wait()
        self.inflight.clear()


def micro_loss_weights(targets, chunks: int, ignore_index: int = -100):
    """Per-micro-batch loss weights that make the micro-batch losses sum to the loss of the whole
    concatenated batch: weight_m = (labelled tokens of m) / (labelled tokens of the batch), device
    tensors (no host sync).  The reference computes ONE CrossEntropyLoss over the concatenated
    pipeline output (/root/reference/model_parallel_training.py:68-75); with MLM labels (-100 on
    ~85 % of the tokens) each micro-batch has a different labelled count, so the plain mean of
    the micro-batch means would weight tokens unequally."""
    counts = torch.stack([(t != ignore_index).sum() for t in torch.chunk(targets, chunks, dim=0)]).float()
    return counts / counts.sum().clamp_min(1.0)


class StagePipeline(nn.Module):
    """Stage ``stage`` of an ``num_stages``-stage pipeline, one stage per rank of ``group``
    (stage s = rank s).

    ``modules``: this stage's module sequence (already on ``device``).  ``act_shape(mb)``: shape
    of the activation passed between stages for a micro-batch of ``mb`` rows; ``act_dtype`` its
    dtype.  ``loss_fn(out, target)``: the last stage's (mean) loss.  ``loss_weighting``:
    "tokens" (default: micro-batch m's mean loss weighted by its share of the batch's labelled
    tokens, ``micro_loss_weights`` -- the loss and gradients of the whole concatenated batch) or
    "mean" (the mean of the micro-batch means).  ``checkpoint``: activation recompute as torch
    Pipe / ``parallel/pipeline.py`` -- "except_last" (every micro-batch but the last keeps only its
    input and recomputes its forward in the backward), "always" or "never".  ``set_micro(m)``
    (optional) keys dropout masks on the micro-batch index, so a recomputed forward draws the same
    masks."""

    def __init__(self, modules, stage: int, num_stages: int, device, act_shape, act_dtype, loss_fn=None,
                 chunks: int = 1, schedule: str = "gpipe", group=None, set_micro=None, checkpoint: str = "never",
                 loss_weighting: str = "tokens", ignore_index: int = -100, overlap: bool = True):
        super().__init__()
        if schedule not in ("gpipe", "1f1b"):
            raise ValueError(schedule)
        if checkpoint not in ("never", "except_last", "always"):
            raise ValueError(checkpoint)
        if loss_weighting not in ("tokens", "mean"):
            raise ValueError(loss_weighting)
        if not overlap and schedule != "gpipe":
            raise ValueError("the blocking form (overlap=False) is a GPipe measurement baseline")
        self.mods = nn.ModuleList(modules)
        self.stage, self.num_stages = stage, num_stages
        self.device = torch.device(device)
        self.act_shape, self.act_dtype = act_shape, act_dtype
        self.loss_fn = loss_fn
        self.chunks, self.schedule = chunks, schedule
        self.set_micro = set_micro
        self.checkpoint = checkpoint
        self.loss_weighting, self.ignore_index = loss_weighting, ignore_index
        # overlap=False: the blocking form (each receive posted at its consumer and waited there,
        # each send waited right after it) -- kept to measure what the overlap buys
        self.overlap = bool(overlap)
        self.link = _Link(group)
        self.first = stage == 0
        self.last = stage == num_stages - 1

    def _fwd(self, m: int, x: torch.Tensor) -> torch.Tensor:
        if self.set_micro is not None:
            self.set_micro(m)
        for mod in self.mods:
            x = mod(x)
        return x

    def _run(self, m: int, x: torch.Tensor) -> torch.Tensor:
        ck = self.checkpoint == "always" or (self.checkpoint == "except_last" and m < self.chunks - 1)
        if ck and torch.is_grad_enabled() and self.training:
            return _ckpt(lambda inp, _m=m: self._fwd(_m, inp), x, use_reentrant=False, preserve_rng_state=False)
        return self._fwd(m, x)

    def _like(self, mb: int) -> torch.Tensor:
        return torch.empty(self.act_shape(mb), dtype=self.act_dtype, device=self.device)

    def train_step(self, inputs: torch.Tensor | None, targets: torch.Tensor | None,
                   rows: int | None = None) -> torch.Tensor | None:
        """Forward + backward of one mini-batch on this stage.  ``inputs`` (stage 0: the token
        ids) and ``targets`` (last stage: the labels) may be None on the other stages, which then
        take the mini-batch size from ``rows``; the rows are split into ``chunks`` equal
        micro-batches.  Returns the mini-batch loss on the last stage (detached), None
        elsewhere."""
        n, S, s = self.chunks, self.num_stages, self.stage
        ref = inputs if inputs is not None else targets
        if ref is None and rows is None:
            raise ValueError("a middle stage needs the mini-batch size (rows)")
        mb = (ref.shape[0] if ref is not None else rows) // n
        mx = list(torch.chunk(inputs, n, dim=0)) if inputs is not None else [None] * n
        mt = list(torch.chunk(targets, n, dim=0)) if targets is not None else [None] * n
        weights = None
        if self.last and self.loss_weighting == "tokens":
            weights = micro_loss_weights(targets.to(self.device), n, self.ignore_index)
        saved = []          # (input activation with grad, output or loss) per micro-batch in flight
        total = None

        def forward(m, x):
            nonlocal total
            if x is not None and not self.first:
                x = x.detach().requires_grad_(True)
            y = self._run(m, mx[m] if self.first else x)
            if self.last:
                y = self.loss_fn(y, mt[m].to(self.device))
                y = y * weights[m] if weights is not None else y / n
                total = y.detach() if total is None else total + y.detach()
            saved.append((x, y))
            return y

        def backward(g):
            x, y = saved.pop(0)
            if self.last:
                y.backward()
            else:
                y.backward(g)
            return None if self.first else x.grad

        # receives are posted one micro-batch ahead of their consumer (double-buffered: the
        # posted buffer and the one being consumed); every send is non-blocking
        def post_fwd(m):
            return None if self.first or m >= n else self.link.irecv(self._like(mb), s - 1)

        def post_bwd(k):
            return None if self.last or k >= n else self.link.irecv(self._like(mb), s + 1)

        def send_fwd(y):
            if not self.last:
                self.link.isend(y, s + 1)
                if not self.overlap:
                    self.link.drain()

        def send_bwd(gx):
            if not self.first:
                self.link.isend(gx, s - 1)
                if not self.overlap:
                    self.link.drain()

        def take(r):
            return None if r is None else r.wait()

        if self.schedule == "gpipe" and not self.overlap:   # the blocking form
            for m in range(n):
                send_fwd(forward(m, take(post_fwd(m))))
            for k in range(n):
                send_bwd(backward(take(post_bwd(k))))
        elif self.schedule == "gpipe":
            nxt = post_fwd(0)
            for m in range(n):
                cur, nxt = nxt, post_fwd(m + 1)
                send_fwd(forward(m, take(cur)))
            nxt = post_bwd(0)
            for k in range(n):
                cur, nxt = nxt, post_bwd(k + 1)
                send_bwd(backward(take(cur)))
        else:
            warm = min(S - s - 1, n)
            nxt = post_fwd(0)
            for m in range(warm):
                cur, nxt = nxt, post_fwd(m + 1)
                send_fwd(forward(m, take(cur)))
            x = take(nxt) if warm < n else None
            pend_x = None
            for i in range(n - warm):
                if pend_x is not None:
                    x = take(pend_x)
                y = forward(warm + i, x)
                # send this output, receive the gradient of the oldest in-flight micro-batch
                g = None if self.last else take(self.link.send_recv(y.detach(), s + 1, self._like(mb)))
                gx = backward(g)
                if i == n - warm - 1:
                    send_bwd(gx)
                    pend_x = None
                elif self.first:
                    x, pend_x = None, None
                else:
                    pend_x = self.link.send_recv(gx, s - 1, self._like(mb))
            nxt = post_bwd(0) if warm else None
            for k in range(warm):
                cur, nxt = nxt, post_bwd(k + 1) if k + 1 < warm else None
                send_bwd(backward(take(cur)))
        self.link.drain()
        if self.set_micro is not None:
            self.set_micro(0)
        return total


def bert_stage(config, stage: int, num_stages: int, device, dtype=torch.float32, impl: str = "auto", seed: int = 0):
    """This rank's stage of ``BertModelWithMP``: the full module list is built on the host with the
    reference's construction order and seed (identical weights on every rank and in the
    sequential model), split with the ``np.array_split`` law and only this stage's modules move
    to ``device``.  Returns (owner model, stage modules)."""
    from ..models.bert_mp import BertModelWithMP
    owner = BertModelWithMP(config=config, devices=["cpu"] * num_stages, dtype=torch.float32, impl=impl,
                            timing="host", seed=seed)
    mods = owner.groups[stage]
    for m in mods:
        m.to(device=device, dtype=dtype)
    owner.rt.rng = owner.rng_states["cpu"]
    if torch.device(device).type == "cuda":
        from ..ops.rng import RngState
        owner.rt.rng = RngState(seed, device=torch.device(device))
    return owner, mods
