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

The loss of micro-batch m is ``loss_fn(out_m, target_m) / chunks`` on the last stage, so the
gradients are those of the mean of the micro-batch losses (torch Pipe + the reference's loss on
the concatenated output give the same for equal micro-batches).
"""
from __future__ import annotations

import torch
import torch.distributed as dist
from torch import nn

from ..comm import logger as clog


class _Link:
    """Point-to-point messages between neighbouring stages.  RCCL sends device tensors directly;
    gloo (CPU tests, or several ranks sharing one GPU) stages device tensors through host memory."""

    def __init__(self, group=None):
        self.group = group
        self.backend = dist.get_backend(group)
        self.rank = dist.get_rank(group)

    def _host(self, t: torch.Tensor) -> bool:
        return self.backend != "nccl" and t.is_cuda

    def send(self, t: torch.Tensor, dst: int) -> None:
        clog.send(t.cpu() if self._host(t) else t.contiguous(), dst, group=self.group)

    def recv(self, like: torch.Tensor, src: int) -> torch.Tensor:
        if self._host(like):
            buf = torch.empty(like.shape, dtype=like.dtype)
            clog.recv(buf, src, group=self.group)
            return buf.to(like.device)
        buf = torch.empty_like(like)
        clog.recv(buf, src, group=self.group)
        return buf

    def send_recv(self, t: torch.Tensor, peer: int, like: torch.Tensor) -> torch.Tensor:
        """Send ``t`` to ``peer`` and receive a ``like``-shaped tensor from it, posted together (the
        peer does the same at the same time: two blocking sends would wait for each other)."""
        host = self._host(t)
        out = torch.empty(like.shape, dtype=like.dtype) if host else torch.empty_like(like)
        ops = [dist.P2POp(dist.isend, t.cpu() if host else t.contiguous(), peer, self.group),
               dist.P2POp(dist.irecv, out, peer, self.group)]
        for w in dist.batch_isend_irecv(ops):
            w.wait()
        return out.to(like.device) if host else out


class StagePipeline(nn.Module):
    """Stage ``stage`` of an ``num_stages``-stage pipeline, one stage per rank of ``group``
    (stage s = rank s).

    ``modules``: this stage's module sequence (already on ``device``).  ``act_shape(mb)``: shape
    of the activation passed between stages for a micro-batch of ``mb`` rows; ``act_dtype`` its
    dtype.  ``loss_fn(out, target)``: the last stage's loss.  ``set_micro(m)`` (optional) keys
    dropout masks on the micro-batch index, as the single-process GPipe does."""

    def __init__(self, modules, stage: int, num_stages: int, device, act_shape, act_dtype, loss_fn=None,
                 chunks: int = 1, schedule: str = "gpipe", group=None, set_micro=None):
        super().__init__()
        if schedule not in ("gpipe", "1f1b"):
            raise ValueError(schedule)
        self.mods = nn.ModuleList(modules)
        self.stage, self.num_stages = stage, num_stages
        self.device = torch.device(device)
        self.act_shape, self.act_dtype = act_shape, act_dtype
        self.loss_fn = loss_fn
        self.chunks, self.schedule = chunks, schedule
        self.set_micro = set_micro
        self.link = _Link(group)
        self.first = stage == 0
        self.last = stage == num_stages - 1

    def _fwd(self, m: int, x: torch.Tensor) -> torch.Tensor:
        if self.set_micro is not None:
            self.set_micro(m)
        for mod in self.mods:
            x = mod(x)
        return x

    def _like(self, mb: int) -> torch.Tensor:
        return torch.empty(self.act_shape(mb), dtype=self.act_dtype, device=self.device)

    def train_step(self, inputs: torch.Tensor | None, targets: torch.Tensor | None,
                   rows: int | None = None) -> torch.Tensor | None:
        """Forward + backward of one mini-batch on this stage.  ``inputs`` (stage 0: the token
        ids) and ``targets`` (last stage: the labels) may be None on the other stages, which then
        take the mini-batch size from ``rows``; the rows are split into ``chunks`` equal
        micro-batches.  Returns the summed micro-batch losses on the last stage (detached), None
        elsewhere."""
        n, S, s = self.chunks, self.num_stages, self.stage
        ref = inputs if inputs is not None else targets
        if ref is None and rows is None:
            raise ValueError("a middle stage needs the mini-batch size (rows)")
        mb = (ref.shape[0] if ref is not None else rows) // n
        mx = list(torch.chunk(inputs, n, dim=0)) if inputs is not None else [None] * n
        mt = list(torch.chunk(targets, n, dim=0)) if targets is not None else [None] * n
        saved = []          # (input activation with grad, output or loss) per micro-batch in flight
        total = None

        def forward(m, x):
            nonlocal total
            if x is not None and not self.first:
                x = x.detach().requires_grad_(True)
            y = self._fwd(m, mx[m] if self.first else x)
            if self.last:
                y = self.loss_fn(y, mt[m].to(self.device)) / n
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

        def recv_fwd():
            return None if self.first else self.link.recv(self._like(mb), s - 1)

        def send_fwd(y):
            if not self.last:
                self.link.send(y.detach(), s + 1)

        def recv_bwd():
            return None if self.last else self.link.recv(self._like(mb), s + 1)

        def send_bwd(gx):
            if not self.first:
                self.link.send(gx, s - 1)

        if self.schedule == "gpipe":
            for m in range(n):
                send_fwd(forward(m, recv_fwd()))
            for _ in range(n):
                send_bwd(backward(recv_bwd()))
        else:
            warm = min(S - s - 1, n)
            for m in range(warm):
                send_fwd(forward(m, recv_fwd()))
            x = recv_fwd() if warm < n else None
            for i in range(n - warm):
                y = forward(warm + i, x)
                # send this output, receive the gradient of the oldest in-flight micro-batch
                g = None if self.last else self.link.send_recv(y.detach(), s + 1, self._like(mb))
                gx = backward(g)
                if i == n - warm - 1:
                    send_bwd(gx)
                elif self.first:
                    x = None
                else:
                    x = self.link.send_recv(gx, s - 1, self._like(mb))
            for _ in range(warm):
                send_bwd(backward(recv_bwd()))
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
