"""Fused Adam/AdamW over flat buffers: one HIP kernel launch per optimizer step.

Replaces DeepSpeed FusedAdam (selected by ``"optimizer": {"type": "Adam"}``,
zero_dp_training.py:28-33, adam_w_mode=True), ``torch.optim.AdamW``
(model_parallel_training.py:50) and ``transformers.AdamW`` (data_parallel_training.py:34)
-- SURVEY.md D12/D21/K9.  Hyper-parameter conventions per script are reproduced by
``hf_eps`` (transformers: eps added to sqrt(v) before bias correction) and the defaults.

Storage: parameters of the optimizer live in a flat buffer (shared with DDP/ZeRO when the
model is wrapped, see ``parallel/flat.py``); gradients in the matching flat ``main_grad``
buffer; fp32 master weights are kept when the model runs in bf16 (the kernel writes the
updated bf16 copy in the same pass).  Step count, lr and the gradient scale live in a small
device array so the step is hipGraph-capturable and clipping needs no host sync.
"""
from __future__ import annotations

import math

import torch

from ..ops import _lib
from ..ops import functional as Fx
from ..parallel.flat import FlatLayout, GradBuffer

MODE_ADAMW, MODE_BIAS_CORR, MODE_HF_EPS = 1, 2, 4


def _flat_view_of(t: torch.Tensor, numel: int) -> torch.Tensor:
    return torch.empty(0, dtype=t.dtype, device=t.device).set_(t.untyped_storage(), 0, (numel,))


def adam_reference_(p, m, v, g, lr, b1, b2, eps, wd, step, mode, grad_scale=1.0):
    """fp32 PyTorch implementation of the kernel math (CPU path and test oracle)."""
    g = g.float() * grad_scale
    if not (mode & MODE_ADAMW) and wd != 0:
        g = g + wd * p
    m.mul_(b1).add_(g, alpha=1 - b1)
    v.mul_(b2).addcmul_(g, g, value=1 - b2)
    if mode & MODE_ADAMW:
        p.mul_(1 - lr * wd)
    bc1 = 1 - b1 ** step if mode & MODE_BIAS_CORR else 1.0
    bc2s = math.sqrt(1 - b2 ** step) if mode & MODE_BIAS_CORR else 1.0
    if mode & MODE_HF_EPS:
        p.addcdiv_(m, v.sqrt().add_(eps), value=-lr * bc2s / bc1)
    else:
        p.addcdiv_(m, v.sqrt().div_(bc2s).add_(eps), value=-lr / bc1)


def stage_chunks(spans, nstages: int, n: int) -> list:
    """Element ranges of a flat buffer [0, n) per optimizer stage.  ``spans``: (start, end, stage)
    of each parameter.  Returns nstages + 1 lists of merged [a, b) ranges: index 0 holds the
    elements no stage owns (padding, parameters registered elsewhere), index k + 1 stage k's.  An
    element shared by several stages (tied parameters) belongs to the first span that covers it;
    together the lists cover [0, n) exactly once."""
    chunks = {k: [] for k in range(-1, nstages)}
    pos = 0
    for a, b, k in sorted(spans):
        a = max(a, pos)
        if a >= b:
            continue
        if a > pos:
            chunks[-1].append((pos, a))
        chunks[k].append((a, b))
        pos = b
    if pos < n:
        chunks[-1].append((pos, n))
    out = []
    for k in range(-1, nstages):
        merged = []
        for a, b in sorted(chunks[k]):
            if merged and merged[-1][1] == a:
                merged[-1] = (merged[-1][0], b)
            else:
                merged.append((a, b))
        out.append(merged)
    return out


class FusedAdam(torch.optim.Optimizer):
    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 0.0,
                 adam_w_mode: bool = True, bias_correction: bool = True, hf_eps: bool = False,
                 max_grad_norm: float | None = None):
        params = list(params)
        defaults = dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay,
                        bias_correction=bias_correction)
        super().__init__(params, defaults)
        self.mode = (MODE_ADAMW if adam_w_mode else 0) | (MODE_BIAS_CORR if bias_correction else 0) | \
            (MODE_HF_EPS if hf_eps else 0)
        self.max_grad_norm = max_grad_norm
        self._setup()

    @classmethod
    def from_flat(cls, master: torch.Tensor, grad: torch.Tensor, lowp: torch.Tensor | None = None, **kw):
        """Optimizer over pre-built flat buffers (a ZeRO partition): fp32 ``master`` weights,
        matching ``grad`` buffer and optional low-precision copy written by the kernel.
        ``param_groups[0]['params'] == [master]`` so its numel is the local partition size."""
        self = cls.__new__(cls)
        defaults = dict(lr=kw.pop("lr", 1e-3), betas=tuple(kw.pop("betas", (0.9, 0.999))), eps=kw.pop("eps", 1e-8),
                        weight_decay=kw.pop("weight_decay", 0.0), bias_correction=kw.get("bias_correction", True))
        torch.optim.Optimizer.__init__(self, [master], defaults)
        self.mode = (MODE_ADAMW if kw.get("adam_w_mode", True) else 0) | \
            (MODE_BIAS_CORR if kw.get("bias_correction", True) else 0) | (MODE_HF_EPS if kw.get("hf_eps", False) else 0)
        self.max_grad_norm = kw.get("max_grad_norm")
        self._params = []
        self.param_flat, self.grad_flat, self.gbuf = master, grad, None
        self.master, self.lowp = master, lowp
        dev, n = master.device, master.numel()
        self.exp_avg = torch.zeros(n, dtype=torch.float32, device=dev)
        self.exp_avg_sq = torch.zeros(n, dtype=torch.float32, device=dev)
        self.hp = torch.zeros(8, dtype=torch.float32, device=dev)
        self._hp_host = None
        self.step_count = 0
        self._chunks = None
        self._push_hparams()
        return self

    # ------------------------------------------------------------------ storage
    def _setup(self) -> None:
        ps = [p for g in self.param_groups for p in g["params"] if p.requires_grad]
        self._params = ps
        shared = self._detect_shared_flat(ps)
        if shared is None:
            layout = FlatLayout(ps)
            self.param_flat = layout.flatten_params_()
            self.gbuf = GradBuffer(layout, ps[0].dtype, ps[0].device)
            self.grad_flat = self.gbuf.buf
        else:
            self.param_flat, self.grad_flat = shared
            self.gbuf = None
        dev = self.param_flat.device
        n = self.param_flat.numel()
        if self.param_flat.dtype == torch.float32:
            self.master, self.lowp = self.param_flat, None
        else:
            self.master, self.lowp = self.param_flat.float(), self.param_flat
        self.exp_avg = torch.zeros(n, dtype=torch.float32, device=dev)
        self.exp_avg_sq = torch.zeros(n, dtype=torch.float32, device=dev)
        self.hp = torch.zeros(8, dtype=torch.float32, device=dev)
        self._hp_host = None
        self.step_count = 0
        self._chunks = None
        self._push_hparams()

    @staticmethod
    def _detect_shared_flat(ps):
        """Params already laid out by DDP/ZeRO: one param storage + one main_grad storage."""
        if not ps or any(getattr(p, "main_grad", None) is None for p in ps):
            return None
        st = {p.untyped_storage().data_ptr() for p in ps}
        gst = {p.main_grad.untyped_storage().data_ptr() for p in ps}
        if len(st) != 1 or len(gst) != 1:
            return None
        if any(p.storage_offset() != p.main_grad.storage_offset() for p in ps):
            return None
        numel = ps[0].untyped_storage().nbytes() // ps[0].element_size()
        gnumel = ps[0].main_grad.untyped_storage().nbytes() // ps[0].main_grad.element_size()
        if numel != gnumel or sum(p.numel() for p in ps) > numel:
            return None
        return _flat_view_of(ps[0], numel), _flat_view_of(ps[0].main_grad, gnumel)

    def _push_hparams(self) -> None:
        g = self.param_groups[0]
        host = (float(g["lr"]), float(g["betas"][0]), float(g["betas"][1]), float(g["eps"]),
                float(g["weight_decay"]))
        if host != self._hp_host:
            self.hp[:5].copy_(torch.tensor(host, dtype=torch.float32))
            self.hp[6] = 1.0
            self._hp_host = host

    # ------------------------------------------------------------------ step
    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        Fx.flush_finalizes()  # a backward's batched bias / LayerNorm finalizes (normally flushed at its end)
        self.synchronize()   # staged updates of the previous step: hp / gradients are rewritten below
        if self.gbuf is not None:  # gradients assigned to p.grad by hand (not via autograd)
            for p in self._params:
                g = p.grad
                if g is not None and g.data_ptr() != p.main_grad.data_ptr():
                    if getattr(p, "_dtd_touched", False):
                        p.main_grad.add_(g.to(p.main_grad.dtype))
                    else:
                        p.main_grad.copy_(g)
                    p._dtd_touched = True
            self.gbuf.zero_untouched_()  # no gradient this step -> zero, not last step's value
        self._push_hparams()
        self.step_count += 1
        self.hp[5:6].add_(1.0)
        if self.max_grad_norm is not None:
            sq = Fx.sq_norm(self.grad_flat)
            red = getattr(self, "_reduce_sqnorm", None)  # ZeRO: sum over partitions (C11)
            if red is not None:
                sq = red(sq)
            norm = sq.sqrt()
            self.hp[6:7].copy_(torch.clamp(self.max_grad_norm / (norm + 1e-6), max=1.0).reshape(1))
        n = self.master.numel()
        if self.master.is_cuda and self._chunks is not None:
            self._step_staged()
        elif self.master.is_cuda:
            _lib.call("dtd_adam_step", self.master.data_ptr(), self.exp_avg.data_ptr(), self.exp_avg_sq.data_ptr(),
                      self.grad_flat.data_ptr(), _lib.dt(self.grad_flat), _lib.ptr(self.lowp), n,
                      self.hp.data_ptr(), self.mode, _lib.stream())
        else:
            g = self.param_groups[0]
            adam_reference_(self.master, self.exp_avg, self.exp_avg_sq, self.grad_flat, g["lr"], g["betas"][0],
                            g["betas"][1], g["eps"], g["weight_decay"], self.step_count, self.mode,
                            float(self.hp[6]))
            if self.lowp is not None:
                self.lowp.copy_(self.master)
        if self.gbuf is not None:
            self.gbuf.reset()
        return loss

    # ------------------------------------------------------------------ overlap with forward
    def overlap_with_forward(self, stages, root=None) -> None:
        """Let the next forward start while later stages' parameters are still being updated.
        ``stages``: the model's modules in forward order (e.g. ``model.zero3_units()``).
        step() then runs the same Adam kernel stage by stage on a side stream and records one
        event per stage; a forward pre-hook on each stage makes the compute stream wait for that
        stage's parameters only, so the HBM-bound update of the later stages runs under the first
        stages' MFMA-bound GEMMs instead of before them.  Elements no stage owns (padding, params
        registered elsewhere) are updated first and waited for by the first stage; a post-hook on
        ``root`` (the whole model; default: the last stage) waits for every chunk before anything
        after the forward runs (the next backward overwrites the gradients the kernel reads).  Per
        element the math is the single launch's: results are bit-identical.

        Contract: between step() and the end of the next forward of ``root``, a parameter may be
        read only inside the forward of its own stage (after that stage's pre-hook).  Code that
        reads weights elsewhere -- a submodule method called directly, EMA / logging of weights,
        evaluation through submodules -- must call ``synchronize()`` first (state_dict,
        load_state_dict and checkpoint saving do).  The scripts enable this only where the
        training loop honours that (bench.py; data_parallel_training.py ``--opt-overlap``)."""
        if not self.master.is_cuda or self._chunks is not None:
            return
        base = self.param_flat
        st = base.untyped_storage().data_ptr()
        n = self.master.numel()
        spans = []   # (start, end, stage index)
        for k, m in enumerate(stages):
            for p in m.parameters():
                if p.untyped_storage().data_ptr() != st or not p.requires_grad:
                    continue
                off = p.storage_offset() - base.storage_offset()
                if 0 <= off and off + p.numel() <= n:
                    spans.append((off, off + p.numel(), k))
        self._chunks = stage_chunks(spans, len(stages), n)
        self._side = torch.cuda.Stream(self.master.device)
        self._events = [None] * len(self._chunks)
        self._hooks = []
        last = len(stages) - 1
        for k, m in enumerate(stages):
            waits = (0, k + 1) if k == 0 else (k + 1,)
            self._hooks.append(m.register_forward_pre_hook(
                lambda mod, inp, w=waits: self._wait(w)))
        self._hooks.append((root if root is not None else stages[last]).register_forward_hook(
            lambda mod, inp, out: self.synchronize()))

    def _wait(self, idx) -> None:
        cur = torch.cuda.current_stream(self.master.device)
        for i in idx:
            ev = self._events[i]
            if ev is not None:
                cur.wait_event(ev)
                self._events[i] = None

    def synchronize(self) -> None:
        """Make the current stream wait for every staged update still pending."""
        if self._chunks is not None:
            self._wait(range(len(self._events)))

    def _step_staged(self) -> None:
        self.synchronize()   # a previous step's chunks no forward waited for
        side = self._side
        side.wait_stream(torch.cuda.current_stream(self.master.device))
        es, gs = 4, self.grad_flat.element_size()
        lp = self.lowp
        with torch.cuda.stream(side):
            for i, rs in enumerate(self._chunks):
                for a, b in rs:
                    _lib.call("dtd_adam_step", self.master.data_ptr() + a * es, self.exp_avg.data_ptr() + a * es,
                              self.exp_avg_sq.data_ptr() + a * es, self.grad_flat.data_ptr() + a * gs,
                              _lib.dt(self.grad_flat), None if lp is None else lp.data_ptr() + a * lp.element_size(),
                              b - a, self.hp.data_ptr(), self.mode, side.cuda_stream)
                ev = torch.cuda.Event()
                ev.record(side)
                self._events[i] = ev

    # ------------------------------------------------------------------ ranges (overlap with backward)
    def begin_ranged_step(self) -> None:
        """Start a step whose update is launched range by range (``step_range``), e.g. by the
        ZeRO engine as each partition segment's gradient becomes final during the backward: the
        step counter and hyper-parameters advance once, here, on the current stream.  Needs no
        global gradient norm (``max_grad_norm`` None)."""
        assert self.max_grad_norm is None and self.master.is_cuda and self._chunks is None
        self._push_hparams()
        self.step_count += 1
        self.hp[5:6].add_(1.0)

    def step_range(self, a: int, b: int, stream) -> None:
        """The fused Adam kernel over elements [a, b) of the flat buffers on ``stream`` (per
        element the same math as the whole-buffer launch: bit-identical results)."""
        if b <= a:
            return
        es, gs, lp = 4, self.grad_flat.element_size(), self.lowp
        _lib.call("dtd_adam_step", self.master.data_ptr() + a * es, self.exp_avg.data_ptr() + a * es,
                  self.exp_avg_sq.data_ptr() + a * es, self.grad_flat.data_ptr() + a * gs,
                  _lib.dt(self.grad_flat), None if lp is None else lp.data_ptr() + a * lp.element_size(),
                  b - a, self.hp.data_ptr(), self.mode, stream.cuda_stream)

    def parameters_ready(self) -> None:
        """Public fence for code that reads parameters outside a stage forward (see the
        contract of overlap_with_forward): the current stream waits for every staged update."""
        self.synchronize()

    def zero_grad(self, set_to_none: bool = True):
        if self.gbuf is not None:
            self.gbuf.reset()
        for p in self._params:
            p.grad = None

    def state_dict(self):
        self.synchronize()
        # under hipGraph replay only the device copy of the step count advances
        step = int(self.hp[5].item()) if self.hp.is_cuda else self.step_count
        return {"step": step, "exp_avg": self.exp_avg, "exp_avg_sq": self.exp_avg_sq,
                "master": self.master, "param_groups": [{k: v for k, v in g.items() if k != "params"}
                                                         for g in self.param_groups]}

    def load_state_dict(self, sd):
        self.synchronize()
        self.step_count = int(sd["step"])
        self.exp_avg.copy_(sd["exp_avg"])
        self.exp_avg_sq.copy_(sd["exp_avg_sq"])
        self.master.copy_(sd["master"])
        if self.lowp is not None:
            self.lowp.copy_(self.master)
        self.hp[5] = float(self.step_count)
        for g, s in zip(self.param_groups, sd["param_groups"]):
            g.update(s)
