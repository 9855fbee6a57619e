"""Launch the training step's kernels once BEFORE the RCCL communicator is created.

Measured on MI355X (docs/PERFORMANCE.md, "Kernels first launched after the RCCL communicator"):
after ``ncclCommInitRank`` every kernel of the BERT step that had not been launched yet runs
5-25 % longer for the rest of the process -- identical L2 / HBM traffic, more cycles
(profiles/r4_s40_rccl_init_pmc.jsonl) -- and the N > 1 step loses ~10 %
(profiles/r4_s33_*, r4_s43_*).  Kernels launched before it keep their speed: creating the group
after the warm-up steps, or after one batch-1 forward/backward of the model, costs nothing.
Loading the code objects, torch's stream pools or a few GEMMs first does not help
(profiles/r4_s44_*, r4_s45_*): the step's own kernels have to run once.

``prewarm_model_kernels`` builds a throwaway copy of the model (``layers`` deep -- every encoder
layer runs the same kernels), runs one batch-1 forward + backward on synthetic tokens and frees
it (and one fused Adam step on its gradients).  The entry scripts call it before ``comm.init`` (env ``DTD_PREWARM=0`` turns it off).

Round-6 bisect (profiles/r6_prewarm_bisect.jsonl: b256 with RCCL bucket all-reduces at world 1,
two interleaved rounds, fresh processes): no prewarm 1.315 / 1.321 M tokens/s; one hipBLASLt
GEMM only (``prewarm_blas``) 1.318 / 1.317 M; a 45 GB allocator reservation only
(``prewarm_reserve``) 1.315 / 1.314 M; the 1-layer step with its products on the hand-written
kernels (hipBLASLt only where they do not tile) 1.459 / 1.462 M; the default prewarm 1.461 /
1.461 M.  So the part that matters is the first launch of the framework's own kernels before the
communicator exists -- not the BLAS handle, not the allocator.  The round-5 post-init probe (a
streaming kernel pair in its own code object) never fired and was removed."""
from __future__ import annotations

import dataclasses
import os

import torch


def prewarm_enabled() -> bool:
    return os.environ.get("DTD_PREWARM", "1") != "0" and torch.cuda.is_available()


def prewarm_model_kernels(name: str, device, dtype=torch.bfloat16, impl: str = "auto", seq_len: int = 512,
                          layers: int | None = 1, batch: int = 1, static_mlm: bool = True, optimizer: bool = True,
                          library_gemms: bool = True, **model_kw) -> None:
    """``library_gemms=False``: the products the hand-written GEMMs tile run on them instead of
    hipBLASLt (the "custom kernels only" arm of the bisect, bench.py --prewarm custom).  Either
    way the one-wave-per-SIMD GEMM takes the batch-1 products (it would not at that size in a
    real step) so that the kernel the big step uses is launched here."""
    from ..ops import gemm as G
    with G.hand_kernels_at_any_size(library=library_gemms):
        _prewarm(name, device, dtype, impl, seq_len, layers, batch, static_mlm, optimizer, **model_kw)


def prewarm_blas(device, dtype=torch.bfloat16, m: int = 4096, n: int = 768, k: int = 768) -> None:
    """Bisect arm: only a hipBLASLt handle / workspace and one GEMM (with bias, the forward form)."""
    a = torch.randn(m, k, device=device, dtype=dtype)
    w = torch.randn(n, k, device=device, dtype=dtype)
    b = torch.randn(n, device=device, dtype=dtype)
    torch.nn.functional.linear(a, w, b)
    torch.cuda.synchronize(device)


def prewarm_reserve(device, nbytes: int) -> None:
    """Bisect arm: only the caching allocator's reservation of ``nbytes`` (the step's peak), freed
    to the cache (not to the driver) so the step's tensors are carved from it."""
    t = torch.empty(nbytes, dtype=torch.uint8, device=device)
    t.fill_(0)
    torch.cuda.synchronize(device)
    del t


def _prewarm(name, device, dtype, impl, seq_len, layers, batch, static_mlm, optimizer, **model_kw) -> None:
    from ..data import SyntheticLMDataset
    from ..models import get_config
    from ..models.bert import BertForMaskedLM
    from ..models.causal_lm import CausalLM
    from ..models.transformer import Runtime
    from ..ops.rng import RngState
    dev = torch.device(device)
    cfg = get_config(name)
    if layers is not None:
        cfg = dataclasses.replace(cfg, num_layers=min(layers, cfg.num_layers))
    rng_state = torch.random.get_rng_state()
    rt = Runtime(impl=impl, rng=RngState(seed=0, device=dev))
    cls = BertForMaskedLM if cfg.family == "bert" else CausalLM
    model = cls(cfg, rt=rt, **model_kw).to(device=dev, dtype=dtype)
    model.train()
    if cfg.family == "bert" and static_mlm:
        from .graphs import mlm_capacity
        rt.mlm_capacity = -(-mlm_capacity(batch * seq_len) // 256) * 256
        rt.mlm_overflow = torch.zeros((), dtype=torch.bool, device=dev)
    ds = SyntheticLMDataset(cfg, num_samples=batch, seq_len=min(seq_len, cfg.max_positions), mlm=cfg.family == "bert",
                            seed=0)
    out = model(ds.input_ids.to(dev), labels=ds.labels.to(dev))
    out.loss.backward()
    if optimizer:
        # the fused Adam kernel (DDP's hf_adamw and the ZeRO engine's optimizer) runs once too
        from ..optim import hf_adamw
        opt = hf_adamw([p for p in model.parameters() if p.grad is not None], lr=0.0)
        opt.step()
        del opt
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    del model, out
    if dev.type == "cuda":
        torch.cuda.empty_cache()   # hand the throwaway model's memory back (large ZeRO-3 runs)
    torch.random.set_rng_state(rng_state)
