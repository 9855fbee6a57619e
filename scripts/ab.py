#!/usr/bin/env python
"""Same-box A/B of bench.py: MI355X boxes differ by a few % in absolute throughput, so a change
is judged by alternating runs of the baseline variant and the candidate on one box.

  python scripts/ab.py VARIANT [VARIANT ...] [--rounds N] [-- bench args]

Variants are named patches applied in a fresh child process before bench.main() runs
("base" = the tree as is).  Prints per-run values and the per-variant median."""
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _old_wgrad_split():
    from distributed_training_and_deepspeed_amd.ops import grad as G

    def old(tokens, out_f, in_f):
        if tokens < 8192:
            return 1
        tiles = -(-out_f // 128) * -(-in_f // 128)
        s = 1
        while tiles * s < 512 and s < 16 and tokens % (2 * s) == 0 and tokens // (2 * s) >= 1024:
            s *= 2
        return s
    G.wgrad_splits = old


def _f32_wgrad_partials():
    from distributed_training_and_deepspeed_amd.ops import grad as G
    orig = G._bmm_partials
    G._bmm_partials = lambda a, b, fp32=True: orig(a, b, True)


def _no_keep_ffn_act():
    from distributed_training_and_deepspeed_amd.models import transformer as T
    orig = T.Runtime.__init__

    def init(self, *a, **k):
        orig(self, *a, **k)
        self.keep_ffn_act = False
    T.Runtime.__init__ = init


def _no_tuned():
    os.environ["PYTORCH_TUNABLEOP_ENABLED"] = "0"


def _mlm_static():
    # static-capacity sparse MLM head in eager mode (no nonzero() host sync per step)
    from distributed_training_and_deepspeed_amd.models import transformer as T
    from distributed_training_and_deepspeed_amd.utils.graphs import mlm_capacity
    orig = T.Runtime.__init__

    def init(self, *a, **k):
        orig(self, *a, **k)
        self.mlm_capacity = -(-mlm_capacity(int(os.environ.get("DTD_BENCH_BATCH", "256")) * 512) // 256) * 256
    T.Runtime.__init__ = init


def _wgrad_fixed(n):
    def f():
        from distributed_training_and_deepspeed_amd.ops import grad as G
        G.wgrad_splits = lambda tokens, out_f, in_f: n if tokens >= 8192 else 1
    return f


def _env(**kv):
    def f():
        os.environ.update(kv)
    return f


PATCHES = {"async_wgrad": lambda: ["--async-wgrad", "on"], "no_tuned": _no_tuned, "mlm_static": _mlm_static, "mlm_dynamic": lambda: ["--mlm-capacity", "dynamic"], "graph": lambda: ["--graph", "on"], "graph_async_wgrad": lambda: ["--graph", "on", "--async-wgrad", "on"],
           "attn_occ_323": _env(DTD_ATTN_OCC="3,2,3"), "attn_occ_222_dq64": _env(DTD_ATTN_TILE="64,64"),
           "attn_occ_322": _env(DTD_ATTN_OCC="3,2,2"), "attn_occ_323_dq64": _env(DTD_ATTN_OCC="3,2,3", DTD_ATTN_TILE="64,64"),
           "wgrad_s1": _wgrad_fixed(1), "wgrad_s4": _wgrad_fixed(4), "wgrad_s8": _wgrad_fixed(8),
           "retuned": _env(DTD_TUNED_TABLE=os.path.join(ROOT, "gpurun_out", "tunableop_new0.csv")),
           "mask_x2": _env(DTD_ATTN_MASK_REPEAT="2"),
           "wgrad_s32": _wgrad_fixed(32), "wgrad_s64": _wgrad_fixed(64),
           "gemm_split": _env(DTD_GEMM_VARIANT="2"), "dgrad_nn": _env(DTD_DGRAD_NT="0"),
           "dkdv_bm64": _env(DTD_ATTN_DKDV_BM="64"), "gemm_all": _env(DTD_GEMM_ALL="1"),
           "attn_fwd_pipe": _env(DTD_ATTN_FWD="pipe"), "attn_pk": _env(DTD_ATTN_FWD_PK="1"),
           "ln_memeff_off": _env(DTD_LN_MEMEFF="0"), "ln_bwd_prefetch": _env(DTD_LN_BWD_PREFETCH="1"),
           "base": lambda: None, "old_wgrad_split": _old_wgrad_split, "f32_wgrad_partials": _f32_wgrad_partials,
           "no_keep_ffn_act": _no_keep_ffn_act, "ew_plain": _env(DTD_EW_MODE="0"),
           "no_gemm": _env(DTD_GEMM="0"), "gemm_bwd_only": _env(DTD_GEMM_FFN_FWD="0"),
           "gemm_fwd_only": _env(DTD_GEMM_FFN_BWD="0"), "gemm_tile": _env(DTD_GEMM_VARIANT="0"),
           "no_gemm_wgrad": _env(DTD_GEMM_WGRAD="0"), "gemm_wgrad": _env(DTD_GEMM_WGRAD="1"),
           "mask_ballot": _env(DTD_ATTN_MASK="0"), "mlm_scatter_off": _env(DTD_MLM_SCATTER="0"), "wt_batch_off": _env(DTD_WT_BATCH="0"), "no_qkv_bias_fused": _env(DTD_ATTN_QKV_BIAS="0"),
           "no_ffn_store_grad": _env(DTD_GEMM_FFN_STORE_GRAD="0"),
           "opt_overlap_off": lambda: ["--opt-overlap", "off"], "gemm_sched_static": _env(DTD_GEMM_SCHED="static"),
           "no_fused_embed_ln": _env(DTD_FUSED_EMBED_LN="0"), "no_fused_xent": _env(DTD_FUSED_XENT="0"), "fused_xent": _env(DTD_FUSED_XENT="1"), "no_defer_finalize": _env(DTD_DEFER_FINALIZE="0"),
           "gemm_stagger2": _env(DTD_GEMM_STAGGER_US="2"), "gemm_stagger4": _env(DTD_GEMM_STAGGER_US="4"),
           "attn_bwd_fused": _env(DTD_ATTN_BWD="fused"), "no_wgrad2": _env(DTD_GEMM_WGRAD="0"),
           "fc": lambda: ["--force-collectives"],
           "fc_prewarm_l1b": lambda: ["--force-collectives", "--prewarm", "layer1-batch"],
           "fc_no_wgrad2": lambda: (os.environ.update(DTD_GEMM_WGRAD="0") or ["--force-collectives"]),
           "fc_noprewarm": lambda: ["--force-collectives", "--prewarm", "none"],
           "fc_noprewarm_eagerload": lambda: (os.environ.update(HIP_ENABLE_DEFERRED_LOADING="0")
                                              or ["--force-collectives", "--prewarm", "none"]),
           "dmabuiltin_so": _env(DTD_KERNELS_SO=os.path.join(ROOT, "distributed_training_and_deepspeed_amd", "ops",
                                                            "_dtd_kernels_dmabuiltin.so")),
           "b320": lambda: ["--batch-size", "320"], "b384": lambda: ["--batch-size", "384"],
           "dkdv_occ1": _env(DTD_ATTN_OCC="3,1,3"),
           "gemm_ln": _env(DTD_GEMM_LN="1"), "gemm_ln_p0": _env(DTD_GEMM_LN="1", DTD_GEMM_LN_PIPE="0"),
           "base_so": _env(DTD_KERNELS_SO=os.path.join(ROOT, "distributed_training_and_deepspeed_amd", "ops",
                                                      "_dtd_kernels_base.so")),
           # round-4 keep-mask generator (per-word xorshift + alignbit insertion), built from the
           # previous attention.hip into ops/_dtd_kernels_oldmask.so
           "oldmask_so": _env(DTD_KERNELS_SO=os.path.join(ROOT, "distributed_training_and_deepspeed_amd", "ops",
                                                         "_dtd_kernels_oldmask.so"))}


def child(variant, bench_args):
    sys.path.insert(0, ROOT)
    extra = PATCHES[variant]() or []
    sys.argv = ["bench.py"] + bench_args + list(extra)
    import bench
    bench.main()


def main():
    args = sys.argv[1:]
    if args and args[0] == "--child":
        child(args[1], args[2:])
        return
    bench_args = []
    if "--" in args:
        i = args.index("--")
        args, bench_args = args[:i], args[i + 1:]
    rounds = 2
    if "--rounds" in args:
        i = args.index("--rounds")
        rounds = int(args[i + 1])
        args = args[:i] + args[i + 2:]
    variants = args or ["base"]
    res = {v: [] for v in variants}
    for _ in range(rounds):
        for v in variants:
            out = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", v] + bench_args,
                                 capture_output=True, text=True, timeout=600)
            line = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
            if out.returncode != 0 or not line:
                print(json.dumps({"variant": v, "error": out.stderr[-500:]}), flush=True)
                sys.exit(1)
            val = json.loads(line[-1])["value"]
            res[v].append(val)
            print(json.dumps({"variant": v, "value": val}), flush=True)
    print(json.dumps({"median": {v: statistics.median(x) for v, x in res.items()}}), flush=True)


if __name__ == "__main__":
    main()
