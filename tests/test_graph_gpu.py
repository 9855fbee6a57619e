"""Whole-step hipGraph capture (utils/graphs.py): replaying the captured step trains exactly like
running the same step eagerly (same kernels, same static MLM capacity, device-side RNG step)."""
import pytest
import torch

from distributed_training_and_deepspeed_amd.data import SyntheticLMDataset
from distributed_training_and_deepspeed_amd.models import build_model
from distributed_training_and_deepspeed_amd.optim import hf_adamw
from distributed_training_and_deepspeed_amd.parallel import DistributedDataParallel
from distributed_training_and_deepspeed_amd.utils.graphs import CapturedStep, mlm_capacity

pytestmark = pytest.mark.gpu


def _setup():
    model = build_model("tiny", dtype=torch.bfloat16, device="cuda", seed=3)
    model.rt.mlm_capacity = mlm_capacity(4 * 128)
    model.rt.mlm_overflow = torch.zeros((), dtype=torch.bool, device="cuda")
    ddp = DistributedDataParallel(model)
    opt = hf_adamw(ddp.parameters(), lr=1e-3)

    def step(input_ids, labels):
        out = ddp(input_ids, labels=labels)
        out.loss.backward()
        opt.step()
        model.rt.rng.advance()
        return out.loss.detach()
    return model, step


def test_captured_step_matches_eager():
    ds = SyntheticLMDataset(build_model("tiny").cfg, 4 * 8, seq_len=128, seed=5)
    ids = ds.input_ids.view(8, 4, 128).cuda()
    lab = ds.labels.view(8, 4, 128).cuda()
    ma, sa = _setup()
    mb, sb = _setup()
    # B: 3 warm-up steps run eagerly inside CapturedStep, then replays; A: the same 3 + replays eagerly
    cap = CapturedStep(sb, {"input_ids": ids[0], "labels": lab[0]}, warmup=3, runtime=mb.rt)
    la = [sa(ids[0], lab[0]) for _ in range(3)]
    la += [sa(ids[i], lab[i]) for i in range(1, 6)]
    lb = [cap(input_ids=ids[i], labels=lab[i]).clone() for i in range(1, 6)]
    torch.cuda.synchronize()
    cap.check()
    assert torch.equal(torch.stack(la[3:]), torch.stack(lb))
    for (n, p), q in zip(ma.named_parameters(), mb.parameters()):
        assert torch.equal(p, q), n


@pytest.mark.parametrize("stage,replicated", [(0, True), (1, True), (2, True), (3, True), (1, False), (2, False), (3, False)])
def test_captured_zero_step_matches_eager(stage, replicated):
    """zero_dp_training.py --graph: a replayed ZeRO step (causal LM, fused Adam with device-side
    step count, parameter refresh, RNG advance; stage 2/3 landing regions and stage-3 gathered
    units from the persistent arenas) equals the eager engine step."""
    import os
    from distributed_training_and_deepspeed_amd import comm
    from distributed_training_and_deepspeed_amd.parallel.zero import initialize
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(31000 + os.getpid() % 1000 + stage + 10 * replicated)
    comm.init(rank=0, world_size=1, backend="nccl", local_rank=0)
    try:
        def setup():
            model = build_model("causal-tiny", dtype=torch.bfloat16, device="cuda", seed=3)
            cfg = {"optimizer": {"type": "Adam", "params": {"lr": 1e-3}}, "comms_logger": {"enabled": False},
                   "zero_optimization": {"stage": stage, "reduce_bucket_size": 100000,
                                         "world1_replicated": replicated}}
            eng, _, _, _ = initialize(model=model, model_parameters=model.parameters(), config=cfg)

            def step(input_ids, labels):
                out = eng(input_ids, labels=labels)
                eng.backward(out.loss)
                eng.step()
                return out.loss.detach()
            return eng, step

        ds = SyntheticLMDataset(build_model("causal-tiny").cfg, 4 * 8, seq_len=128, mlm=False, seed=5)
        ids = ds.input_ids.view(8, 4, 128).cuda()
        lab = ds.labels.view(8, 4, 128).cuda()
        ea, sa = setup()
        eb, sb = setup()
        cap = CapturedStep(sb, {"input_ids": ids[0], "labels": lab[0]}, warmup=3, runtime=eb.module.rt)
        la = [sa(ids[0], lab[0]) for _ in range(3)]
        la += [sa(ids[i], lab[i]) for i in range(1, 6)]
        lb = [cap(input_ids=ids[i], labels=lab[i]).clone() for i in range(1, 6)]
        torch.cuda.synchronize()
        assert torch.equal(torch.stack(la[3:]), torch.stack(lb))
        assert torch.equal(ea.master, eb.master)
    finally:
        comm.destroy()


@pytest.mark.parametrize("stage", [0, 2, 3])
def test_zero_script_graph_trains_like_eager(stage):
    """zero_dp_training.py end to end: --graph (default on one GPU) warms up on the first real
    batches and replays the rest -- the same steps on the same batches as --graph off."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    res = {}
    for mode in ("off", "on"):
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(32000 + os.getpid() % 1000 + len(res)))
        out = subprocess.run([sys.executable, os.path.join(root, "zero_dp_training.py"), "--model-name", "causal-tiny",
                              "--training-steps", "8", "--seq-len", "128", "--batch-size", "2", "--quiet",
                              "--no-memstats", "--graph", mode, "--stage", str(stage)],
                             env=env, capture_output=True, text=True, timeout=100, cwd=root)
        assert out.returncode == 0, out.stderr[-2000:]
        res[mode] = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][-1])
    assert res["on"]["hip_graph"] and not res["off"]["hip_graph"]
    assert res["on"]["final_loss"] == res["off"]["final_loss"]


def test_zero_script_graph_captures_bert_mlm_head():
    """zero_dp_training.py with a BERT model at world size 1 captures the step as a hipGraph: the
    sparse MLM head's labelled-row gather gets a static size (the script's causal-LM data labels
    every position) instead of a host-synchronising nonzero()."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(32000 + os.getpid() % 1000))
    r = subprocess.run([sys.executable, os.path.join(root, "zero_dp_training.py"), "--model-name", "bert-tiny",
                        "--stage", "2", "--batch-size", "2", "--training-steps", "8", "--seq-len", "128", "--quiet",
                        "--no-memstats"], cwd=root, env=env, capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{") and "tokens_per_s" in ln][-1]
    d = json.loads(line)
    assert d["hip_graph"] is True and d["stage"] == 2
    assert d["final_loss"] == d["final_loss"]   # finite (not NaN)


@pytest.mark.parametrize("mode", ["naive", "gpipe", "1f1b"])
def test_mp_script_graph_trains_like_eager(mode):
    """model_parallel_training.py with two virtual stages on one GPU: --graph (the whole step --
    every micro-batch forward/backward of both stages, loss, per-device optimizer, RNG advance --
    as one hipGraph) trains the same steps on the same batches as the eager issue."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    res = {}
    extra = [] if mode == "naive" else ["--pipeline", "--schedule", mode, "--checkpoint", "never"]
    for g in ("off", "on"):
        r = subprocess.run([sys.executable, os.path.join(root, "model_parallel_training.py"), "--model", "bert-tiny",
                            "--devices", "cuda:0,cuda:0", "--batch-size", "8", "--micro-batch-count", "4",
                            "--training-steps", "8", "--seq-len", "128", "--graph", g] + extra,
                           cwd=root, capture_output=True, text=True, timeout=150)
        assert r.returncode == 0, r.stderr[-3000:]
        res[g] = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert res["on"]["graph"] and not res["off"]["graph"]
    a, b = res["off"]["final_loss"], res["on"]["final_loss"]
    assert abs(a - b) <= 1e-3 * abs(a), (a, b)


@pytest.mark.parametrize("engine", ["ddp", "zero2", "zero3"])
def test_captured_step_with_rccl_collectives_matches_eager(engine):
    """The N > 1 data path inside a hipGraph: force_collectives makes DDP issue its bucket
    all-reduces (RCCL, from the autograd thread, on RCCL's stream) at world 1, ZeRO-2/3 their
    reduce-scatters and refresh all-gathers; the captured step (collectives included) replays
    exactly like the eager one.  rocprofv3 of bench.py --force-collectives shows the RCCL kernels in
    the step (profiles/r4_force_collectives_kernels.txt).  Inside a capture the ZeRO engine issues
    its collectives on the capturing stream (on a side stream hipStreamEndCapture crashes:
    scripts/diag/capture_collectives.py side_stream_rs) and defers their waits to the readers of
    the results, so in the graph each collective is a branch parallel to the following backward.

    The cases run in THIS process, after the captured ZeRO tests above (each creating and
    destroying its own RCCL group): that sequence is the regression test of the round-5 crash, a
    segfault in hipGraphLaunch on the first replay of the DDP graph.  Its cause was in the HIP
    runtime's multi-queue graph replay (hip::Graph::UpdateStreams read past its parallel-stream
    list when those streams shared the launch stream's hardware queue); the framework replays
    graphs on one queue (DEBUG_HIP_FORCE_GRAPH_QUEUES=1, set at package import and in conftest.py).
    DTD_RCCL_CAPTURE_INPROC=0 runs each case in a fresh process instead."""
    import os
    import subprocess
    import sys
    if os.environ.get("DTD_RCCL_CAPTURE_INPROC", "1") == "1":
        os.environ["MASTER_PORT"] = str(32000 + os.getpid() % 1000 + len(engine))
        _rccl_capture_case(engine)
        return
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(32000 + os.getpid() % 1000 + len(engine)))
    r = subprocess.run([sys.executable, "-c", f"import tests.test_graph_gpu as t; t._rccl_capture_case({engine!r})"],
                       cwd=root, env=env, capture_output=True, text=True, timeout=200)
    assert r.returncode == 0 and "RCCL_CAPTURE_OK" in r.stdout, (r.returncode, r.stdout[-2000:], r.stderr[-3000:])


def _rccl_capture_case(engine):
    import os
    from distributed_training_and_deepspeed_amd import comm
    from distributed_training_and_deepspeed_amd.parallel.zero import initialize
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    comm.init(rank=0, world_size=1, backend="nccl", local_rank=0)
    try:
        def setup():
            if engine == "ddp":
                model = build_model("tiny", dtype=torch.bfloat16, device="cuda", seed=3)
                model.rt.mlm_capacity = mlm_capacity(4 * 128)
                model.rt.mlm_overflow = torch.zeros((), dtype=torch.bool, device="cuda")
                ddp = DistributedDataParallel(model, bucket_cap_mb=0.25, force_collectives=True)
                assert ddp.collectives and len(ddp.buckets) > 2
                opt = hf_adamw(ddp.parameters(), lr=1e-3)

                def step(input_ids, labels):
                    out = ddp(input_ids, labels=labels)
                    out.loss.backward()
                    opt.step()
                    model.rt.rng.advance()
                    return out.loss.detach()
                return model, step
            model = build_model("causal-tiny", dtype=torch.bfloat16, device="cuda", seed=3)
            cfg = {"optimizer": {"type": "Adam", "params": {"lr": 1e-3}},
                   "zero_optimization": {"stage": int(engine[-1]), "reduce_bucket_size": 100000,
                                         "world1_replicated": False, "force_collectives": True}}
            eng, _, _, _ = initialize(model=model, model_parameters=model.parameters(), config=cfg)
            assert eng.collect

            def step(input_ids, labels):
                out = eng(input_ids, labels=labels)
                eng.backward(out.loss)
                eng.step()
                return out.loss.detach()
            return model, step

        mlm = engine == "ddp"
        cfg = build_model("tiny" if mlm else "causal-tiny").cfg
        ds = SyntheticLMDataset(cfg, 4 * 8, seq_len=128, mlm=mlm, seed=5)
        ids = ds.input_ids.view(8, 4, 128).cuda()
        lab = ds.labels.view(8, 4, 128).cuda()
        ma, sa = setup()
        mb, sb = setup()
        cap = CapturedStep(sb, {"input_ids": ids[0], "labels": lab[0]}, warmup=3, runtime=mb.rt)
        la = [sa(ids[0], lab[0]) for _ in range(3)]
        la += [sa(ids[i], lab[i]) for i in range(1, 6)]
        lb = [cap(input_ids=ids[i], labels=lab[i]).clone() for i in range(1, 6)]
        torch.cuda.synchronize()
        assert torch.equal(torch.stack(la[3:]), torch.stack(lb)), (la[3:], lb)
        print("RCCL_CAPTURE_OK", flush=True)
    finally:
        comm.destroy()
