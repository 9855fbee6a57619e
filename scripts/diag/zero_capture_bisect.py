#!/usr/bin/env python
"""Bisect the ZeRO capture crash with RCCL collectives (world 1, force_collectives): each variant
captures a causal-tiny ZeRO step in its own child process and reports whether capture + replay
survive (variants *_nostream drop the comm stream by hand; the engine now does that itself while
capturing -- every variant passed on the box, profiles/r4_s12_results.jsonl)."""
import json
import os
import subprocess
import sys

VARIANTS = {
    "s1_fwd_bwd_only": {"stage": 1, "_part": "fb"},
    "s1_step_only": {"stage": 1, "_part": "step"},
    "s1_fwd_only": {"stage": 1, "_part": "f"},
    "s1_fwd_bwd_nostream": {"stage": 1, "_part": "fb", "_nostream": True},
    "s1_step_only_nostream": {"stage": 1, "_part": "step", "_nostream": True},
    "s2_nostream": {"stage": 2, "_nostream": True},
    "s1": {"stage": 1},
    "s2": {"stage": 2},
    "s3": {"stage": 3},
    "s2_no_overlap_comm": {"stage": 2, "overlap_comm": False},
    "s2_no_refresh_overlap": {"stage": 2, "overlap_param_refresh": False},
    "s2_neither": {"stage": 2, "overlap_comm": False, "overlap_param_refresh": False},
    "s2_one_bucket": {"stage": 2, "reduce_bucket_size": 10 ** 9, "allgather_bucket_size": 10 ** 9},
}


def child(name):
    import torch
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
    from distributed_training_and_deepspeed_amd import comm
    from distributed_training_and_deepspeed_amd.data import SyntheticLMDataset
    from distributed_training_and_deepspeed_amd.models import build_model
    from distributed_training_and_deepspeed_amd.parallel.zero import initialize
    from distributed_training_and_deepspeed_amd.utils.graphs import CapturedStep
    comm.init(rank=0, world_size=1, backend="nccl", local_rank=0)
    z = {"reduce_bucket_size": 100000, "world1_replicated": False, "force_collectives": True}
    z.update(VARIANTS[name])
    part = z.pop("_part", "all")
    nostream = z.pop("_nostream", False)
    model = build_model("causal-tiny", dtype=torch.bfloat16, device="cuda", seed=3)
    cfg = {"optimizer": {"type": "Adam", "params": {"lr": 1e-3}}, "zero_optimization": z}
    eng, _, _, _ = initialize(model=model, model_parameters=model.parameters(), config=cfg)
    if nostream:                                # collectives on the capturing stream itself
        eng.comm_stream = None
    ds = SyntheticLMDataset(model.cfg, 4 * 4, seq_len=128, mlm=False, seed=5)
    ids, lab = ds.input_ids.view(4, 4, 128).cuda(), ds.labels.view(4, 4, 128).cuda()

    def step(input_ids, labels):
        out = eng(input_ids, labels=labels)
        eng.backward(out.loss)
        eng.step()
        return out.loss.detach()
    for i in range(2):                          # eager warm-up: communicator, arenas, solutions
        step(ids[i], lab[i])
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    if part == "step":
        out = eng(ids[0], labels=lab[0])
        eng.backward(out.loss)
        torch.cuda.synchronize()
        with torch.cuda.graph(g):
            eng.step()
        loss = out.loss.detach()
    elif part in ("fb", "f"):
        with torch.cuda.graph(g):
            out = eng(ids[0], labels=lab[0])
            if part == "fb":
                eng.backward(out.loss)
            loss = out.loss.detach()
    else:
        cap = CapturedStep(step, {"input_ids": ids[0], "labels": lab[0]}, warmup=1, runtime=model.rt)
        loss = cap(input_ids=ids[1], labels=lab[1])
    if part != "all":
        g.replay()
    torch.cuda.synchronize()
    print(json.dumps({"variant": name, "ok": True, "loss": float(loss)}), flush=True)
    comm.destroy()


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "--child":
        child(sys.argv[2])
        return
    names = sys.argv[1:] or list(VARIANTS)
    for i, name in enumerate(names):
        env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(29700 + i))
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", name], env=env,
                           capture_output=True, text=True, timeout=150)
        ok = r.returncode == 0 and '"ok": true' in r.stdout
        tail = "" if ok else " | ".join(r.stderr.strip().splitlines()[-3:])[:400]
        print(json.dumps({"variant": name, "ok": ok, "returncode": r.returncode, "err": tail}), flush=True)
        if r.returncode < 0 or r.returncode >= 128:   # a crashed child: start nothing more on the GPU
            print(json.dumps({"stopped_after": r.returncode}), flush=True)
            sys.exit(3)


if __name__ == "__main__":
    main()
