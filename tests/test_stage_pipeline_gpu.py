"""One pipeline stage per process on the GPU (parallel/stage_pipeline.py).

Two ranks share cuda:0 over gloo (RCCL refuses two ranks on one device; the 8-GPU node uses RCCL
send/recv), each running its stage with the native fp32 kernels; the stage gradients must match
the sequential fp32 model's (CPU reference ops) for GPipe and 1F1B.  The entry script's
stage-per-process mode (model_parallel_training.py under torchrun) must run with the native
library loaded and report the stage-per-process mode.  Reference: model/bert_mp.py:39-47,73-99,
model_parallel_training.py:43-44,65-78.
"""
import json
import os
import subprocess
import sys

import pytest
import torch
import torch.multiprocessing as mp

from .test_stage_pipeline_cpu import _sequential, _worker

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("schedule", ["gpipe", "1f1b"])
def test_two_stage_processes_share_one_gpu(tmp_path, free_port, schedule):
    mp.spawn(_worker, args=(2, free_port, str(tmp_path), schedule, "cuda:0", "auto"), nprocs=2, join=True)
    ref, ref_loss = _sequential()
    seen = set()
    for r in range(2):
        res = torch.load(tmp_path / f"stage{r}.pt", weights_only=True)
        for n, g in res["grads"].items():
            err = ((g - ref[n]).norm() / (ref[n].norm() + 1e-12)).item()
            assert err < 2e-3, (schedule, r, n, err)
            seen.add(n)
        if r == 1:
            assert abs(float(res["loss"]) - ref_loss) < 1e-3 * abs(ref_loss)
    assert seen == set(ref)


def test_entry_script_stage_per_process(free_port):
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, DTD_NO_BUILD="1")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(free_port),
                        os.path.join(root, "model_parallel_training.py"), "--model", "bert-tiny", "--batch-size", "8",
                        "--training-steps", "5", "--seq-len", "64", "--pipeline", "--micro-batch-count", "4",
                        "--schedule", "1f1b", "--pipe-backend", "gloo"],
                       capture_output=True, text=True, timeout=240, env=env, cwd=root)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
    res = json.loads(line)
    assert res["mode"] == "stage-per-process" and res["stages"] == 2 and res["transport"] == "gloo"
    assert res["final_loss"] is not None and res["final_loss"] == res["final_loss"]
