"""bench.py driver contract on CPU: launched exactly as the driver does (torch.distributed.run,
one rank per device, gloo here), rank 0 prints ONE JSON line with the whole-job tokens/s."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
        "vs_baseline", "dtype", "data", "config"}


def _run(port, *extra, nproc=2):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", str(nproc),
           "--steps", "2", "--warmup", "1", "--batch-size", "2", "--seq-len", "64", *extra]
    env = dict(os.environ, OMP_NUM_THREADS="2")
    out = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=600, env=env)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.parametrize("extra,engine", [(("--model", "tiny"), "DDP"),
                                          (("--model", "tiny", "--zero-stage", "2"), "ZeRO-2")])
def test_bench_json_line_world2(free_port, extra, engine):
    r = _run(free_port, *extra)
    assert KEYS <= set(r)
    assert r["n_gpus"] == 2 and r["steps"] == 2 and r["warmup"] == 1
    assert r["higher_is_better"] is True and r["scaling"] == "weak"
    assert engine in r["metric"]
    cfg = r["config"]
    assert cfg["global_batch"] == 4 and cfg["seq_len"] == 64
    # value is the whole-job rate: world * batch * seq tokens per step over the (max-rank) step time
    assert r["value"] == pytest.approx(4 * 64 / (r["ms_per_step"] / 1e3), rel=2e-3)
