"""RCCL busbw sweep harness (bench/comm_sweep.py) rehearsed on gloo: bandwidth law and bucket pick."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bench"))

import comm_sweep  # noqa: E402


def test_busbw_law_and_recommendation():
    assert comm_sweep.busbw_factor("all_reduce", 8) == 2 * 7 / 8
    assert comm_sweep.busbw_factor("all_gather_into_tensor", 8) == 7 / 8
    rows = [{"op": "all_reduce", "bytes": 1 << k, "busbw_GBps": bw} for k, bw in
            [(20, 10.0), (22, 50.0), (24, 91.0), (26, 100.0), (28, 99.0)]]
    rec = comm_sweep.recommend_bucket(rows)
    assert rec["bucket_bytes"] == 1 << 24 and rec["peak_busbw_GBps"] == 100.0


def test_sweep_runs_on_gloo(tmp_path):
    out = tmp_path / "sweep.json"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench", "comm_sweep.py"), "--nproc", "2", "--backend",
                        "gloo", "--max-bytes", "65536", "--min-bytes", "4096", "--iters", "2", "--warmup", "1",
                        "--dtype", "fp32", "--recommend", "--out", str(out)],
                       capture_output=True, text=True, timeout=240, env={**os.environ, "MASTER_ADDR": "127.0.0.1"})
    assert r.returncode == 0, r.stderr[-2000:]
    res = json.loads(out.read_text())
    assert len(res["rows"]) == 4 * 5 and all(x["world"] == 2 and x["ms"] > 0 for x in res["rows"])
    assert res["recommended_bucket"]["bucket_bytes"] >= 4096
