#!/usr/bin/env python
"""Limiter probe of the four-wave GEMM (ops/csrc/gemm4.hip): the same product timed with parts of
the main loop removed (DTD_GEMM4_DIAG builds; timing only, results wrong): no barrier, L2-hot
loads, no LDS staging stores, no loads.  One process per variant (the diag value is read once),
run back to back; compare against the full kernel and hipBLASLt in the same process."""
import json
import os
import statistics
import subprocess
import sys

CODE = r'''
import json, os, statistics, sys, torch
sys.path.insert(0, os.getcwd())
from distributed_training_and_deepspeed_amd.ops import gemm as G
T, H, F = 131072, 768, 3072
x = torch.randn(T, H, device="cuda", dtype=torch.bfloat16)
w = {"qkv": torch.randn(3 * H, H, device="cuda", dtype=torch.bfloat16), "fc1": torch.randn(F, H, device="cuda", dtype=torch.bfloat16)}
def timed(fn, reps=10):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn(); torch.cuda.synchronize(); s.record()
    for _ in range(reps): fn()
    e.record(); torch.cuda.synchronize(); return s.elapsed_time(e) / reps * 1e3
out = {}
for n, ww in w.items():
    ts = [timed(lambda: G.gemm4_bt(x, ww)) for _ in range(5)]
    hb = [timed(lambda: torch.nn.functional.linear(x, ww)) for _ in range(5)]
    out[n] = {"gemm4_us": round(statistics.median(ts), 1), "hipblaslt_us": round(statistics.median(hb), 1)}
print(json.dumps({"form": int(os.environ.get("DTD_GEMM4_FORM", "1")), "diag": int(os.environ.get("DTD_GEMM4_DIAG", "0")), **out}), flush=True)
'''

for form, d in ((0, 0), (1, 0), (0, 1), (0, 2), (0, 4), (0, 8), (0, 15), (1, 1), (1, 2), (1, 4), (1, 8), (1, 15)):
    env = dict(os.environ, DTD_GEMM4_DIAG=str(d), DTD_GEMM4_FORM=str(form))
    r = subprocess.run([sys.executable, "-c", CODE], env=env, capture_output=True, text=True, timeout=240)
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    print(line[-1] if line else json.dumps({"form": form, "diag": d, "error": r.stderr[-500:]}), flush=True)
    if r.returncode != 0:
        sys.exit(r.returncode)
