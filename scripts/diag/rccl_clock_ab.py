"""Same-process A/B: a compute-bound bf16 GEMM loop and a memory-bound copy loop timed before
RCCL init, after comm.init (world 1, no collective issued) and after comm.destroy.  Round 4 s41:
after the communicator is created every kernel of the step runs 5-25 % longer with identical
L2 / HBM traffic and a lower shader clock (s40 PMC)."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402
from distributed_training_and_deepspeed_amd import comm  # noqa: E402

torch.cuda.set_device(0)
a = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
b = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)
x = torch.empty(512 << 20, device="cuda", dtype=torch.uint8)
y = torch.empty_like(x)


def timeit(fn, n):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n


def measure():
    g = timeit(lambda: a @ b, 100)
    c = timeit(lambda: y.copy_(x), 200)
    return {"gemm_tflops": round(2 * 8192 ** 3 / g / 1e12, 1), "copy_gbs": round(2 * x.numel() / c / 1e9, 1)}


res = {"before": measure(), "before2": measure()}
comm.init(rank=0, world_size=1, local_rank=0)
res["after_init"] = measure()
time.sleep(2)
res["after_init_2s"] = measure()
comm.destroy()
res["after_destroy"] = measure()
print(json.dumps(res), flush=True)
