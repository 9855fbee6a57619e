"""What process-wide HIP state does creating the RCCL communicator change?  Prints device limits,
flags and cache config before / after comm.init at world 1 (round 4 s37: the communicator's
creation alone slows every later kernel by ~10 %, and destroying it does not undo that)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402
from distributed_training_and_deepspeed_amd import comm  # noqa: E402

torch.cuda.set_device(0)
torch.zeros(1, device="cuda")
hip = ctypes.CDLL(next(ln.split()[-1] for ln in open("/proc/self/maps") if "libamdhip64" in ln))


def state():
    out = {}
    for name, lim in (("stack", 0), ("printf_fifo", 1), ("malloc_heap", 2)):
        v = ctypes.c_size_t()
        out[name] = (hip.hipDeviceGetLimit(ctypes.byref(v), ctypes.c_int(lim)), v.value)
        hip.hipGetLastError()   # an unsupported limit latches an error torch would raise later
    f = ctypes.c_uint()
    out["device_flags"] = (hip.hipGetDeviceFlags(ctypes.byref(f)), f.value)
    c = ctypes.c_int()
    out["cache_config"] = (hip.hipDeviceGetCacheConfig(ctypes.byref(c)), c.value)
    hip.hipGetLastError()
    out["env_changed"] = None
    return out


env0 = dict(os.environ)
s0 = state()
comm.init(rank=0, world_size=1, local_rank=0)
s1 = state()
s1["env_changed"] = {k: os.environ.get(k) for k in set(os.environ) ^ set(env0) | {k for k in env0 if os.environ.get(k) != env0[k]}}
print({"before": s0, "after": s1}, flush=True)
comm.destroy()
