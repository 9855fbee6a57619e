"""Does creating the RCCL communicator change the calling thread's CPU affinity?  Prints the
affinity before and after comm.init at world 1 (the N > 1 step's slowdown probe, round 4 s35)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402
from distributed_training_and_deepspeed_amd import comm  # noqa: E402

before = sorted(os.sched_getaffinity(0))
torch.cuda.set_device(0)
comm.init(rank=0, world_size=1, local_rank=0)
after = sorted(os.sched_getaffinity(0))
print({"before_n": len(before), "before": before[:8], "after_n": len(after), "after": after[:8],
       "changed": before != after}, flush=True)
comm.destroy()
