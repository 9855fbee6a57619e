"""Target script for the launcher tests: gloo all-reduce of the rank, result written per rank."""
import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist

p = argparse.ArgumentParser()
p.add_argument("--out", required=True)
p.add_argument("--fail-rank", type=int, default=-1)
args, unknown = p.parse_known_args()
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
if rank == args.fail_rank:
    sys.exit(3)
if args.fail_rank >= 0:
    time.sleep(120)      # must be terminated by the launcher's fail-fast
    sys.exit(0)
dist.init_process_group("gloo", rank=rank, world_size=world)
t = torch.tensor([float(rank + 1)])
dist.all_reduce(t)
with open(os.path.join(args.out, f"r{rank}.json"), "w") as f:
    json.dump({"sum": t.item(), "local_rank": int(os.environ["LOCAL_RANK"]), "unknown": unknown,
               "node_rank": int(os.environ["NODE_RANK"]), "local_world": int(os.environ["LOCAL_WORLD_SIZE"])}, f)
dist.destroy_process_group()
