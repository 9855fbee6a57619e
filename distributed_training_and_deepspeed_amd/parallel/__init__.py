"""Parallelism strategies: DDP (bucketed RCCL all-reduce), ZeRO stages 0-3, layer-wise model
parallelism and GPipe pipelining, on flat MI355X-resident buffers."""
from .ddp import DistributedDataParallel  # noqa: F401
from .flat import FlatLayout, GradBuffer  # noqa: F401
