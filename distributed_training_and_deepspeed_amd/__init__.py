"""MI355X-native distributed training (DDP, GPipe / stage-per-process pipelines, ZeRO 0-3) with
hand-written gfx950 kernels; see README.md."""
import os as _os

# hipGraph replay on ONE hardware queue (read by the HIP runtime when it initialises, so it is set
# at import, before any HIP call).  Round 6, profiles/r6_graph_queues.jsonl: the runtime's
# multi-queue replay (a stream per parallel branch of the graph, event joins between them) ran the
# captured BERT-base b4 step at 107-110 k tokens/s against 302 k on one queue, and on the first
# launch of a graph whose parallel streams shared the launch stream's hardware queue it indexed
# past its parallel-stream list and segfaulted inside hipGraphLaunch (hip::Graph::UpdateStreams,
# native backtrace in docs/PERFORMANCE.md) -- the in-process RCCL-capture crash of round 5.
_os.environ.setdefault("DEBUG_HIP_FORCE_GRAPH_QUEUES", "1")
