// Post-communicator kernel probe (bench.py, utils/prewarm.py::KernelProbe).
//
// Round 4 measured that kernels launched for the FIRST time after the RCCL communicator is created
// (ncclCommInitRank) run 5-25 % slower for the life of the process -- same L2 / HBM traffic, more
// cycles, microsecond kernels hit hardest (profiles/r4_s30_s46_rccl_init.jsonl).  The entry scripts
// work around it by running the step's kernels once before comm.init (utils/prewarm.py), which
// only covers what that throwaway step launches.  This probe detects the effect in a run: two
// code-identical kernels in separate translation units (so separate code objects, each loaded by
// its own first launch): this one first launched before comm.init, probe_post.hip's after it --
// timed back to back after the init.  A ratio
// t1 / t0 above 1.05 means kernels first used after the init (a hipBLASLt solution for another
// shape, a ZeRO-3 gather-path kernel) run slow in this process.
//
// The body (probe_body.h) streams a buffer through HBM: the memory-bound kernels are the ones the
// effect hits.
#include "probe_body.h"

DTD_EXPORT int dtd_probe(const float* x, float* y, size_t n, int blocks, hipStream_t s) {
  return probe_launch<0>(x, y, n, blocks, s);
}
