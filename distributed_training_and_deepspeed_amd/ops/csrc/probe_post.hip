// The post-communicator twin of probe.hip's kernel (see there): its own translation unit, so its
// code object is loaded by its first launch, after comm.init.
#include "probe_body.h"

DTD_EXPORT int dtd_probe_post(const float* x, float* y, size_t n, int blocks, hipStream_t s) {
  return probe_launch<1>(x, y, n, blocks, s);
}
