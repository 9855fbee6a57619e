// Body of the post-communicator kernel probe (probe.hip / probe_post.hip): one kernel per
// translation unit, so each twin is its own code object and is loaded by its own first launch --
// probe_post.hip's only after comm.init.  The kernel streams a buffer through HBM (16-byte loads
// and stores, y = a x + b): in round 4's slow runs the memory-bound kernels were the ones hit
// (split-K reduce and column-sum finalize 3x, LayerNorm +15-30 %, profiles/r4_s38_rccl_init_kernels.txt),
// and compute-loop probes -- in or out of the instruction cache -- showed no difference.
#pragma once
#include "common.h"

namespace {

typedef float f32x4p __attribute__((ext_vector_type(4)));

template <int ID>
__global__ void __launch_bounds__(256) probe_kernel(const f32x4p* __restrict__ x, f32x4p* __restrict__ y, size_t n4) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += stride) {
    const f32x4p v = x[i];
    y[i] = v * 1.0001f + (float)(ID + 1);
  }
}

template <int ID>
int probe_launch(const float* x, float* y, size_t n, int blocks, hipStream_t s) {
  if (blocks <= 0 || !x || !y || n % 4) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(probe_kernel<ID>, dim3(blocks), dim3(256), 0, s, (const f32x4p*)x, (f32x4p*)y, n / 4);
  DTD_LAUNCH_CHECK();
}

}  // namespace
