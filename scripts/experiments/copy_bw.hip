// HBM streaming ceiling on one MI355X: variants of a bf16 "y = f(x)" pass (16-byte vectors),
// to choose the load/store form of the elementwise kernels.  Prints GB/s (read + write bytes).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int U, bool NT>
__global__ void __launch_bounds__(256) copy_k(const u32x4* __restrict__ x, u32x4* __restrict__ y, size_t n) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  for (; i + (U - 1) * stride < n; i += U * stride) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = NT ? __builtin_nontemporal_load(x + i + u * stride) : x[i + u * stride];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (NT) __builtin_nontemporal_store(v[u], y + i + u * stride);
      else y[i + u * stride] = v[u];
    }
  }
  for (; i < n; i += stride) y[i] = x[i];
}

template <int U, bool NT>
float run(const u32x4* x, u32x4* y, size_t n, int blocks) {
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  for (int i = 0; i < 3; ++i) hipLaunchKernelGGL((copy_k<U, NT>), dim3(blocks), dim3(256), 0, 0, x, y, n);
  hipEventRecord(a);
  const int iters = 20;
  for (int i = 0; i < iters; ++i) hipLaunchKernelGGL((copy_k<U, NT>), dim3(blocks), dim3(256), 0, 0, x, y, n);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return (float)(2.0 * n * 16 * iters / (ms * 1e-3) / 1e9);
}

int main() {
  const size_t bytes = 402653184;  // [65536, 3072] bf16
  const size_t n = bytes / 16;
  u32x4 *x, *y;
  hipMalloc(&x, bytes); hipMalloc(&y, bytes);
  hipMemset(x, 1, bytes);
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const int grids[] = {cus * 8, cus * 16, cus * 32, (int)((n + 255) / 256)};
  for (int g : grids) {
    printf("blocks %7d  U1 %6.0f  U2 %6.0f  U4 %6.0f  | nt U1 %6.0f  U2 %6.0f  U4 %6.0f GB/s\n", g,
           run<1, false>(x, y, n, g), run<2, false>(x, y, n, g), run<4, false>(x, y, n, g),
           run<1, true>(x, y, n, g), run<2, true>(x, y, n, g), run<4, true>(x, y, n, g));
  }
  return 0;
}
