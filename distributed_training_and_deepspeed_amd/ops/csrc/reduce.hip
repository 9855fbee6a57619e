// Split-K epilogue for the weight-gradient GEMMs (ops/grad.py::emit_wgrad).
//
// dW = dY^T X has a small output (e.g. 768 x 3072) and a huge K (= tokens), so the GEMM is run
// as s batched K-slices to fill the 256 CUs; this kernel folds the s partial products and lands
// the result in the gradient slot in ONE pass:  dst = (acc ? dst : 0) + sum_k parts[k]
// (fp32 accumulation, partials fp32 or bf16, dst fp32 or bf16 -- a view into the DDP/ZeRO flat
// gradient buffer).  It replaces the reduce + dtype-copy (+ accumulate) chain of three
// PyTorch kernels.  8 elements (16-32 B) per lane per access; grid-stride over n/8 vectors.
#include "common.h"

using namespace dtd;

namespace {

template <typename P, typename D, int VEC>
__global__ void __launch_bounds__(256) splitk_reduce_kernel(const P* __restrict__ parts, int s, size_t n,
                                                          D* __restrict__ dst, int acc) {
  const size_t nv = n / VEC;
  for (size_t v = (size_t)blockIdx.x * blockDim.x + threadIdx.x; v < nv; v += (size_t)gridDim.x * blockDim.x) {
    const size_t i = v * VEC;
    float t[VEC];
    if (acc) {
      vload<D, VEC>(dst + i, t);
    } else {
#pragma unroll
      for (int j = 0; j < VEC; ++j) t[j] = 0.f;
    }
    for (int k = 0; k < s; ++k) {
      float u[VEC];
      vload<P, VEC>(parts + (size_t)k * n + i, u);
#pragma unroll
      for (int j = 0; j < VEC; ++j) t[j] += u[j];
    }
    vstore<D, VEC>(dst + i, t);
  }
}

template <typename P, typename D>
void launch(const void* parts, int s, size_t n, void* dst, int acc, hipStream_t st) {
  const int vec = (n % 8 == 0) ? 8 : 1;
  const size_t nv = n / vec;
  const int grid = (int)std::min<size_t>((nv + 255) / 256, 256 * 8);
  if (vec == 8)
    hipLaunchKernelGGL((splitk_reduce_kernel<P, D, 8>), dim3(grid), dim3(256), 0, st, (const P*)parts, s, n, (D*)dst, acc);
  else
    hipLaunchKernelGGL((splitk_reduce_kernel<P, D, 1>), dim3(grid), dim3(256), 0, st, (const P*)parts, s, n, (D*)dst, acc);
}

}  // namespace

DTD_EXPORT int dtd_splitk_reduce(const void* parts, int pdt, int s, long long n, void* dst, int ddt, int acc,
                                 hipStream_t st) {
  if (n <= 0) return 0;
  if (pdt == kF32 && ddt == kBF16) launch<float, bf16>(parts, s, (size_t)n, dst, acc, st);
  else if (pdt == kF32 && ddt == kF32) launch<float, float>(parts, s, (size_t)n, dst, acc, st);
  else if (pdt == kBF16 && ddt == kBF16) launch<bf16, bf16>(parts, s, (size_t)n, dst, acc, st);
  else launch<bf16, float>(parts, s, (size_t)n, dst, acc, st);
  DTD_LAUNCH_CHECK();
}
