// Row softmax forward / backward: the standalone softmax of the instrumented
// TransformerBlock (reference model/transformer.py:43,81), which keeps every op a hookable
// module and therefore cannot use the fused flash-attention kernel.
//
//   fwd: y = exp(x - max) / sum(exp(x - max))           over the last dim (width n)
//   bwd: dx = y * (dy - sum(dy * y))
//
// One 64-lane wave per row; lanes stride the row in VEC-element (16 B for bf16x8) vectors.
// Rows up to 64*VEC*KMAX elements stay in registers (one HBM read, one write); wider rows take
// an online-softmax pass (running max/sum) and a second normalising pass.
#include "common.h"

using namespace dtd;

namespace {

constexpr int KMAX = 4;   // register-resident chunks per lane

template <typename T, int VEC>
__global__ void __launch_bounds__(256) softmax_fwd_kernel(const T* __restrict__ x, T* __restrict__ y, int rows, int n) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const T* xr = x + (size_t)row * n;
  T* yr = y + (size_t)row * n;
  const int step = 64 * VEC;
  const int nchunks = (n + step - 1) / step;
  if (nchunks <= KMAX) {
    float v[KMAX][VEC];
    float m = -INFINITY;
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
      const int c = k * step + lane * VEC;
      if (k < nchunks && c < n) {
        vload<T, VEC>(xr + c, v[k]);
#pragma unroll
        for (int j = 0; j < VEC; ++j) m = fmaxf(m, v[k][j]);
      }
    }
    m = wave_max(m);
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
      const int c = k * step + lane * VEC;
      if (k < nchunks && c < n) {
#pragma unroll
        for (int j = 0; j < VEC; ++j) { v[k][j] = __expf(v[k][j] - m); s += v[k][j]; }
      }
    }
    const float inv = 1.f / wave_sum(s);
#pragma unroll
    for (int k = 0; k < KMAX; ++k) {
      const int c = k * step + lane * VEC;
      if (k < nchunks && c < n) {
#pragma unroll
        for (int j = 0; j < VEC; ++j) v[k][j] *= inv;
        vstore<T, VEC>(yr + c, v[k]);
      }
    }
    return;
  }
  // wide rows: online max / sum, then normalise
  float m = -INFINITY, s = 0.f;
  for (int c = lane * VEC; c < n; c += step) {
    float t[VEC];
    vload<T, VEC>(xr + c, t);
    float cm = t[0];
#pragma unroll
    for (int j = 1; j < VEC; ++j) cm = fmaxf(cm, t[j]);
    const float nm = fmaxf(m, cm);
    s *= __expf(m - nm);
#pragma unroll
    for (int j = 0; j < VEC; ++j) s += __expf(t[j] - nm);
    m = nm;
  }
  const float gm = wave_max(m);
  s = wave_sum(s * __expf(m - gm));
  const float inv = 1.f / s;
  for (int c = lane * VEC; c < n; c += step) {
    float t[VEC];
    vload<T, VEC>(xr + c, t);
#pragma unroll
    for (int j = 0; j < VEC; ++j) t[j] = __expf(t[j] - gm) * inv;
    vstore<T, VEC>(yr + c, t);
  }
}

template <typename T, int VEC>
__global__ void __launch_bounds__(256) softmax_bwd_kernel(const T* __restrict__ y, const T* __restrict__ dy,
                                                          T* __restrict__ dx, int rows, int n) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const size_t off = (size_t)row * n;
  const int step = 64 * VEC;
  float d = 0.f;
  for (int c = lane * VEC; c < n; c += step) {
    float a[VEC], b[VEC];
    vload<T, VEC>(y + off + c, a);
    vload<T, VEC>(dy + off + c, b);
#pragma unroll
    for (int j = 0; j < VEC; ++j) d += a[j] * b[j];
  }
  d = wave_sum(d);
  for (int c = lane * VEC; c < n; c += step) {
    float a[VEC], b[VEC];
    vload<T, VEC>(y + off + c, a);
    vload<T, VEC>(dy + off + c, b);
#pragma unroll
    for (int j = 0; j < VEC; ++j) b[j] = a[j] * (b[j] - d);
    vstore<T, VEC>(dx + off + c, b);
  }
}

template <typename T>
void fwd(const void* x, void* y, int rows, int n, hipStream_t s) {
  dim3 g((rows + 3) / 4), b(256);
  if (n % 8 == 0) hipLaunchKernelGGL((softmax_fwd_kernel<T, 8>), g, b, 0, s, (const T*)x, (T*)y, rows, n);
  else hipLaunchKernelGGL((softmax_fwd_kernel<T, 1>), g, b, 0, s, (const T*)x, (T*)y, rows, n);
}

template <typename T>
void bwd(const void* y, const void* dy, void* dx, int rows, int n, hipStream_t s) {
  dim3 g((rows + 3) / 4), b(256);
  if (n % 8 == 0) hipLaunchKernelGGL((softmax_bwd_kernel<T, 8>), g, b, 0, s, (const T*)y, (const T*)dy, (T*)dx, rows, n);
  else hipLaunchKernelGGL((softmax_bwd_kernel<T, 1>), g, b, 0, s, (const T*)y, (const T*)dy, (T*)dx, rows, n);
}

}  // namespace

DTD_EXPORT int dtd_softmax_fwd(int dtype, const void* x, void* y, int rows, int n, hipStream_t s) {
  if (rows <= 0 || n <= 0) return 0;
  if (dtype == kBF16) fwd<bf16>(x, y, rows, n, s);
  else fwd<float>(x, y, rows, n, s);
  DTD_LAUNCH_CHECK();
}

DTD_EXPORT int dtd_softmax_bwd(int dtype, const void* y, const void* dy, void* dx, int rows, int n, hipStream_t s) {
  if (rows <= 0 || n <= 0) return 0;
  if (dtype == kBF16) bwd<bf16>(y, dy, dx, rows, n, s);
  else bwd<float>(y, dy, dx, rows, n, s);
  DTD_LAUNCH_CHECK();
}
