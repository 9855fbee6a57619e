// Fused Adam / AdamW step over flat parameter buffers, plus the flat-buffer utility kernels
// (scale+cast for gradient buckets, squared L2 norm partials for clipping).
//
// Replaces DeepSpeed FusedAdam (`multi_tensor_adam.cu`, selected by zero_dp_training.py:28-33),
// torch AdamW foreach kernels (model_parallel_training.py:50) and the per-parameter Python loop
// of transformers.AdamW (data_parallel_training.py:34) -- SURVEY.md D12/D21/K9.
//
// The framework keeps parameters, fp32 master weights, moments and gradients in flat buffers,
// so one launch updates the whole model (or the local ZeRO partition): 16 B per lane per
// stream, HBM-bound at ~28 B/param.  Hyper-parameters are read from a small device array so
// a hipGraph replay sees the current step (bias correction) and a device-computed gradient
// scale (1/world, clipping) without host round trips:
//   hp[0] lr   hp[1] beta1   hp[2] beta2   hp[3] eps   hp[4] weight_decay
//   hp[5] step (already incremented for this update)   hp[6] grad scale
// mode bits: 1 = decoupled weight decay (AdamW; else L2 added to the gradient),
//            2 = bias correction,
//            4 = HF transformers eps placement: p -= lr*sqrt(bc2)/bc1 * m / (sqrt(v) + eps)
//                (torch / DeepSpeed: p -= lr/bc1 * m / (sqrt(v)/sqrt(bc2) + eps)).
#include "common.h"

using namespace dtd;

namespace {

struct AdamArgs {
  float* p; float* m; float* v; const void* g; bf16* p_lp; size_t n; const float* hp; int mode; int g_dtype;
};

// Contraction off: the same element must round identically in the 8-wide body and in the scalar
// tail (a staged update launches per stage span, so an element can be a tail element in one launch
// and a vector element in the whole-buffer launch; with the compiler free to fuse multiply-adds
// differently in the two contexts the results differed in the last bit -- r5 s19).
__device__ __forceinline__ void adam_elem(float& p, float& m, float& v, float g, float lr, float b1, float b2,
                                          float eps, float wd, float bc1, float bc2_sqrt, int mode) {
#pragma clang fp contract(off)
  if (!(mode & 1) && wd != 0.f) g += wd * p;
  m = b1 * m + (1.f - b1) * g;
  v = b2 * v + (1.f - b2) * g * g;
  if (mode & 1) p -= lr * wd * p;
  if (mode & 4) {
    const float step = lr * bc2_sqrt / bc1;
    p -= step * m / (sqrtf(v) + eps);
  } else {
    const float denom = sqrtf(v) / bc2_sqrt + eps;
    p -= (lr / bc1) * m / denom;
  }
}

typedef float f32x4 __attribute__((ext_vector_type(4)));

// One 8-element group per thread (no grid-stride loop) with non-temporal 16-byte stores: every
// byte is touched exactly once, and a flat grid keeps more bytes in flight per CU than a
// 2048-block grid-stride loop (the same change moved the streaming GELU / LayerNorm kernels from
// ~4.9 to ~6 TB/s, profiles/r1_elementwise_roofline.jsonl).  The loads are plain: with four
// read streams and four write streams per element, cached loads measured 5.24-5.26 TB/s against
// 5.05-5.09 for non-temporal ones at 1-2 G elements (profiles/r6_adam_forms.jsonl).
template <bool NT, typename V>
__device__ __forceinline__ V ld(const V* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}

// ILP: independent 8-element groups per thread (all loads issued before any math: more bytes in
// flight per wave); NTL: non-temporal loads (stores are always non-temporal).
template <bool GBF16, int ILP = 1, bool NTL = true>
__global__ void __launch_bounds__(256) adam_kernel(AdamArgs a) {
  const float lr = a.hp[0], b1 = a.hp[1], b2 = a.hp[2], eps = a.hp[3], wd = a.hp[4];
  const float step = a.hp[5], gs = a.hp[6];
  float bc1 = 1.f, bc2s = 1.f;
  if (a.mode & 2) {
    bc1 = 1.f - powf(b1, step);
    bc2s = sqrtf(1.f - powf(b2, step));
  }
  const size_t ng = a.n / 8;
  const size_t base = (size_t)blockIdx.x * blockDim.x * ILP + threadIdx.x;
  f32x4 p0[ILP], p1[ILP], m0[ILP], m1[ILP], v0[ILP], v1[ILP];
  float g[ILP][8];
#pragma unroll
  for (int u = 0; u < ILP; ++u) {
    const size_t i = base + (size_t)u * blockDim.x;
    if (i < ng) {
      const f32x4* P = reinterpret_cast<const f32x4*>(a.p) + 2 * i;
      const f32x4* M = reinterpret_cast<const f32x4*>(a.m) + 2 * i;
      const f32x4* V = reinterpret_cast<const f32x4*>(a.v) + 2 * i;
      p0[u] = ld<NTL>(P); p1[u] = ld<NTL>(P + 1);
      m0[u] = ld<NTL>(M); m1[u] = ld<NTL>(M + 1);
      v0[u] = ld<NTL>(V); v1[u] = ld<NTL>(V + 1);
      if constexpr (GBF16) {
        if constexpr (NTL) vload_nt<bf16, 8>((const bf16*)a.g + i * 8, g[u]);
        else vload<bf16, 8>((const bf16*)a.g + i * 8, g[u]);
      } else {
        const f32x4* G = reinterpret_cast<const f32x4*>(a.g) + 2 * i;
        const f32x4 g0 = ld<NTL>(G), g1 = ld<NTL>(G + 1);
#pragma unroll
        for (int j = 0; j < 4; ++j) { g[u][j] = g0[j]; g[u][4 + j] = g1[j]; }
      }
    }
  }
#pragma unroll
  for (int u = 0; u < ILP; ++u) {
    const size_t i = base + (size_t)u * blockDim.x;
    if (i < ng) {
      float q[8], mm[8], vv[8];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        q[j] = p0[u][j]; q[4 + j] = p1[u][j];
        mm[j] = m0[u][j]; mm[4 + j] = m1[u][j];
        vv[j] = v0[u][j]; vv[4 + j] = v1[u][j];
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) adam_elem(q[j], mm[j], vv[j], g[u][j] * gs, lr, b1, b2, eps, wd, bc1, bc2s, a.mode);
      f32x4 o0, o1, n0, n1, w0, w1;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        o0[j] = q[j]; o1[j] = q[4 + j];
        n0[j] = mm[j]; n1[j] = mm[4 + j];
        w0[j] = vv[j]; w1[j] = vv[4 + j];
      }
      f32x4* P = reinterpret_cast<f32x4*>(a.p) + 2 * i;
      f32x4* M = reinterpret_cast<f32x4*>(a.m) + 2 * i;
      f32x4* V = reinterpret_cast<f32x4*>(a.v) + 2 * i;
      __builtin_nontemporal_store(o0, P); __builtin_nontemporal_store(o1, P + 1);
      __builtin_nontemporal_store(n0, M); __builtin_nontemporal_store(n1, M + 1);
      __builtin_nontemporal_store(w0, V); __builtin_nontemporal_store(w1, V + 1);
      if (a.p_lp) vstore_nt<bf16, 8>(a.p_lp + i * 8, q);
    }
  }
  // tail (n % 8 elements): the first threads of the last block
  const size_t e = ng * 8 + threadIdx.x;
  if (blockIdx.x == gridDim.x - 1 && e < a.n) {
    float gt = GBF16 ? (float)((const bf16*)a.g)[e] : ((const float*)a.g)[e];
    adam_elem(a.p[e], a.m[e], a.v[e], gt * gs, lr, b1, b2, eps, wd, bc1, bc2s, a.mode);
    if (a.p_lp) a.p_lp[e] = (bf16)a.p[e];
  }
}

template <typename S, typename D>
__global__ void __launch_bounds__(256) scale_cast_kernel(const S* __restrict__ src, D* __restrict__ dst, size_t n,
                                                         float scale, const float* __restrict__ dscale) {
  const float sc = dscale ? scale * dscale[0] : scale;
  const size_t nv = n / 8;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nv; i += (size_t)gridDim.x * blockDim.x) {
    float t[8];
    vload<S, 8>(src + i * 8, t);
#pragma unroll
    for (int j = 0; j < 8; ++j) t[j] *= sc;
    vstore<D, 8>(dst + i * 8, t);
  }
  if (blockIdx.x == 0)
    for (size_t e = nv * 8 + threadIdx.x; e < n; e += blockDim.x) dst[e] = (D)((float)src[e] * sc);
}

// Per-block partial sums of x^2 (fp32), written to part[blockIdx.x].
template <typename S>
__global__ void __launch_bounds__(256) sqnorm_kernel(const S* __restrict__ x, size_t n, float* __restrict__ part) {
  __shared__ float sh[8];
  float acc = 0.f;
  const size_t nv = n / 8;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nv; i += (size_t)gridDim.x * blockDim.x) {
    float t[8];
    vload<S, 8>(x + i * 8, t);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += t[j] * t[j];
  }
  if (blockIdx.x == 0)
    for (size_t e = nv * 8 + threadIdx.x; e < n; e += blockDim.x) { float t = (float)x[e]; acc += t * t; }
  acc = block_sum(acc, sh);
  if (threadIdx.x == 0) part[blockIdx.x] = acc;
}

size_t grid_for(size_t nvec) {
  size_t b = (nvec + 255) / 256;
  if (b < 1) b = 1;
  if (b > 2048) b = 2048;
  return b;
}

}  // namespace

DTD_EXPORT int dtd_adam_step(float* p, float* m, float* v, const void* g, int g_dtype, void* p_lp, size_t n,
                             const float* hp, int mode, hipStream_t s) {
  if (n == 0) return 0;
  AdamArgs a{p, m, v, g, (bf16*)p_lp, n, hp, mode, g_dtype};
  // DTD_ADAM_FORM (measurement knob): 1c (default) = one 8-element group per thread, cached
  // loads; 2c = two groups per thread; 1 / 2 = the same with non-temporal loads
  const char* fe = getenv("DTD_ADAM_FORM");
  const int form = fe ? (fe[0] == '2' ? 2 : 1) + (fe[0] && fe[1] == 'c' ? 10 : 0) : 11;
  const int ilp = form % 10;
  // 8 elements per thread and group; at least one block so the tail always has an owner
  const size_t per = 256 * (size_t)ilp;
  const size_t blocks = (n / 8 + per - 1) / per > 0 ? (n / 8 + per - 1) / per : 1;
  const bool bf = g_dtype == kBF16;
  switch (form) {
    case 2: if (bf) hipLaunchKernelGGL((adam_kernel<true, 2, true>), dim3(blocks), dim3(256), 0, s, a);
            else hipLaunchKernelGGL((adam_kernel<false, 2, true>), dim3(blocks), dim3(256), 0, s, a); break;
    case 11: if (bf) hipLaunchKernelGGL((adam_kernel<true, 1, false>), dim3(blocks), dim3(256), 0, s, a);
             else hipLaunchKernelGGL((adam_kernel<false, 1, false>), dim3(blocks), dim3(256), 0, s, a); break;
    case 12: if (bf) hipLaunchKernelGGL((adam_kernel<true, 2, false>), dim3(blocks), dim3(256), 0, s, a);
             else hipLaunchKernelGGL((adam_kernel<false, 2, false>), dim3(blocks), dim3(256), 0, s, a); break;
    default: if (bf) hipLaunchKernelGGL((adam_kernel<true, 1, true>), dim3(blocks), dim3(256), 0, s, a);
             else hipLaunchKernelGGL((adam_kernel<false, 1, true>), dim3(blocks), dim3(256), 0, s, a); break;
  }
  DTD_LAUNCH_CHECK();
}

DTD_EXPORT int dtd_scale_cast(const void* src, int src_dtype, void* dst, int dst_dtype, size_t n, float scale,
                              const float* dscale, hipStream_t s) {
  if (n == 0) return 0;
  dim3 grid(grid_for(n / 8));
  if (src_dtype == kBF16 && dst_dtype == kBF16)
    hipLaunchKernelGGL((scale_cast_kernel<bf16, bf16>), grid, dim3(256), 0, s, (const bf16*)src, (bf16*)dst, n, scale, dscale);
  else if (src_dtype == kBF16)
    hipLaunchKernelGGL((scale_cast_kernel<bf16, float>), grid, dim3(256), 0, s, (const bf16*)src, (float*)dst, n, scale, dscale);
  else if (dst_dtype == kBF16)
    hipLaunchKernelGGL((scale_cast_kernel<float, bf16>), grid, dim3(256), 0, s, (const float*)src, (bf16*)dst, n, scale, dscale);
  else
    hipLaunchKernelGGL((scale_cast_kernel<float, float>), grid, dim3(256), 0, s, (const float*)src, (float*)dst, n, scale, dscale);
  DTD_LAUNCH_CHECK();
}

DTD_EXPORT int dtd_sqnorm_num_partials(size_t n) { return (int)grid_for(n / 8); }

DTD_EXPORT int dtd_sqnorm_partials(const void* x, int dtype, size_t n, float* part, hipStream_t s) {
  dim3 grid(grid_for(n / 8));
  if (dtype == kBF16) hipLaunchKernelGGL(sqnorm_kernel<bf16>, grid, dim3(256), 0, s, (const bf16*)x, n, part);
  else hipLaunchKernelGGL(sqnorm_kernel<float>, grid, dim3(256), 0, s, (const float*)x, n, part);
  DTD_LAUNCH_CHECK();
}
