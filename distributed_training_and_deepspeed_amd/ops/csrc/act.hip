// Activation (GELU-erf / GELU-tanh / ReLU) forward and backward with fused bias-gradient
// column partials, plus the deterministic column-sum finaliser used by every kernel that
// produces parameter-gradient partials (LayerNorm gamma/beta, Linear biases).
//
// Reference ops replaced: HF BertIntermediate `gelu` (erf), BLOOM/GPT-2 tanh-GELU, OPT/
// TransformerBlock ReLU (reference model/transformer.py:52,101) and the implicit
// `bias.grad = dY.sum(0)` reductions of every nn.Linear (SURVEY.md K5, K1 epilogues).
// The Linear bias itself is added by the hipBLASLt epilogue of the producing GEMM, so the
// forward here is a pure elementwise pass over the pre-activation `u`.
#include "common.h"

using namespace dtd;

namespace {

enum Act : int { kNone = 0, kGeluErf = 1, kGeluTanh = 2, kRelu = 3 };

// Standard-normal CDF Phi(x) = 0.5 (1 + erf(x / sqrt 2)) from one exponential: Abramowitz &
// Stegun 7.1.26 (|erf error| <= 1.5e-7, far below the bf16 rounding of the outputs) with
// e = exp(-x^2 / 2), which is also the Gaussian density the GELU derivative needs -- one v_exp,
// one v_rcp and a handful of FMAs instead of the libm erff's branches and polynomials (the
// GELU passes are VALU-, not HBM-bound with the libm form).
__device__ __forceinline__ float phi_cdf(float x, float e) {
  // t = 1 / (1 + p |x| / sqrt 2): one FMA with an |x| source modifier
  const float t = __builtin_amdgcn_rcpf(fmaf(fabsf(x), 0.3275911f * 0.70710678118654752f, 1.f));
  const float poly = t * fmaf(t, fmaf(t, fmaf(t, fmaf(t, 1.061405429f, -1.453152027f), 1.421413741f), -0.284496736f),
                              0.254829592f);
  const float erfa = 1.f - poly * e;                  // erf(|x| / sqrt 2)
  return 0.5f + 0.5f * copysignf(erfa, x);
}
// exp(-x^2 / 2) as v_exp_f32 (= 2^y) of y = x^2 * (-log2(e) / 2): two multiplies (packable)
__device__ __forceinline__ float gauss_e(float x) { return __builtin_amdgcn_exp2f((x * x) * -0.72134752044448170f); }
// tanh(y) = 1 - 2 / (1 + e^{2y}): one v_exp + one v_rcp; saturates correctly at +-inf.
__device__ __forceinline__ float fast_tanh(float y) {
  return 1.f - 2.f * __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(y * 2.8853900817779268f));   // e^{2y}
}

template <int ACT>
__device__ __forceinline__ float act_f(float x) {
  if constexpr (ACT == kGeluErf) {
    return x * phi_cdf(x, gauss_e(x));
  } else if constexpr (ACT == kGeluTanh) {
    const float k = 0.7978845608028654f;
    return 0.5f * x * (1.f + fast_tanh(k * fmaf(0.044715f * x, x * x, x)));
  } else if constexpr (ACT == kRelu) {
    return x > 0.f ? x : 0.f;
  } else {
    return x;
  }
}
template <int ACT>
__device__ __forceinline__ float act_df(float x) {
  if constexpr (ACT == kGeluErf) {
    const float e = gauss_e(x);
    return fmaf(x * 0.3989422804014327f, e, phi_cdf(x, e));
  } else if constexpr (ACT == kGeluTanh) {
    const float k = 0.7978845608028654f;
    const float t = fast_tanh(k * fmaf(0.044715f * x, x * x, x));
    return 0.5f * (1.f + t) + 0.5f * x * (1.f - t * t) * k * (1.f + 3.f * 0.044715f * x * x);
  } else if constexpr (ACT == kRelu) {
    return x > 0.f ? 1.f : 0.f;
  } else {
    return 1.f;
  }
}
// act(x) and act'(x) together (the backward recompute path shares the exponential)
template <int ACT>
__device__ __forceinline__ void act_fdf(float x, float& y, float& dy) {
  if constexpr (ACT == kGeluErf) {
    const float e = gauss_e(x);
    const float c = phi_cdf(x, e);
    y = x * c;
    dy = fmaf(x * 0.3989422804014327f, e, c);
  } else {
    y = act_f<ACT>(x);
    dy = act_df<ACT>(x);
  }
}

template <typename T, int ACT, int NT>
__global__ void __launch_bounds__(256) act_fwd_kernel(const T* __restrict__ u, T* __restrict__ y, size_t n) {
  const size_t nv = n / 8;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nv; i += (size_t)gridDim.x * blockDim.x) {
    float t[8];
    if (NT & 1) vload_nt<T, 8>(u + i * 8, t); else vload<T, 8>(u + i * 8, t);
#pragma unroll
    for (int j = 0; j < 8; ++j) t[j] = act_f<ACT>(t[j]);
    if (NT & 2) vstore_nt<T, 8>(y + i * 8, t); else vstore<T, 8>(y + i * 8, t);
  }
  // tail (n % 8) handled by block 0
  if (blockIdx.x == 0) {
    for (size_t i = nv * 8 + threadIdx.x; i < n; i += blockDim.x) y[i] = (T)act_f<ACT>((float)u[i]);
  }
}

// du = dy * act'(u) (act == kNone: du = dy), plus per-block column partials of du.  With
// `yout`, the activation act(u) is recomputed in the same pass (the FFN backward needs it for
// the second projection's weight gradient; storing it in forward would cost a T x 4h tensor).
// grid = (ceil(cols / (64*VEC)), G); block = 4 waves sharing one 64*VEC-column tile; each wave
// strides over rows with 4 rows in flight (ILP), and the 4 waves' column sums are combined
// through LDS into one partial row per block row-group.
template <typename T, int VEC, int ACT, int NT>
__global__ void __launch_bounds__(256) act_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ u,
                                                      T* __restrict__ du, float* __restrict__ part,
                                                      T* __restrict__ yout, int rows, int cols) {
  constexpr bool kAct = ACT != kNone;
#define LD(p, o) do { if (NT & 1) vload_nt<T, VEC>(p, o); else vload<T, VEC>(p, o); } while (0)
#define ST(p, o) do { if (NT & 2) vstore_nt<T, VEC>(p, o); else vstore<T, VEC>(p, o); } while (0)
  __shared__ float sh[4][64 * VEC];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int col = (blockIdx.x * 64 + lane) * VEC;
  const bool cv = col < cols;
  float acc[VEC];
#pragma unroll
  for (int j = 0; j < VEC; ++j) acc[j] = 0.f;
  const int stride = gridDim.y * 4;
  int r = blockIdx.y * 4 + w;
  if (cv) {
    for (; r + 3 * stride < rows; r += 4 * stride) {
      float d[4][VEC], x[4][VEC];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const size_t off = (size_t)(r + k * stride) * cols + col;
        LD(dy + off, d[k]);
        if (kAct) LD(u + off, x[k]);
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        if (kAct && yout) {
          float a[VEC];
#pragma unroll
          for (int j = 0; j < VEC; ++j) {
            float g;
            act_fdf<ACT>(x[k][j], a[j], g);
            d[k][j] *= g;
          }
          ST(yout + (size_t)(r + k * stride) * cols + col, a);
        } else if (kAct) {
#pragma unroll
          for (int j = 0; j < VEC; ++j) d[k][j] *= act_df<ACT>(x[k][j]);
        }
        if (du) ST(du + (size_t)(r + k * stride) * cols + col, d[k]);
#pragma unroll
        for (int j = 0; j < VEC; ++j) acc[j] += d[k][j];
      }
    }
    for (; r < rows; r += stride) {
      const size_t off = (size_t)r * cols + col;
      float d[VEC];
      LD(dy + off, d);
      if (kAct) {
        float x[VEC];
        LD(u + off, x);
        if (yout) {
          float a[VEC];
#pragma unroll
          for (int j = 0; j < VEC; ++j) {
            float g;
            act_fdf<ACT>(x[j], a[j], g);
            d[j] *= g;
          }
          ST(yout + off, a);
        } else {
#pragma unroll
          for (int j = 0; j < VEC; ++j) d[j] *= act_df<ACT>(x[j]);
        }
      }
      if (du) ST(du + off, d);
#pragma unroll
      for (int j = 0; j < VEC; ++j) acc[j] += d[j];
    }
  }
#undef LD
#undef ST
  if (!part) return;
#pragma unroll
  for (int j = 0; j < VEC; ++j) sh[w][lane * VEC + j] = acc[j];
  __syncthreads();
  for (int c = threadIdx.x; c < 64 * VEC; c += 256) {
    const int gc = blockIdx.x * 64 * VEC + c;
    if (gc < cols) part[(size_t)blockIdx.y * cols + gc] = (sh[0][c] + sh[1][c]) + (sh[2][c] + sh[3][c]);
  }
}

template <typename T, int VEC>
void launch_act_bwd(const void* dy, const void* u, void* du, float* part, void* yout, int rows, int cols, int act,
                    int groups, hipStream_t s) {
  dim3 grid((cols / VEC + 63) / 64, groups);
  const int nt = ew_nt_bits();
#define DTD_ACT_BWD_NT(A, N)                                                                                    \
  hipLaunchKernelGGL((act_bwd_kernel<T, VEC, A, N>), grid, dim3(256), 0, s, (const T*)dy, (const T*)u, (T*)du, part, \
                     (T*)yout, rows, cols)
#define DTD_ACT_BWD(A)                                                                                          \
  switch (nt) {                                                                                                 \
    case 3: DTD_ACT_BWD_NT(A, 3); break;                                                                        \
    default: DTD_ACT_BWD_NT(A, 0); break;                                                                       \
  }
  switch (act) {
    case kGeluErf: DTD_ACT_BWD(kGeluErf); break;
    case kGeluTanh: DTD_ACT_BWD(kGeluTanh); break;
    case kRelu: DTD_ACT_BWD(kRelu); break;
    default: DTD_ACT_BWD(kNone); break;
  }
#undef DTD_ACT_BWD
#undef DTD_ACT_BWD_NT
}

template <typename T>
void dispatch_act_bwd(const void* dy, const void* u, void* du, float* part, void* yout, int rows, int cols, int act,
                      int groups, hipStream_t s) {
  if (cols % 8 == 0) launch_act_bwd<T, 8>(dy, u, du, part, yout, rows, cols, act, groups, s);
  else if (cols % 4 == 0) launch_act_bwd<T, 4>(dy, u, du, part, yout, rows, cols, act, groups, s);
  else if (cols % 2 == 0) launch_act_bwd<T, 2>(dy, u, du, part, yout, rows, cols, act, groups, s);
  else launch_act_bwd<T, 1>(dy, u, du, part, yout, rows, cols, act, groups, s);
}

// out[c] = (accumulate ? out[c] : 0) + scale * sum_p part[p][c]; fixed summation order.
// block = 1024 threads = 64 columns x 16 part-slices combined through LDS; grid.y selects one
// of up to 4 (part, out) pairs so the LayerNorm backward finalises gamma/beta/bias in one launch.
struct FinalizeSet {
  const float* part[4]; void* out[4]; int dtype[4]; int acc[4];
};

// Column sums of [nparts x cols] fp32 partials.  Block = 16 columns x 64 row-lanes (1024
// threads): each wave reads 4 rows x 16 columns (64 B segments), so a 768-wide array spreads
// over 48 blocks per partial array instead of 12 (the finalize is latency-, not bandwidth-bound).
// Fixed summation order: deterministic.
__global__ void __launch_bounds__(1024) colsum_finalize_kernel(FinalizeSet fs, int nparts, int cols, float scale) {
  __shared__ float sh[64][17];
  const int c = threadIdx.x & 15, rl = threadIdx.x >> 4;  // rl: row-lane 0..63
  const int col = blockIdx.x * 16 + c;
  const int k = blockIdx.y;
  const float* part = fs.part[k];
  float t0 = 0.f, t1 = 0.f;
  if (col < cols) {
    int p = rl;
    for (; p + 64 < nparts; p += 128) {
      t0 += part[(size_t)p * cols + col];
      t1 += part[(size_t)(p + 64) * cols + col];
    }
    if (p < nparts) t0 += part[(size_t)p * cols + col];
  }
  sh[rl][c] = t0 + t1;
  __syncthreads();
  if (rl == 0 && col < cols) {
    float s = 0.f;
#pragma unroll 16
    for (int i = 0; i < 64; ++i) s += sh[i][c];
    s *= scale;
    if (fs.dtype[k] == kBF16) {
      bf16* o = (bf16*)fs.out[k];
      if (fs.acc[k]) s += (float)o[col];
      o[col] = (bf16)s;
    } else {
      float* o = (float*)fs.out[k];
      if (fs.acc[k]) s += o[col];
      o[col] = s;
    }
  }
}

// A batch of independent finalizes in one launch (grid.y = job): the backward queues the column-sum
// finalizes of its bias / LayerNorm gradients and flushes them together before anything reads a
// gradient (ops/functional.py flush_finalizes) -- 53 launches of ~5 us per BERT-base step become a
// few.  Same per-column arithmetic and order as colsum_finalize_kernel.
struct FinalizeJob {
  const float* part; void* out; int nparts, cols, dtype, acc; float scale; int pad;
};
constexpr int kFinalizeBatch = 32;
struct FinalizeBatch {
  FinalizeJob j[kFinalizeBatch];
};

__global__ void __launch_bounds__(1024) colsum_finalize_batch_kernel(FinalizeBatch b) {
  __shared__ float sh[64][17];
  const FinalizeJob& jb = b.j[blockIdx.y];
  if ((int)blockIdx.x * 16 >= jb.cols) return;   // uniform per block: this job has fewer columns
  const int c = threadIdx.x & 15, rl = threadIdx.x >> 4;
  const int col = blockIdx.x * 16 + c, cols = jb.cols, nparts = jb.nparts;
  const float* part = jb.part;
  float t0 = 0.f, t1 = 0.f;
  if (col < cols) {
    int p = rl;
    for (; p + 64 < nparts; p += 128) {
      t0 += part[(size_t)p * cols + col];
      t1 += part[(size_t)(p + 64) * cols + col];
    }
    if (p < nparts) t0 += part[(size_t)p * cols + col];
  }
  sh[rl][c] = t0 + t1;
  __syncthreads();
  if (rl == 0 && col < cols) {
    float s = 0.f;
#pragma unroll 16
    for (int i = 0; i < 64; ++i) s += sh[i][c];
    s *= jb.scale;
    if (jb.dtype == kBF16) {
      bf16* o = (bf16*)jb.out;
      if (jb.acc) s += (float)o[col];
      o[col] = (bf16)s;
    } else {
      float* o = (float*)jb.out;
      if (jb.acc) s += o[col];
      o[col] = s;
    }
  }
}

}  // namespace

// jobs: host array of `n` (1..32) FinalizeJob records (part, out, nparts, cols, dtype, acc, scale, pad)
DTD_EXPORT int dtd_colsum_finalize_batch(int n, const void* jobs, hipStream_t s) {
  if (n <= 0) return 0;
  if (n > kFinalizeBatch) return (int)hipErrorInvalidValue;
  FinalizeBatch b{};
  const FinalizeJob* src = (const FinalizeJob*)jobs;
  int maxc = 0;
  for (int i = 0; i < n; ++i) {
    b.j[i] = src[i];
    if (b.j[i].cols > maxc) maxc = b.j[i].cols;
  }
  if (maxc <= 0) return 0;
  hipLaunchKernelGGL(colsum_finalize_batch_kernel, dim3((maxc + 15) / 16, n), dim3(1024), 0, s, b);
  DTD_LAUNCH_CHECK();
}

DTD_EXPORT int dtd_act_fwd(int dtype, const void* u, void* y, size_t n, int act, hipStream_t s) {
  if (n == 0) return 0;
  const int mode = ew_mode(), nt = ew_nt_bits();
  size_t blocks = (n / 8 + 255) / 256;
  if (blocks < 1) blocks = 1;
  if (mode == 0 && blocks > 4096) blocks = 4096;   // streaming form: one 16-byte vector per thread
#define DTD_ACT_FWD_NT(T, A, N) hipLaunchKernelGGL((act_fwd_kernel<T, A, N>), dim3(blocks), dim3(256), 0, s, (const T*)u, (T*)y, n)
#define DTD_ACT_FWD(T, A)                         \
  switch (nt) {                                   \
    case 3: DTD_ACT_FWD_NT(T, A, 3); break;       \
    default: DTD_ACT_FWD_NT(T, A, 0); break;      \
  }
#define DTD_ACT_FWD_T(T)                                \
  switch (act) {                                        \
    case kGeluErf: DTD_ACT_FWD(T, kGeluErf); break;     \
    case kGeluTanh: DTD_ACT_FWD(T, kGeluTanh); break;   \
    case kRelu: DTD_ACT_FWD(T, kRelu); break;           \
    default: DTD_ACT_FWD(T, kNone); break;              \
  }
  if (dtype == kBF16) { DTD_ACT_FWD_T(bf16) } else { DTD_ACT_FWD_T(float) }
#undef DTD_ACT_FWD_T
#undef DTD_ACT_FWD
#undef DTD_ACT_FWD_NT
  DTD_LAUNCH_CHECK();
}

// Row groups used by dtd_act_bwd for a [rows, cols] operand (callers size `part` [n, cols]).
DTD_EXPORT int dtd_act_bwd_num_partials(int rows, int cols) {
  (void)cols;
  int g = (rows + 15) / 16;
  if (g < 1) g = 1;
  if (g > 256) g = 256;
  return g;
}

// yout (may be null): also write act(u) -- requires act != none.
DTD_EXPORT int dtd_act_bwd(int dtype, const void* dy, const void* u, void* du, float* part, void* yout, int rows,
                           int cols, int act, hipStream_t s) {
  if (rows <= 0) return 0;
  if (yout && (act == kNone || !u)) return (int)hipErrorInvalidValue;
  const int groups = dtd_act_bwd_num_partials(rows, cols);
  if (dtype == kBF16) dispatch_act_bwd<bf16>(dy, u, du, part, yout, rows, cols, act, groups, s);
  else dispatch_act_bwd<float>(dy, u, du, part, yout, rows, cols, act, groups, s);
  DTD_LAUNCH_CHECK();
}

DTD_EXPORT int dtd_colsum_finalize(const float* part, int nparts, int cols, void* out, int out_dtype, int accumulate,
                                   float scale, hipStream_t s) {
  if (cols <= 0) return 0;
  FinalizeSet fs{};
  fs.part[0] = part; fs.out[0] = out; fs.dtype[0] = out_dtype; fs.acc[0] = accumulate;
  hipLaunchKernelGGL(colsum_finalize_kernel, dim3((cols + 15) / 16, 1), dim3(1024), 0, s, fs, nparts, cols, scale);
  DTD_LAUNCH_CHECK();
}

// Up to 4 partial arrays laid out back to back in `parts` ([n][nparts][cols]).
DTD_EXPORT int dtd_colsum_finalize_multi(int n, const float* parts, int nparts, int cols, void* out0, int dt0, int acc0,
                                         void* out1, int dt1, int acc1, void* out2, int dt2, int acc2, hipStream_t s) {
  if (cols <= 0 || n <= 0) return 0;
  FinalizeSet fs{};
  void* outs[3] = {out0, out1, out2};
  int dts[3] = {dt0, dt1, dt2}, accs[3] = {acc0, acc1, acc2};
  for (int i = 0; i < n && i < 3; ++i) {
    fs.part[i] = parts + (size_t)i * nparts * cols;
    fs.out[i] = outs[i]; fs.dtype[i] = dts[i]; fs.acc[i] = accs[i];
  }
  hipLaunchKernelGGL(colsum_finalize_kernel, dim3((cols + 15) / 16, n), dim3(1024), 0, s, fs, nparts, cols, 1.f);
  DTD_LAUNCH_CHECK();
}
