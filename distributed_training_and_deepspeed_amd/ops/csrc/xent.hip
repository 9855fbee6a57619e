// Softmax cross-entropy with ignore_index (-100) for the MLM / causal-LM heads.
//
// Reference: HF BertForMaskedLM / *ForCausalLM `CrossEntropyLoss()(logits.view(-1, V), labels)`
// and model_parallel_training.py:51,73.  ATen runs log_softmax + nll_loss as
// separate passes over the [N, V] logits; here
//   forward : one read of each row -> per-row loss and log-sum-exp (online max/sum in fp32)
//   reduce  : one block -> mean loss over valid rows + valid count (device scalars; no host sync)
//   backward: one read + one write -> dlogits = (softmax - onehot) * grad_out / count
// One 256-thread workgroup per row.  Rows are read with 16-byte vectors whatever V is: a row of
// an odd vocabulary (GPT-2, 50257) starts at any 2-byte boundary, so each row is split into a
// scalar head up to the next 16-byte boundary, an aligned 16-byte body and a scalar tail (the
// first version fell back to 2-byte loads for odd V and ran at ~1.8 TB/s).
#include "common.h"

using namespace dtd;

namespace {

// [0, head) scalar, [head, body) 16-byte vectors of VEC elements, [body, V) scalar.
template <typename T, int VEC>
__device__ __forceinline__ void row_split(const T* z, int V, int& head, int& body) {
  const int mis = (int)((reinterpret_cast<uintptr_t>(z) & 15) / sizeof(T));
  head = mis ? min(V, VEC - mis) : 0;
  body = head + (V - head) / VEC * VEC;
}

template <typename T>
__global__ void __launch_bounds__(256) xent_fwd_kernel(const T* __restrict__ logits, const int64_t* __restrict__ labels,
                                                       float* __restrict__ loss_row, float* __restrict__ lse_row,
                                                       int rows, int V, int ignore_index) {
  constexpr int VEC = 16 / sizeof(T);
  __shared__ float sh[8];
  const int row = blockIdx.x;
  const int64_t y = labels[row];
  if (y == ignore_index) {  // uniform per block
    if (threadIdx.x == 0) { loss_row[row] = 0.f; lse_row[row] = 0.f; }
    return;
  }
  const T* z = logits + (size_t)row * V;
  int head, body;
  row_split<T, VEC>(z, V, head, body);
  float m = -INFINITY, s = 0.f;
  auto add1 = [&](float t) {
    if (t > m) { s *= __expf(m - t); m = t; }
    s += __expf(t - m);
  };
  if ((int)threadIdx.x < head) add1((float)z[threadIdx.x]);
#pragma unroll 2
  for (int c = head + threadIdx.x * VEC; c < body; c += blockDim.x * VEC) {
    float t[VEC];
    vload<T, VEC>(z + c, t);
    float lm = t[0];
#pragma unroll
    for (int j = 1; j < VEC; ++j) lm = fmaxf(lm, t[j]);
    if (lm > m) { s *= __expf(m - lm); m = lm; }
#pragma unroll
    for (int j = 0; j < VEC; ++j) s += __expf(t[j] - m);
  }
  for (int c = body + threadIdx.x; c < V; c += blockDim.x) add1((float)z[c]);
  const float M = block_max(m, sh);
  s = (m == -INFINITY) ? 0.f : s * __expf(m - M);
  const float S = block_sum(s, sh);
  if (threadIdx.x == 0) {
    const float lse = M + __logf(S);
    lse_row[row] = lse;
    loss_row[row] = lse - (float)z[y];
  }
}

// out[0] = sum(loss_row) / count, out[1] = count (number of rows with a valid label).  One block
// of 1024 threads with 4 independent row loads in flight per thread (a 256-thread loop of dependent
// loads was latency-bound: 57 us for 21k rows).
__global__ void __launch_bounds__(1024) xent_reduce_kernel(const float* __restrict__ loss_row,
                                                           const int64_t* __restrict__ labels, int rows,
                                                           int ignore_index, float* __restrict__ out) {
  __shared__ float sh[16];
  float s = 0.f, c = 0.f;
  const int n = blockDim.x;
  int r = threadIdx.x;
  for (; r + 3 * n < rows; r += 4 * n) {
    int64_t y[4];
    float l[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      y[k] = labels[r + k * n];
      l[k] = loss_row ? loss_row[r + k * n] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (y[k] != ignore_index) { s += l[k]; c += 1.f; }
  }
  for (; r < rows; r += n) {
    if (labels[r] != ignore_index) { s += loss_row ? loss_row[r] : 0.f; c += 1.f; }
  }
  s = block_sum(s, sh);
  c = block_sum(c, sh);
  if (threadIdx.x == 0) { out[0] = c > 0.f ? s / c : NAN; out[1] = c; }
}

// logits and dlogits share their 16-byte phase (checked on the host), so one split serves both.
template <typename T>
__global__ void __launch_bounds__(256) xent_bwd_kernel(const T* __restrict__ logits, const int64_t* __restrict__ labels,
                                                       const float* __restrict__ lse_row, const float* __restrict__ stats,
                                                       const float* __restrict__ grad_out, T* __restrict__ dlogits,
                                                       int rows, int V, int ignore_index) {
  constexpr int VEC = 16 / sizeof(T);
  const int row = blockIdx.x;
  const int64_t y = labels[row];
  const T* z = logits + (size_t)row * V;
  T* dz = dlogits + (size_t)row * V;
  int head, body;
  row_split<T, VEC>(z, V, head, body);
  const bool ign = y == ignore_index;   // uniform per block: the row's gradient is zero
  const float g = ign ? 0.f : grad_out[0] / stats[1];
  const float lse = ign ? 0.f : lse_row[row];
  auto grad1 = [&](int c) {
    float p = ign ? 0.f : __expf((float)z[c] - lse);
    if (c == y) p -= 1.f;
    dz[c] = (T)(p * g);
  };
  if ((int)threadIdx.x < head) grad1(threadIdx.x);
#pragma unroll 2
  for (int c = head + threadIdx.x * VEC; c < body; c += blockDim.x * VEC) {
    float t[VEC];
    if (ign) {
#pragma unroll
      for (int j = 0; j < VEC; ++j) t[j] = 0.f;
    } else {
      vload<T, VEC>(z + c, t);
#pragma unroll
      for (int j = 0; j < VEC; ++j) {
        float p = __expf(t[j] - lse);
        if (c + j == y) p -= 1.f;
        t[j] = p * g;
      }
    }
    vstore<T, VEC>(dz + c, t);
  }
  for (int c = body + threadIdx.x; c < V; c += blockDim.x) grad1(c);
}

// Backward with the decoder-bias gradient fused in (SURVEY.md K8 + the MLM head's bias): the bias
// gradient is the column sum of dlogits, which the unfused path re-reads from HBM (1.2 GB at
// bench.py's b256: a 266 us pass).  A block owns a fixed column set -- 4-wide groups c = 4 (t + 512 k),
// k < XB_GROUPS -- and strides over rows, so every row's dlogits stay in registers for the column
// sums; each block writes one fp32 partial row ([gridDim.x][V], summed by colsum_finalize).
// Needs V % 4 == 0 (8-byte row alignment of bf16 rows) and V <= 4 * XB_THREADS * XB_GROUPS.
constexpr int XB_GROUPS = 16, XB_THREADS = 512;
// FWD = true (training forward, dtd_xent_fwd_train): the block also computes each row's
// log-sum-exp from the row it holds in registers (two block reductions per row) and writes
// lse_row / loss_row, with the gradient scale 1 / count (grad_out = 1; the backward rescales
// when the loss gradient is not 1) -- the logits are read once for the loss and the gradient.
template <bool FWD>
__global__ void __launch_bounds__(XB_THREADS) xent_bwd_colsum_kernel(const bf16* __restrict__ logits,
                                                              const int64_t* __restrict__ labels,
                                                              float* __restrict__ lse_row,
                                                              const float* __restrict__ stats,
                                                              const float* __restrict__ grad_out,
                                                              bf16* __restrict__ dlogits, float* __restrict__ part,
                                                              float* __restrict__ loss_row,
                                                              int rows, int V, int ignore_index) {
  __shared__ float sh[XB_THREADS / 64];
  const int tid = threadIdx.x;
  const float gs = (FWD ? 1.f : grad_out[0]) / stats[1];
  float acc[XB_GROUPS][4];
#pragma unroll
  for (int k = 0; k < XB_GROUPS; ++k)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[k][j] = 0.f;
  for (int row = blockIdx.x; row < rows; row += gridDim.x) {
    const int64_t y = labels[row];
    const bf16* z = logits + (size_t)row * V;
    bf16* dz = dlogits + (size_t)row * V;
    if (y == ignore_index) {   // zero gradient row (uniform per block)
#pragma unroll
      for (int k = 0; k < XB_GROUPS; ++k) {
        const int c = 4 * (tid + XB_THREADS * k);
        if (c < V) *reinterpret_cast<bf16x4*>(dz + c) = bf16x4{0, 0, 0, 0};
      }
      if (FWD && tid == 0) { lse_row[row] = 0.f; loss_row[row] = 0.f; }
      continue;
    }
    float lse;
    if constexpr (FWD) {
      float mx = -INFINITY;
#pragma unroll
      for (int k = 0; k < XB_GROUPS; ++k) {
        const int c = 4 * (tid + XB_THREADS * k);
        if (c < V) {
          const bf16x4 q = *reinterpret_cast<const bf16x4*>(z + c);
#pragma unroll
          for (int j = 0; j < 4; ++j) mx = fmaxf(mx, (float)q[j]);
        }
      }
      const float M = block_max(mx, sh);
      float se = 0.f;
#pragma unroll
      for (int k = 0; k < XB_GROUPS; ++k) {
        const int c = 4 * (tid + XB_THREADS * k);
        if (c < V) {
          const bf16x4 q = *reinterpret_cast<const bf16x4*>(z + c);   // L1/L2 hit: read just above
#pragma unroll
          for (int j = 0; j < 4; ++j) se += __expf((float)q[j] - M);
        }
      }
      lse = M + __logf(block_sum(se, sh));
      if (tid == 0) { lse_row[row] = lse; loss_row[row] = lse - (float)z[y]; }
    } else {
      lse = lse_row[row];
    }
    const int yr = (int)y - 4 * tid;   // label column relative to this thread's first column
    // 8 column groups per chunk: loads in flight without holding the whole row in registers
#pragma unroll
    for (int kc = 0; kc < XB_GROUPS; kc += 8) {
      bf16x4 zin[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int c = 4 * (tid + XB_THREADS * (kc + k));
        zin[k] = c < V ? *reinterpret_cast<const bf16x4*>(z + c) : bf16x4{0, 0, 0, 0};
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int c = 4 * (tid + XB_THREADS * (kc + k));
        if (c < V) {
          bf16x4 o;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            float p = __expf((float)zin[k][j] - lse);
            if (4 * XB_THREADS * (kc + k) + j == yr) p -= 1.f;
            const bf16 d = (bf16)(p * gs);
            o[j] = d;
            acc[kc + k][j] += (float)d;   // the bias gradient of the stored (bf16) dlogits
          }
          *reinterpret_cast<bf16x4*>(dz + c) = o;
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
#pragma unroll
  for (int k = 0; k < XB_GROUPS; ++k) {
    const int c = 4 * (tid + XB_THREADS * k);
    if (c < V)
      *reinterpret_cast<f32x4*>(part + (size_t)blockIdx.x * V + c) = f32x4{acc[k][0], acc[k][1], acc[k][2], acc[k][3]};
  }
}

}  // namespace

DTD_EXPORT int dtd_xent_fwd(int dtype, const void* logits, const int64_t* labels, float* loss_row, float* lse_row,
                            float* stats, int rows, int V, int ignore_index, hipStream_t s) {
  if (rows <= 0) return 0;
  if (dtype == kBF16)
    hipLaunchKernelGGL(xent_fwd_kernel<bf16>, dim3(rows), dim3(256), 0, s, (const bf16*)logits, labels, loss_row,
                       lse_row, rows, V, ignore_index);
  else
    hipLaunchKernelGGL(xent_fwd_kernel<float>, dim3(rows), dim3(256), 0, s, (const float*)logits, labels, loss_row,
                       lse_row, rows, V, ignore_index);
  hipLaunchKernelGGL(xent_reduce_kernel, dim3(1), dim3(1024), 0, s, loss_row, labels, rows, ignore_index, stats);
  DTD_LAUNCH_CHECK();
}

DTD_EXPORT int dtd_xent_bwd(int dtype, const void* logits, const int64_t* labels, const float* lse_row,
                            const float* stats, const float* grad_out, void* dlogits, int rows, int V,
                            int ignore_index, hipStream_t s) {
  if (rows <= 0) return 0;
  if ((reinterpret_cast<uintptr_t>(logits) & 15) != (reinterpret_cast<uintptr_t>(dlogits) & 15)) return -1;
  if (dtype == kBF16)
    hipLaunchKernelGGL(xent_bwd_kernel<bf16>, dim3(rows), dim3(256), 0, s, (const bf16*)logits, labels, lse_row,
                       stats, grad_out, (bf16*)dlogits, rows, V, ignore_index);
  else
    hipLaunchKernelGGL(xent_bwd_kernel<float>, dim3(rows), dim3(256), 0, s, (const float*)logits, labels, lse_row,
                       stats, grad_out, (float*)dlogits, rows, V, ignore_index);
  DTD_LAUNCH_CHECK();
}

// dlogits and the fp32 column partials of dlogits ([parts][V]; colsum_finalize sums them into the
// decoder-bias gradient).  parts = dtd_xent_bwd_colsum_parts(rows).
DTD_EXPORT int dtd_xent_bwd_colsum_parts(int rows) { return rows < 256 ? (rows > 0 ? rows : 1) : 256; }
DTD_EXPORT int dtd_xent_bwd_colsum_supported(int V) { return V > 0 && V % 4 == 0 && V <= 4 * XB_THREADS * XB_GROUPS; }
DTD_EXPORT int dtd_xent_bwd_colsum(const void* logits, const int64_t* labels, const float* lse_row,
                                   const float* stats, const float* grad_out, void* dlogits, float* part, int rows,
                                   int V, int ignore_index, hipStream_t s) {
  if (rows <= 0) return 0;
  if (!dtd_xent_bwd_colsum_supported(V)) return (int)hipErrorInvalidValue;
  if (((reinterpret_cast<uintptr_t>(logits) | reinterpret_cast<uintptr_t>(dlogits)) & 7) ||
      (reinterpret_cast<uintptr_t>(part) & 15))
    return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(xent_bwd_colsum_kernel<false>, dim3(dtd_xent_bwd_colsum_parts(rows)), dim3(XB_THREADS), 0, s,
                     (const bf16*)logits, labels, const_cast<float*>(lse_row), stats, grad_out, (bf16*)dlogits,
                     part, (float*)nullptr, rows, V, ignore_index);
  DTD_LAUNCH_CHECK();
}

// Training forward of the mean cross-entropy in one pass over the logits: loss (stats[0]), valid
// count (stats[1]), lse / loss per row, dlogits for a loss gradient of 1 and the fp32 column
// partials of dlogits ([parts][V], the bias gradient).  Same shape contract as
// dtd_xent_bwd_colsum.  The backward scales by the actual loss gradient (dtd_xent_grad_scale).
DTD_EXPORT int dtd_xent_fwd_train(const void* logits, const int64_t* labels, float* loss_row, float* lse_row,
                                  float* stats, void* dlogits, float* part, int rows, int V, int ignore_index,
                                  hipStream_t s) {
  if (rows <= 0) return 0;
  if (!dtd_xent_bwd_colsum_supported(V)) return (int)hipErrorInvalidValue;
  if (((reinterpret_cast<uintptr_t>(logits) | reinterpret_cast<uintptr_t>(dlogits)) & 7) ||
      (reinterpret_cast<uintptr_t>(part) & 15))
    return (int)hipErrorInvalidValue;
  // the valid-label count first (the gradient scale), the loss mean after
  hipLaunchKernelGGL(xent_reduce_kernel, dim3(1), dim3(1024), 0, s, (const float*)nullptr, labels, rows, ignore_index,
                     stats);
  hipLaunchKernelGGL(xent_bwd_colsum_kernel<true>, dim3(dtd_xent_bwd_colsum_parts(rows)), dim3(XB_THREADS), 0, s,
                     (const bf16*)logits, labels, lse_row, (const float*)stats, (const float*)nullptr,
                     (bf16*)dlogits, part, loss_row, rows, V, ignore_index);
  hipLaunchKernelGGL(xent_reduce_kernel, dim3(1), dim3(1024), 0, s, (const float*)loss_row, labels, rows,
                     ignore_index, stats);
  DTD_LAUNCH_CHECK();
}

// x *= g[0] (bf16, in place) unless g[0] == 1: every block reads g and returns at once in the
// usual case (the loss gradient of a plain loss.backward()).
__global__ void __launch_bounds__(256) xent_grad_scale_kernel(bf16* __restrict__ x, size_t n,
                                                              const float* __restrict__ g) {
  const float sc = g[0];
  if (sc == 1.f) return;
  for (size_t i = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) * 4; i < n; i += (size_t)gridDim.x * blockDim.x * 4) {
    if (i + 4 <= n) {
      bf16x4 v = *reinterpret_cast<const bf16x4*>(x + i);
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = (bf16)((float)v[j] * sc);
      *reinterpret_cast<bf16x4*>(x + i) = v;
    } else {
      for (size_t e = i; e < n; ++e) x[e] = (bf16)((float)x[e] * sc);
    }
  }
}

DTD_EXPORT int dtd_xent_grad_scale(void* x, size_t n, const float* g, hipStream_t s) {
  if (n == 0) return 0;
  if (reinterpret_cast<uintptr_t>(x) & 7) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(xent_grad_scale_kernel, dim3(1024), dim3(256), 0, s, (bf16*)x, n, g);
  DTD_LAUNCH_CHECK();
}
