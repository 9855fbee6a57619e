// Softmax cross-entropy with ignore_index (-100) for the MLM / causal-LM heads.
//
// Reference: HF BertForMaskedLM / *ForCausalLM `CrossEntropyLoss()(logits.view(-1, V), labels)`
// and model_parallel_training.py:51,73.  ATen runs log_softmax + nll_loss as
// separate passes over the [N, V] logits; here
//   forward : one read of each row -> per-row loss and log-sum-exp (online max/sum in fp32)
//   reduce  : one block -> mean loss over valid rows + valid count (device scalars; no host sync)
//   backward: one read + one write -> dlogits = (softmax - onehot) * grad_out / count
// One 256-thread workgroup per row; rows are read with the widest vector (8/4/2/1 elements)
// that divides V, so odd vocabularies (GPT-2, 50257) stay correct.
#include "common.h"

using namespace dtd;

namespace {

template <typename T, int VEC>
__global__ void __launch_bounds__(256) xent_fwd_kernel(const T* __restrict__ logits, const int64_t* __restrict__ labels,
                                                       float* __restrict__ loss_row, float* __restrict__ lse_row,
                                                       int rows, int V, int ignore_index) {
  __shared__ float sh[8];
  const int row = blockIdx.x;
  const int64_t y = labels[row];
  if (y == ignore_index) {  // uniform per block
    if (threadIdx.x == 0) { loss_row[row] = 0.f; lse_row[row] = 0.f; }
    return;
  }
  const T* z = logits + (size_t)row * V;
  float m = -INFINITY, s = 0.f;
  for (int c = threadIdx.x * VEC; c < V; c += blockDim.x * VEC) {
    float t[VEC];
    vload<T, VEC>(z + c, t);
    float lm = t[0];
#pragma unroll
    for (int j = 1; j < VEC; ++j) lm = fmaxf(lm, t[j]);
    if (lm > m) { s *= __expf(m - lm); m = lm; }
#pragma unroll
    for (int j = 0; j < VEC; ++j) s += __expf(t[j] - m);
  }
  const float M = block_max(m, sh);
  s = (m == -INFINITY) ? 0.f : s * __expf(m - M);
  const float S = block_sum(s, sh);
  if (threadIdx.x == 0) {
    const float lse = M + __logf(S);
    lse_row[row] = lse;
    loss_row[row] = lse - (float)z[y];
  }
}

// out[0] = sum(loss_row) / count, out[1] = count (number of rows with a valid label).
__global__ void __launch_bounds__(256) xent_reduce_kernel(const float* __restrict__ loss_row,
                                                          const int64_t* __restrict__ labels, int rows,
                                                          int ignore_index, float* __restrict__ out) {
  __shared__ float sh[8];
  float s = 0.f, c = 0.f;
  for (int r = threadIdx.x; r < rows; r += blockDim.x) {
    if (labels[r] != ignore_index) { s += loss_row[r]; c += 1.f; }
  }
  s = block_sum(s, sh);
  c = block_sum(c, sh);
  if (threadIdx.x == 0) { out[0] = c > 0.f ? s / c : NAN; out[1] = c; }
}

template <typename T, int VEC>
__global__ void __launch_bounds__(256) xent_bwd_kernel(const T* __restrict__ logits, const int64_t* __restrict__ labels,
                                                       const float* __restrict__ lse_row, const float* __restrict__ stats,
                                                       const float* __restrict__ grad_out, T* __restrict__ dlogits,
                                                       int rows, int V, int ignore_index) {
  const int row = blockIdx.x;
  const int64_t y = labels[row];
  T* dz = dlogits + (size_t)row * V;
  if (y == ignore_index) {
    float zero[VEC];
#pragma unroll
    for (int j = 0; j < VEC; ++j) zero[j] = 0.f;
    for (int c = threadIdx.x * VEC; c < V; c += blockDim.x * VEC) vstore<T, VEC>(dz + c, zero);
    return;
  }
  const float g = grad_out[0] / stats[1];
  const float lse = lse_row[row];
  const T* z = logits + (size_t)row * V;
  for (int c = threadIdx.x * VEC; c < V; c += blockDim.x * VEC) {
    float t[VEC];
    vload<T, VEC>(z + c, t);
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      float p = __expf(t[j] - lse);
      if (c + j == y) p -= 1.f;
      t[j] = p * g;
    }
    vstore<T, VEC>(dz + c, t);
  }
}

template <typename T>
int launch_fwd(const void* logits, const int64_t* labels, float* loss_row, float* lse_row, int rows, int V, int ign,
               hipStream_t s) {
  const T* z = (const T*)logits;
  if (V % 8 == 0) hipLaunchKernelGGL((xent_fwd_kernel<T, 8>), dim3(rows), dim3(256), 0, s, z, labels, loss_row, lse_row, rows, V, ign);
  else if (V % 4 == 0) hipLaunchKernelGGL((xent_fwd_kernel<T, 4>), dim3(rows), dim3(256), 0, s, z, labels, loss_row, lse_row, rows, V, ign);
  else if (V % 2 == 0) hipLaunchKernelGGL((xent_fwd_kernel<T, 2>), dim3(rows), dim3(256), 0, s, z, labels, loss_row, lse_row, rows, V, ign);
  else hipLaunchKernelGGL((xent_fwd_kernel<T, 1>), dim3(rows), dim3(256), 0, s, z, labels, loss_row, lse_row, rows, V, ign);
  return 0;
}
template <typename T>
int launch_bwd(const void* logits, const int64_t* labels, const float* lse_row, const float* stats, const float* gout,
               void* dlogits, int rows, int V, int ign, hipStream_t s) {
  const T* z = (const T*)logits;
  T* d = (T*)dlogits;
  if (V % 8 == 0) hipLaunchKernelGGL((xent_bwd_kernel<T, 8>), dim3(rows), dim3(256), 0, s, z, labels, lse_row, stats, gout, d, rows, V, ign);
  else if (V % 4 == 0) hipLaunchKernelGGL((xent_bwd_kernel<T, 4>), dim3(rows), dim3(256), 0, s, z, labels, lse_row, stats, gout, d, rows, V, ign);
  else if (V % 2 == 0) hipLaunchKernelGGL((xent_bwd_kernel<T, 2>), dim3(rows), dim3(256), 0, s, z, labels, lse_row, stats, gout, d, rows, V, ign);
  else hipLaunchKernelGGL((xent_bwd_kernel<T, 1>), dim3(rows), dim3(256), 0, s, z, labels, lse_row, stats, gout, d, rows, V, ign);
  return 0;
}

}  // namespace

DTD_EXPORT int dtd_xent_fwd(int dtype, const void* logits, const int64_t* labels, float* loss_row, float* lse_row,
                            float* stats, int rows, int V, int ignore_index, hipStream_t s) {
  if (rows <= 0) return 0;
  if (dtype == kBF16) launch_fwd<bf16>(logits, labels, loss_row, lse_row, rows, V, ignore_index, s);
  else launch_fwd<float>(logits, labels, loss_row, lse_row, rows, V, ignore_index, s);
  hipLaunchKernelGGL(xent_reduce_kernel, dim3(1), dim3(256), 0, s, loss_row, labels, rows, ignore_index, stats);
  DTD_LAUNCH_CHECK();
}

DTD_EXPORT int dtd_xent_bwd(int dtype, const void* logits, const int64_t* labels, const float* lse_row,
                            const float* stats, const float* grad_out, void* dlogits, int rows, int V,
                            int ignore_index, hipStream_t s) {
  if (rows <= 0) return 0;
  if (dtype == kBF16) launch_bwd<bf16>(logits, labels, lse_row, stats, grad_out, dlogits, rows, V, ignore_index, s);
  else launch_bwd<float>(logits, labels, lse_row, stats, grad_out, dlogits, rows, V, ignore_index, s);
  DTD_LAUNCH_CHECK();
}
