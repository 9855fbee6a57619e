// Embedding gather-sum forward and deterministic scatter backward, plus standalone dropout.
//
// Reference ops replaced: HF BertEmbeddings (word + position + token-type -> LN -> dropout),
// GPT-2 wte+wpe, OPT embed_tokens + learned positions (offset 2), BLOOM word embeddings
// (SURVEY.md K7).  The LayerNorm is the shared norm kernel; dropout after the LN is
// `dtd_dropout` below (mask regenerated in backward from the counter RNG).
//
// Backward of the word table (up to 250,880 x 1024 for BLOOM) is a *sorted segment sum*:
// token ids are sorted once (on device), and each run of equal ids is summed in fp32 by one
// workgroup that owns that table row exclusively, so there are no float atomics and the
// result is bitwise reproducible (cdna_hip_programming.md Appendix B "Scatter / gather").
#include <algorithm>
#include "common.h"

using namespace dtd;

namespace {

struct GatherArgs {
  const int64_t* ids; const int64_t* type_ids;
  const void* word; const void* pos; const void* type;
  void* out; int rows, h, seq, pos_offset;
};

// One wave per output row (4 rows per block), VEC-wide (16-byte for bf16) loads of the word,
// position and token-type rows.
template <typename T, int VEC>
__global__ void __launch_bounds__(256) embed_fwd_kernel(GatherArgs a) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= a.rows) return;
  const int64_t id = a.ids[row];
  const int pidx = (row % a.seq) + a.pos_offset;
  const int64_t tid = a.type_ids ? a.type_ids[row] : 0;
  const T* w = (const T*)a.word + (size_t)id * a.h;
  const T* p = a.pos ? (const T*)a.pos + (size_t)pidx * a.h : nullptr;
  const T* t = a.type ? (const T*)a.type + (size_t)tid * a.h : nullptr;
  T* o = (T*)a.out + (size_t)row * a.h;
  for (int c = lane * VEC; c < a.h; c += 64 * VEC) {
    float x[VEC], y[VEC];
    vload<T, VEC>(w + c, x);
    if (p) {
      vload<T, VEC>(p + c, y);
#pragma unroll
      for (int j = 0; j < VEC; ++j) x[j] += y[j];
    }
    if (t) {
      vload<T, VEC>(t + c, y);
#pragma unroll
      for (int j = 0; j < VEC; ++j) x[j] += y[j];
    }
    vstore<T, VEC>(o + c, x);
  }
}

// One block per sorted position; only the first position of each run of equal ids works.
template <typename T, typename G>
__global__ void __launch_bounds__(256) embed_word_bwd_kernel(const int64_t* __restrict__ sorted_ids,
                                                             const int64_t* __restrict__ perm,
                                                             const T* __restrict__ dz, G* __restrict__ grad,
                                                             int rows, int h, int accumulate, int padding_idx) {
  const int i = blockIdx.x;
  const int64_t id = sorted_ids[i];
  if (i > 0 && sorted_ids[i - 1] == id) return;
  if (id == padding_idx) return;
  int j = i + 1;
  while (j < rows && sorted_ids[j] == id) ++j;
  G* g = grad + (size_t)id * h;
  for (int c = threadIdx.x * 2; c < h; c += blockDim.x * 2) {
    float acc[2] = {0.f, 0.f};
    for (int k = i; k < j; ++k) {
      float x[2];
      vload<T, 2>(dz + (size_t)perm[k] * h + c, x);
      acc[0] += x[0]; acc[1] += x[1];
    }
    if (accumulate) {
      float old[2];
      vload<G, 2>(g + c, old);
      acc[0] += old[0]; acc[1] += old[1];
    }
    vstore<G, 2>(g + c, acc);
  }
}

// Chunked variant for skewed id distributions (e.g. thousands of [MASK] tokens in one MLM
// batch): pass 1 sums runs of at most CH rows of one id into fp32 scratch rows (one workgroup
// per chunk), pass 2 adds a segment's chunk sums in order into the table row.  seg_lo/seg_hi
// are the [first, last+1) sorted positions of each position's id (searchsorted left/right).
constexpr int kChunk = 16;
constexpr int kUnroll = 8;   // rows (chunk sums) loaded ahead per step of the serial sums below
// Chunk length of a segment: at least kChunk, and ~sqrt(len) for long ones, so neither pass
// sums more than ~sqrt(len) rows serially in one wave (synthetic MLM batches hold one [MASK]
// segment of ~12 % of all tokens: 7.9k rows at b128, 492 serial partial rows with fixed chunks).
__device__ __forceinline__ int chunk_len(int len) {
  const int r = (int)ceilf(sqrtf((float)len));
  return r > kChunk ? r : kChunk;
}

// One WAVE per sorted position (4 per block), VEC-wide loads (16 B for bf16 rows with h % 8 ==
// 0): positions that are not chunk leaders return at once, so a block-per-position grid spent
// most of its time dispatching idle workgroups (~40 % of the step's non-GEMM "other" time).
template <typename T, int VEC>
__global__ void __launch_bounds__(256) embed_chunk_sum_kernel(const int64_t* __restrict__ perm,
                                                              const int64_t* __restrict__ seg_lo,
                                                              const int64_t* __restrict__ seg_hi,
                                                              const T* __restrict__ dz, float* __restrict__ scratch,
                                                              int rows, int h) {
  const int lane = threadIdx.x & 63;
  // grid-stride over sorted positions (one wave each): a grid of one wave per position spent its
  // time dispatching the waves of non-leader positions, which exit at once
  for (int i = blockIdx.x * 4 + (threadIdx.x >> 6); i < rows; i += gridDim.x * 4) {
  const int lo = (int)seg_lo[i], shi = (int)seg_hi[i];
  const int ch = chunk_len(shi - lo);
  if ((i - lo) % ch) continue;
  const int end = min(i + ch, shi);
  for (int c = lane * VEC; c < h; c += 64 * VEC) {
    float acc[VEC];
#pragma unroll
    for (int j = 0; j < VEC; ++j) acc[j] = 0.f;
    // kUnroll rows' loads in flight at once, summed in row order (the same result as one row at
    // a time): a chunk of a long segment is ~sqrt(len) rows, and one dependent HBM round trip per
    // row made the longest chunk the kernel's critical path
    int k = i;
    for (; k + kUnroll <= end; k += kUnroll) {
      float x[kUnroll][VEC];
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) vload<T, VEC>(dz + (size_t)perm[k + u] * h + c, x[u]);
#pragma unroll
      for (int u = 0; u < kUnroll; ++u)
#pragma unroll
        for (int j = 0; j < VEC; ++j) acc[j] += x[u][j];
    }
    for (; k < end; ++k) {
      float x[VEC];
      vload<T, VEC>(dz + (size_t)perm[k] * h + c, x);
#pragma unroll
      for (int j = 0; j < VEC; ++j) acc[j] += x[j];
    }
    vstore<float, VEC>(scratch + (size_t)i * h + c, acc);
  }
  }
}

template <typename G, int VEC>
__global__ void __launch_bounds__(256) embed_chunk_add_kernel(const int64_t* __restrict__ sorted_ids,
                                                              const int64_t* __restrict__ seg_lo,
                                                              const int64_t* __restrict__ seg_hi,
                                                              const float* __restrict__ scratch, G* __restrict__ grad,
                                                              int rows, int h, int accumulate, int padding_idx) {
  const int lane = threadIdx.x & 63;
  for (int i = blockIdx.x * 4 + (threadIdx.x >> 6); i < rows; i += gridDim.x * 4) {   // grid-stride, as above
  if (seg_lo[i] != i) continue;
  const int64_t id = sorted_ids[i];
  if (id == padding_idx) continue;
  const int hi = (int)seg_hi[i];
  const int ch = chunk_len(hi - i);
  G* g = grad + (size_t)id * h;
  for (int c = lane * VEC; c < h; c += 64 * VEC) {
    float acc[VEC];
#pragma unroll
    for (int j = 0; j < VEC; ++j) acc[j] = 0.f;
    int k = i;
    for (; k + kUnroll * ch <= hi; k += kUnroll * ch) {   // kUnroll chunk sums in flight, added in order
      float x[kUnroll][VEC];
#pragma unroll
      for (int u = 0; u < kUnroll; ++u) vload<float, VEC>(scratch + (size_t)(k + u * ch) * h + c, x[u]);
#pragma unroll
      for (int u = 0; u < kUnroll; ++u)
#pragma unroll
        for (int j = 0; j < VEC; ++j) acc[j] += x[u][j];
    }
    for (; k < hi; k += ch) {
      float x[VEC];
      vload<float, VEC>(scratch + (size_t)k * h + c, x);
#pragma unroll
      for (int j = 0; j < VEC; ++j) acc[j] += x[j];
    }
    if (accumulate) {
      float old[VEC];
      vload<G, VEC>(g + c, old);
#pragma unroll
      for (int j = 0; j < VEC; ++j) acc[j] += old[j];
    }
    vstore<G, VEC>(g + c, acc);
  }
  }
}

// grad_pos[s + offset] (+)= sum_b dz[b*seq + s].  grid = (seq, ceil(h / (64*VEC))); the 4 waves
// of a block split the batch rows (4 independent load chains instead of one serial one) and
// combine in LDS in a fixed order (deterministic).
template <typename T, typename G, int VEC>
__global__ void __launch_bounds__(256) embed_pos_bwd_kernel(const T* __restrict__ dz, G* __restrict__ grad, int batch,
                                                            int seq, int h, int pos_offset, int accumulate) {
  __shared__ float sh[4][64 * VEC];
  const int s = blockIdx.x, lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = (blockIdx.y * 64 + lane) * VEC;
  float acc[VEC];
#pragma unroll
  for (int j = 0; j < VEC; ++j) acc[j] = 0.f;
  if (c < h) {
    for (int b = w; b < batch; b += 4) {
      float x[VEC];
      vload<T, VEC>(dz + ((size_t)b * seq + s) * h + c, x);
#pragma unroll
      for (int j = 0; j < VEC; ++j) acc[j] += x[j];
    }
  }
#pragma unroll
  for (int j = 0; j < VEC; ++j) sh[w][lane * VEC + j] = acc[j];
  __syncthreads();
  if (w == 0 && c < h) {
    float tot[VEC];
#pragma unroll
    for (int j = 0; j < VEC; ++j) tot[j] = (sh[0][lane * VEC + j] + sh[1][lane * VEC + j]) + (sh[2][lane * VEC + j] + sh[3][lane * VEC + j]);
    G* g = grad + (size_t)(s + pos_offset) * h + c;
    if (accumulate) {
      float old[VEC];
      vload<G, VEC>(g, old);
#pragma unroll
      for (int j = 0; j < VEC; ++j) tot[j] += old[j];
    }
    vstore<G, VEC>(g, tot);
  }
}

// Backward of a row gather (the sparse MLM head's labelled rows, models/layers.py::_GatherRows):
// out[r] = g[p] where idx[p] == r for p < n (idx[0:n) ascending, unique), else 0 -- one pass that
// writes every row once, instead of a zero fill plus an index_add.  n = min(*count, cap) when a
// device count is given (static-capacity gather: entries past the count are padding), else cap.
template <int VEC>
__global__ void __launch_bounds__(256) scatter_rows_kernel(const bf16* __restrict__ g, const int64_t* __restrict__ idx,
                                                           const int64_t* __restrict__ count, int cap,
                                                           bf16* __restrict__ out, int rows, int h) {
  const int lane = threadIdx.x & 63;
  const int n = count ? (int)min((int64_t)cap, *count) : cap;
  for (int r = blockIdx.x * 4 + (threadIdx.x >> 6); r < rows; r += gridDim.x * 4) {
    int lo = 0, hi = n;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (idx[mid] < r) lo = mid + 1;
      else hi = mid;
    }
    const bool hit = lo < n && idx[lo] == r;
    bf16* o = out + (size_t)r * h;
    for (int c = lane * VEC; c < h; c += 64 * VEC) {
      float v[VEC];
      if (hit) {
        vload<bf16, VEC>(g + (size_t)lo * h + c, v);
      } else {
#pragma unroll
        for (int j = 0; j < VEC; ++j) v[j] = 0.f;
      }
      vstore<bf16, VEC>(o + c, v);
    }
  }
}

template <typename T>
// y = dropout(x), or y = res + dropout(x) with the sum in fp32 (pre-LN residual branch: one pass
// instead of a dropout pass + an add pass)
__global__ void __launch_bounds__(256) dropout_kernel(const T* __restrict__ x, const T* __restrict__ res,
                                                      T* __restrict__ y, size_t n, float p,
                                                      const uint64_t* rng, uint32_t stream_id) {
  DropoutRng g(rng, stream_id);
  const uint32_t thr = keep_threshold(p);
  const float scale = 1.f / (1.f - p);
  const size_t nv = n / 8;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nv; i += (size_t)gridDim.x * blockDim.x) {
    float t[8];
    vload<T, 8>(x + i * 8, t);
#pragma unroll
    for (int j = 0; j < 8; j += 2) {
      const uint32_t b = g.bits((i * 8 + j) >> 1);
      t[j] *= ((b & 0xffffu) >= thr) ? scale : 0.f;
      t[j + 1] *= ((b >> 16) >= thr) ? scale : 0.f;
    }
    if (res) {
      float u[8];
      vload<T, 8>(res + i * 8, u);
#pragma unroll
      for (int j = 0; j < 8; ++j) t[j] += u[j];
    }
    vstore<T, 8>(y + i * 8, t);
  }
  if (blockIdx.x == 0) {
    for (size_t e = nv * 8 + threadIdx.x; e < n; e += blockDim.x) {
      const uint32_t b = g.bits(e >> 1);
      const uint32_t h16 = (e & 1) ? (b >> 16) : (b & 0xffffu);
      y[e] = (T)((float)x[e] * (h16 >= thr ? scale : 0.f) + (res ? (float)res[e] : 0.f));
    }
  }
}

}  // namespace

DTD_EXPORT int dtd_scatter_rows(const void* g, const int64_t* idx, const int64_t* count, int cap, void* out, int rows,
                                int h, hipStream_t s) {
  if (rows <= 0) return 0;
  if (h % 8 || ((uintptr_t)g | (uintptr_t)out) % 16) return (int)hipErrorInvalidValue;
  const dim3 grid(std::min((rows + 3) / 4, 256 * 8));
  hipLaunchKernelGGL(scatter_rows_kernel<8>, grid, dim3(256), 0, s, (const bf16*)g, idx, count, cap, (bf16*)out, rows, h);
  DTD_LAUNCH_CHECK();
}

DTD_EXPORT int dtd_embed_fwd(int dtype, const int64_t* ids, const int64_t* type_ids, const void* word, const void* pos,
                             const void* type, void* out, int rows, int h, int seq, int pos_offset, hipStream_t s) {
  if (rows <= 0) return 0;
  if (h % 2) return (int)hipErrorInvalidValue;
  GatherArgs a{ids, type_ids, word, pos, type, out, rows, h, seq, pos_offset};
  const dim3 grid((rows + 3) / 4);
  if (dtype == kBF16) {
    if (h % 8 == 0) hipLaunchKernelGGL((embed_fwd_kernel<bf16, 8>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((embed_fwd_kernel<bf16, 2>), grid, dim3(256), 0, s, a);
  } else {
    if (h % 4 == 0) hipLaunchKernelGGL((embed_fwd_kernel<float, 4>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((embed_fwd_kernel<float, 2>), grid, dim3(256), 0, s, a);
  }
  DTD_LAUNCH_CHECK();
}

DTD_EXPORT int dtd_embed_word_bwd(int dtype, int grad_dtype, const int64_t* sorted_ids, const int64_t* perm,
                                  const void* dz, void* grad, int rows, int h, int accumulate, int padding_idx,
                                  hipStream_t s) {
  if (rows <= 0) return 0;
  if (dtype == kBF16 && grad_dtype == kBF16)
    hipLaunchKernelGGL((embed_word_bwd_kernel<bf16, bf16>), dim3(rows), dim3(256), 0, s, sorted_ids, perm, (const bf16*)dz, (bf16*)grad, rows, h, accumulate, padding_idx);
  else if (dtype == kBF16)
    hipLaunchKernelGGL((embed_word_bwd_kernel<bf16, float>), dim3(rows), dim3(256), 0, s, sorted_ids, perm, (const bf16*)dz, (float*)grad, rows, h, accumulate, padding_idx);
  else if (grad_dtype == kBF16)
    hipLaunchKernelGGL((embed_word_bwd_kernel<float, bf16>), dim3(rows), dim3(256), 0, s, sorted_ids, perm, (const float*)dz, (bf16*)grad, rows, h, accumulate, padding_idx);
  else
    hipLaunchKernelGGL((embed_word_bwd_kernel<float, float>), dim3(rows), dim3(256), 0, s, sorted_ids, perm, (const float*)dz, (float*)grad, rows, h, accumulate, padding_idx);
  DTD_LAUNCH_CHECK();
}

DTD_EXPORT int dtd_embed_pos_bwd(int dtype, int grad_dtype, const void* dz, void* grad, int batch, int seq, int h,
                                 int pos_offset, int accumulate, hipStream_t s) {
  if (batch <= 0) return 0;
#define DTD_POS_BWD(T, G, V)                                                                              \
  hipLaunchKernelGGL((embed_pos_bwd_kernel<T, G, V>), dim3(seq, (h + 64 * V - 1) / (64 * V)), dim3(256), 0, s, \
                     (const T*)dz, (G*)grad, batch, seq, h, pos_offset, accumulate)
#define DTD_POS_BWD_V(T, G) \
  if (h % 8 == 0) { DTD_POS_BWD(T, G, 8); } else if (h % 2 == 0) { DTD_POS_BWD(T, G, 2); } else { DTD_POS_BWD(T, G, 1); }
  if (dtype == kBF16 && grad_dtype == kBF16) { DTD_POS_BWD_V(bf16, bf16) }
  else if (dtype == kBF16) { DTD_POS_BWD_V(bf16, float) }
  else if (grad_dtype == kBF16) { DTD_POS_BWD_V(float, bf16) }
  else { DTD_POS_BWD_V(float, float) }
#undef DTD_POS_BWD_V
#undef DTD_POS_BWD
  DTD_LAUNCH_CHECK();
}

// y = dropout(x) (res == nullptr) or y = res + dropout(x)
DTD_EXPORT int dtd_dropout(int dtype, const void* x, const void* res, void* y, size_t n, float p, const uint64_t* rng,
                           uint32_t stream_id, hipStream_t s) {
  if (n == 0) return 0;
  size_t blocks = (n / 8 + 255) / 256;
  if (blocks < 1) blocks = 1;
  if (blocks > 4096) blocks = 4096;
  if (dtype == kBF16)
    hipLaunchKernelGGL(dropout_kernel<bf16>, dim3(blocks), dim3(256), 0, s, (const bf16*)x, (const bf16*)res, (bf16*)y, n,
                       p, rng, stream_id);
  else
    hipLaunchKernelGGL(dropout_kernel<float>, dim3(blocks), dim3(256), 0, s, (const float*)x, (const float*)res,
                       (float*)y, n, p, rng, stream_id);
  DTD_LAUNCH_CHECK();
}

DTD_EXPORT int dtd_embed_word_bwd_chunked(int dtype, int grad_dtype, const int64_t* sorted_ids, const int64_t* perm,
                                          const int64_t* seg_lo, const int64_t* seg_hi, float* scratch, const void* dz,
                                          void* grad, int rows, int h, int accumulate, int padding_idx, hipStream_t s) {
  if (rows <= 0) return 0;
  const dim3 grid(std::min((rows + 3) / 4, 256 * 6));   // grid-stride kernels: one round of waves
#define DTD_EMB_LAUNCH(V)                                                                                      \
  if (dtype == kBF16)                                                                                          \
    hipLaunchKernelGGL((embed_chunk_sum_kernel<bf16, V>), grid, dim3(256), 0, s, perm, seg_lo, seg_hi,         \
                       (const bf16*)dz, scratch, rows, h);                                                     \
  else                                                                                                         \
    hipLaunchKernelGGL((embed_chunk_sum_kernel<float, V>), grid, dim3(256), 0, s, perm, seg_lo, seg_hi,        \
                       (const float*)dz, scratch, rows, h);                                                    \
  if (grad_dtype == kBF16)                                                                                     \
    hipLaunchKernelGGL((embed_chunk_add_kernel<bf16, V>), grid, dim3(256), 0, s, sorted_ids, seg_lo, seg_hi,   \
                       scratch, (bf16*)grad, rows, h, accumulate, padding_idx);                                \
  else                                                                                                         \
    hipLaunchKernelGGL((embed_chunk_add_kernel<float, V>), grid, dim3(256), 0, s, sorted_ids, seg_lo, seg_hi,  \
                       scratch, (float*)grad, rows, h, accumulate, padding_idx)
  if (h % 8 == 0) { DTD_EMB_LAUNCH(8); } else if (h % 2 == 0) { DTD_EMB_LAUNCH(2); } else { DTD_EMB_LAUNCH(1); }
#undef DTD_EMB_LAUNCH
  DTD_LAUNCH_CHECK();
}
