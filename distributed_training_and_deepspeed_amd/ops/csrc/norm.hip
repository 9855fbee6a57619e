// Fused residual-add + dropout + LayerNorm (forward and backward) for gfx950.
//
// Replaces the reference's separate ATen kernels for `dropout(y)`, `x + residual` and
// `nn.LayerNorm` (HF BertSelfOutput/BertOutput post-LN, OPT/GPT-2/BLOOM pre-LN;
// SURVEY.md K4/K6, reference model/transformer.py:95-104).
//
//   forward :  z   = r + dropout(y)            (y or r may be absent)
//              out = (z - mean) * rstd * gamma + beta
//   backward:  dz  = rstd * (g - mean(g) - xhat * mean(g * xhat)) + dz_extra,  g = (dout + dout2) * gamma
//              dy  = dropout_bwd(dz)                              (mask regenerated, not stored)
//              column partials of dout*xhat (dgamma), dout (dbeta), dy (bias of y's producer)
//
// Layout: one 64-lane wave per row while a row fits in registers (h <= 2048), lane l holding
// VEC contiguous elements at column (c*64 + l)*VEC for c < ITERS, so every access is a
// coalesced 8/16-byte-per-lane vector access and the two-pass mean/variance stays in registers.
// Wider rows (the h=9216 estimator block) take a block-per-row kernel.  Column partials
// are reduced inside the block through LDS and written once per block; `dtd_colsum_finalize`
// sums them in a fixed order, so parameter gradients are bitwise deterministic (no atomics).
#include "common.h"

using namespace dtd;

namespace {

struct LnFwdArgs {
  const void* y; const void* r; const void* gamma; const void* beta;
  void* z; void* out; float* mean; float* rstd;
  int rows, h; float eps, p; const uint64_t* rng; uint32_t stream_id;
};

struct LnBwdArgs {
  const void* dout; const void* dout2;  // dout2: optional second upstream gradient term
  const void* dz_extra; const void* z; const float* mean; const float* rstd;
  const void* gamma; void* dz; void* dy; float* part_gamma; float* part_beta; float* part_bias;
  int rows, h; float p; const uint64_t* rng; uint32_t stream_id;
  const void* xo; const void* beta;     // memory-efficient form: LN output + beta instead of z / mean
};

// keep/scale for element e of a [rows, h] tensor.
__device__ __forceinline__ float drop_factor(const DropoutRng& g, uint64_t e, uint32_t thr, float scale) {
  uint32_t b = g.bits(e >> 1);
  uint32_t h16 = (e & 1) ? (b >> 16) : (b & 0xffffu);
  return h16 >= thr ? scale : 0.f;
}

// Sum over the LPR lanes of a row group (LPR = 64: whole wave; 32: half-wave rows).
template <int LPR>
__device__ __forceinline__ float row_sum(float v) {
#pragma unroll
  for (int o = LPR / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// NT bit 0 / bit 1: streaming (non-temporal) loads / stores of the [rows, h] tensors (common.h)
#define LDNT(p, o) do { if (NT & 1) vload_nt<T, VEC>(p, o); else vload<T, VEC>(p, o); } while (0)
#define STNT(p, o) do { if (NT & 2) vstore_nt<T, VEC>(p, o); else vstore<T, VEC>(p, o); } while (0)

// LPR lanes per row (64, or 32 = two rows per wave so that h = 768 / 1280 rows still move in
// 16-byte bf16x8 vectors: 768 = 32 lanes x 3 x 8).
template <typename T, int VEC, int ITERS, int LPR, int NT>
__global__ void __launch_bounds__(256) ln_fwd_wave(LnFwdArgs a) {
  constexpr int NPL = VEC * ITERS, RPW = 64 / LPR;
  const int lane = threadIdx.x & 63, sub = lane % LPR;
  const int row0 = (blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * RPW + lane / LPR;
  const bool valid = row0 < a.rows;
  const int row = valid ? row0 : a.rows - 1;     // keep every lane of the wave in the shuffles
  const int h = a.h;
  const size_t base = (size_t)row * h;
  const bool has_drop = a.p > 0.f && a.y != nullptr;
  DropoutRng g(a.rng, a.stream_id);
  const uint32_t thr = keep_threshold(a.p);
  const float scale = has_drop ? 1.f / (1.f - a.p) : 1.f;
  float z[NPL];
#pragma unroll
  for (int c = 0; c < ITERS; ++c) {
    const int col = (c * LPR + sub) * VEC;
    float t[VEC];
    if (a.y) {
      LDNT((const T*)a.y + base + col, t);
      if (has_drop) {
#pragma unroll
        for (int j = 0; j < VEC; ++j) t[j] *= drop_factor(g, base + col + j, thr, scale);
      }
    } else {
#pragma unroll
      for (int j = 0; j < VEC; ++j) t[j] = 0.f;
    }
    if (a.r) {
      float rr[VEC];
      LDNT((const T*)a.r + base + col, rr);
#pragma unroll
      for (int j = 0; j < VEC; ++j) t[j] += rr[j];
    }
    if (a.z && valid) STNT((T*)a.z + base + col, t);
#pragma unroll
    for (int j = 0; j < VEC; ++j) z[c * VEC + j] = t[j];
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NPL; ++i) s += z[i];
  const float mu = row_sum<LPR>(s) / h;
  float v = 0.f;
#pragma unroll
  for (int i = 0; i < NPL; ++i) { float d = z[i] - mu; v += d * d; }
  const float rs = rsqrtf(row_sum<LPR>(v) / h + a.eps);
  if (!valid) return;
  if (sub == 0) { a.mean[row] = mu; a.rstd[row] = rs; }
#pragma unroll
  for (int c = 0; c < ITERS; ++c) {
    const int col = (c * LPR + sub) * VEC;
    float gm[VEC], bt[VEC], o[VEC];
    vload<T, VEC>((const T*)a.gamma + col, gm);
    vload<T, VEC>((const T*)a.beta + col, bt);
#pragma unroll
    for (int j = 0; j < VEC; ++j) o[j] = (z[c * VEC + j] - mu) * rs * gm[j] + bt[j];
    STNT((T*)a.out + base + col, o);
  }
}

// Raw (unconverted) VEC-element vector of a [rows, h] tensor: the backward's next-row prefetch
// holds its loads packed (bf16: VEC / 2 registers) until the row is processed.
template <typename T, int N> struct RawVec { typedef T type __attribute__((ext_vector_type(N))); };
template <typename T, int VEC, int NT>
__device__ __forceinline__ typename RawVec<T, VEC>::type ld_raw(const T* p) {
  typedef typename RawVec<T, VEC>::type vt;
  if constexpr ((NT & 1) != 0) return __builtin_nontemporal_load(reinterpret_cast<const vt*>(p));
  else return *reinterpret_cast<const vt*>(p);
}

// x-hat of the memory-efficient backward (FO): the forward stored only its output
// o = x-hat * gamma + beta, so x-hat = (o - beta) / gamma (reciprocal of gamma held per lane;
// |gamma| is clamped at 1e-12 -- an exactly-zero gamma column gets x-hat 0 and no dgamma, the
// known limit of the form).
__device__ __forceinline__ float safe_rcp(float g) {
  return 1.f / (fabsf(g) < 1e-12f ? copysignf(1e-12f, g) : g);
}

// One row per wave (the two-rows-per-wave layout of the forward doubles this kernel's per-lane
// state and costs occupancy).  The row loop is software-pipelined: the next row's loads (z or the
// LN output, dout, dout2, rstd) are issued before this row's reductions, so each wave keeps one
// row of HBM reads in flight behind its arithmetic instead of a serial load -> reduce -> store
// chain.  FO: x-hat from the LN output (LnBwdArgs::xo, beta) instead of z and the mean.
template <typename T, int VEC, int ITERS, int NT, bool FO, bool PF>
__global__ void __launch_bounds__(256) ln_bwd_wave(LnBwdArgs a) {
  constexpr int NPL = VEC * ITERS, LPR = 64;
  typedef typename RawVec<T, VEC>::type vt;
  // the row is wave-uniform: readfirstlane lets hipcc keep the row base in SGPRs (saddr loads /
  // stores with a 32-bit lane offset) instead of a 64-bit address pair per access
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), nw = blockDim.x >> 6;
  const int sub = lane;
  const int h = a.h;
  const bool has_drop = a.p > 0.f && a.dy != nullptr;
  DropoutRng g(a.rng, a.stream_id);
  const uint32_t thr = keep_threshold(a.p);
  const float scale = has_drop ? 1.f / (1.f - a.p) : 1.f;
  float pg[NPL], pb[NPL], py[NPL];
  // LDS: FO's per-column constants during the row loop, the column-partial reduction after it
  __shared__ __attribute__((aligned(16))) float sh[4][2048];  // nw <= 4 waves, h <= 2048
  // non-FO: gamma stays packed (bf16: VEC / 2 registers per chunk) and is widened at each use.
  // FO: gamma, beta and 1/gamma as fp32 columns in LDS, re-read (ds_read_b128) for every row --
  // the compiler barrier at the top of each row stops hipcc from hoisting them as 3 x NPL loop
  // invariants into registers (4 -> 3 waves / SIMD: measured slower than the extra LDS reads)
  vt gmr[FO ? 1 : ITERS];
  float* const cg = &sh[0][0];
  float* const cb = cg + h;
  float* const cr = cb + h;
#pragma unroll
  for (int i = 0; i < NPL; ++i) { pg[i] = 0.f; pb[i] = 0.f; py[i] = 0.f; }
  if constexpr (!FO) {
#pragma unroll
    for (int c = 0; c < ITERS; ++c) gmr[c] = ld_raw<T, VEC, 0>((const T*)a.gamma + (c * LPR + sub) * VEC);
  } else {
    for (int col = threadIdx.x; col < h; col += blockDim.x) {
      const float gv = (float)((const T*)a.gamma)[col];
      cg[col] = gv;
      cb[col] = (float)((const T*)a.beta)[col];
      cr[col] = safe_rcp(gv);
    }
    __syncthreads();
  }
  const T* src = (const T*)(FO ? a.xo : a.z);
  const bool two = a.dout2 != nullptr;
  const int stride = gridDim.x * nw;
  vt nz[ITERS], nd[ITERS], ne[ITERS];
  float nmu = 0.f, nrs = 0.f;
  auto fetch = [&](int r) {
    const size_t b = (size_t)r * h;
#pragma unroll
    for (int c = 0; c < ITERS; ++c) {
      const int col = (c * LPR + sub) * VEC;
      nz[c] = ld_raw<T, VEC, NT>(src + b + col);
      nd[c] = ld_raw<T, VEC, NT>((const T*)a.dout + b + col);
      if (two) ne[c] = ld_raw<T, VEC, NT>((const T*)a.dout2 + b + col);
    }
    if constexpr (!FO) nmu = a.mean[r];
    nrs = a.rstd[r];
  };
  int row = blockIdx.x * nw + w;
  if (PF && row < a.rows) fetch(row);
  for (; row < a.rows; row += stride) {
    const size_t base = (size_t)row * h;
    if constexpr (FO) asm volatile("" ::: "memory");
    if (!PF) fetch(row);
    vt cz[ITERS], cd[ITERS], ce[ITERS];
#pragma unroll
    for (int c = 0; c < ITERS; ++c) { cz[c] = nz[c]; cd[c] = nd[c]; ce[c] = ne[c]; }
    const float mu = nmu, rs = nrs;
    if (PF && row + stride < a.rows) fetch(row + stride);
    float xh[NPL], dg[NPL];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int c = 0; c < ITERS; ++c) {
      float zz[VEC], dd[VEC];
#pragma unroll
      for (int j = 0; j < VEC; ++j) {
        zz[j] = (float)cz[c][j];
        dd[j] = (float)cd[c][j];
        if (two) dd[j] += (float)ce[c][j];
      }
#pragma unroll
      for (int j = 0; j < VEC; ++j) {
        const int i = c * VEC + j;
        float gmv;
        if constexpr (FO) {
          const int col = (c * LPR + sub) * VEC + j;
          gmv = cg[col];
          xh[i] = (zz[j] - cb[col]) * cr[col];
        } else {
          gmv = (float)gmr[c][j];
          xh[i] = (zz[j] - mu) * rs;
        }
        dg[i] = dd[j] * gmv;
        s1 += dg[i];
        s2 += dg[i] * xh[i];
        pg[i] += dd[j] * xh[i];
        pb[i] += dd[j];
      }
    }
    const float m1 = wave_sum(s1) / h, m2 = wave_sum(s2) / h;
#pragma unroll
    for (int c = 0; c < ITERS; ++c) {
      const int col = (c * LPR + sub) * VEC;
      float dz[VEC];
#pragma unroll
      for (int j = 0; j < VEC; ++j) {
        const int i = c * VEC + j;
        dz[j] = rs * (dg[i] - m1 - xh[i] * m2);
      }
      if (a.dz_extra) {
        float e[VEC];
        LDNT((const T*)a.dz_extra + base + col, e);
#pragma unroll
        for (int j = 0; j < VEC; ++j) dz[j] += e[j];
      }
      if (a.dz) STNT((T*)a.dz + base + col, dz);
      if (a.dy) {
        float dy[VEC];
#pragma unroll
        for (int j = 0; j < VEC; ++j) {
          dy[j] = has_drop ? dz[j] * drop_factor(g, base + col + j, thr, scale) : dz[j];
          py[c * VEC + j] += dy[j];
        }
        STNT((T*)a.dy + base + col, dy);
      }
    }
  }
  // Block-level reduction of the column partials through LDS (one array at a time; the first
  // barrier also retires every wave's reads of FO's constants)
  float* outs[3] = {a.part_gamma, a.part_beta, a.part_bias};
  float* srcs[3] = {pg, pb, py};
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    if (!outs[k]) continue;
    __syncthreads();
#pragma unroll
    for (int c = 0; c < ITERS; ++c)
#pragma unroll
      for (int j = 0; j < VEC; ++j) sh[w][(c * LPR + sub) * VEC + j] = srcs[k][c * VEC + j];
    __syncthreads();
    for (int col = threadIdx.x; col < h; col += blockDim.x) {
      float t = 0.f;
      for (int i = 0; i < nw; ++i) t += sh[i][col];
      outs[k][(size_t)blockIdx.x * h + col] = t;
    }
  }
}

#undef LDNT
#undef STNT

// ---- generic block-per-row kernels (any even h; used for h > 2048) ----
template <typename T>
__global__ void __launch_bounds__(256) ln_fwd_block(LnFwdArgs a) {
  __shared__ float red[8];
  const int row = blockIdx.x;
  const int h = a.h;
  const size_t base = (size_t)row * h;
  const bool has_drop = a.p > 0.f && a.y != nullptr;
  DropoutRng g(a.rng, a.stream_id);
  const uint32_t thr = keep_threshold(a.p);
  const float scale = has_drop ? 1.f / (1.f - a.p) : 1.f;
  float s = 0.f;
  // pass 1: z, written to a.z or (if absent) recomputed in pass 2/3
  for (int col = threadIdx.x * 2; col < h; col += blockDim.x * 2) {
    float t[2] = {0.f, 0.f};
    if (a.y) {
      vload<T, 2>((const T*)a.y + base + col, t);
      if (has_drop) { t[0] *= drop_factor(g, base + col, thr, scale); t[1] *= drop_factor(g, base + col + 1, thr, scale); }
    }
    if (a.r) { float rr[2]; vload<T, 2>((const T*)a.r + base + col, rr); t[0] += rr[0]; t[1] += rr[1]; }
    if (a.z) vstore<T, 2>((T*)a.z + base + col, t);
    s += t[0] + t[1];
  }
  const float mu = block_sum(s, red) / h;
  auto zval = [&](int col, float* t) {
    if (a.z) { vload<T, 2>((const T*)a.z + base + col, t); return; }
    t[0] = t[1] = 0.f;
    if (a.y) {
      vload<T, 2>((const T*)a.y + base + col, t);
      if (has_drop) { t[0] *= drop_factor(g, base + col, thr, scale); t[1] *= drop_factor(g, base + col + 1, thr, scale); }
    }
    if (a.r) { float rr[2]; vload<T, 2>((const T*)a.r + base + col, rr); t[0] += rr[0]; t[1] += rr[1]; }
  };
  float v = 0.f;
  for (int col = threadIdx.x * 2; col < h; col += blockDim.x * 2) {
    float t[2]; zval(col, t);
    v += (t[0] - mu) * (t[0] - mu) + (t[1] - mu) * (t[1] - mu);
  }
  const float rs = rsqrtf(block_sum(v, red) / h + a.eps);
  if (threadIdx.x == 0) { a.mean[row] = mu; a.rstd[row] = rs; }
  for (int col = threadIdx.x * 2; col < h; col += blockDim.x * 2) {
    float t[2], gm[2], bt[2], o[2];
    zval(col, t);
    vload<T, 2>((const T*)a.gamma + col, gm);
    vload<T, 2>((const T*)a.beta + col, bt);
    o[0] = (t[0] - mu) * rs * gm[0] + bt[0];
    o[1] = (t[1] - mu) * rs * gm[1] + bt[1];
    vstore<T, 2>((T*)a.out + base + col, o);
  }
}

// Block-per-row backward; column partials accumulate per block over a strided row set in
// a global partial row (each block owns row blockIdx.x of the partial arrays).
template <typename T>
__global__ void __launch_bounds__(256) ln_bwd_block(LnBwdArgs a) {
  __shared__ float red[8];
  const int h = a.h;
  const bool has_drop = a.p > 0.f && a.dy != nullptr;
  DropoutRng g(a.rng, a.stream_id);
  const uint32_t thr = keep_threshold(a.p);
  const float scale = has_drop ? 1.f / (1.f - a.p) : 1.f;
  float* pgp = a.part_gamma ? a.part_gamma + (size_t)blockIdx.x * h : nullptr;
  float* pbp = a.part_beta ? a.part_beta + (size_t)blockIdx.x * h : nullptr;
  float* pyp = a.part_bias ? a.part_bias + (size_t)blockIdx.x * h : nullptr;
  for (int col = threadIdx.x; col < h; col += blockDim.x) {
    if (pgp) pgp[col] = 0.f;
    if (pbp) pbp[col] = 0.f;
    if (pyp) pyp[col] = 0.f;
  }
  __syncthreads();
  for (int row = blockIdx.x; row < a.rows; row += gridDim.x) {
    const size_t base = (size_t)row * h;
    const float mu = a.xo ? 0.f : a.mean[row], rs = a.rstd[row];
    // x-hat of column pair col: from z and the mean, or (memory-efficient form) from the output
    auto xhat = [&](int col, const float* gm, float* xh) {
      float zz[2];
      if (a.xo) {
        float bt[2];
        vload<T, 2>((const T*)a.xo + base + col, zz);
        vload<T, 2>((const T*)a.beta + col, bt);
        xh[0] = (zz[0] - bt[0]) * safe_rcp(gm[0]);
        xh[1] = (zz[1] - bt[1]) * safe_rcp(gm[1]);
      } else {
        vload<T, 2>((const T*)a.z + base + col, zz);
        xh[0] = (zz[0] - mu) * rs;
        xh[1] = (zz[1] - mu) * rs;
      }
    };
    float s1 = 0.f, s2 = 0.f;
    for (int col = threadIdx.x * 2; col < h; col += blockDim.x * 2) {
      float xv[2], dd[2], gm[2];
      vload<T, 2>((const T*)a.dout + base + col, dd);
      if (a.dout2) { float e[2]; vload<T, 2>((const T*)a.dout2 + base + col, e); dd[0] += e[0]; dd[1] += e[1]; }
      vload<T, 2>((const T*)a.gamma + col, gm);
      xhat(col, gm, xv);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const float xh = xv[j], dg = dd[j] * gm[j];
        s1 += dg; s2 += dg * xh;
        if (pgp) pgp[col + j] += dd[j] * xh;   // same thread owns the same columns every row
        if (pbp) pbp[col + j] += dd[j];
      }
    }
    const float m1 = block_sum(s1, red) / h, m2 = block_sum(s2, red) / h;
    for (int col = threadIdx.x * 2; col < h; col += blockDim.x * 2) {
      float xv[2], dd[2], gm[2], dz[2];
      vload<T, 2>((const T*)a.dout + base + col, dd);
      if (a.dout2) { float e[2]; vload<T, 2>((const T*)a.dout2 + base + col, e); dd[0] += e[0]; dd[1] += e[1]; }
      vload<T, 2>((const T*)a.gamma + col, gm);
      xhat(col, gm, xv);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const float xh = xv[j], dg = dd[j] * gm[j];
        dz[j] = rs * (dg - m1 - xh * m2);
      }
      if (a.dz_extra) { float e[2]; vload<T, 2>((const T*)a.dz_extra + base + col, e); dz[0] += e[0]; dz[1] += e[1]; }
      if (a.dz) vstore<T, 2>((T*)a.dz + base + col, dz);
      if (a.dy) {
        float dy[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          dy[j] = has_drop ? dz[j] * drop_factor(g, base + col + j, thr, scale) : dz[j];
          if (pyp) pyp[col + j] += dy[j];
        }
        vstore<T, 2>((T*)a.dy + base + col, dy);
      }
    }
  }
}

// DTD_LN_BWD_PREFETCH=1: the software-pipelined row loop (next row's loads in flight behind this
// row's arithmetic, at 3 waves / SIMD); 0: one row's loads at a time at 4 waves / SIMD.
inline bool ln_bwd_prefetch() {
  const char* e = getenv("DTD_LN_BWD_PREFETCH");   // read per call (A/B tests flip it in-process)
  return e != nullptr && atoi(e) != 0;
}

template <typename T, int VEC, int ITERS, bool PF>
void launch_bwd(const LnBwdArgs& b, int nblocks, int nt, hipStream_t s) {
  const dim3 grid(nblocks), block(256);
  if (b.xo) {
    if (nt == 3) hipLaunchKernelGGL((ln_bwd_wave<T, VEC, ITERS, 3, true, PF>), grid, block, 0, s, b);
    else hipLaunchKernelGGL((ln_bwd_wave<T, VEC, ITERS, 0, true, PF>), grid, block, 0, s, b);
  } else {
    if (nt == 3) hipLaunchKernelGGL((ln_bwd_wave<T, VEC, ITERS, 3, false, PF>), grid, block, 0, s, b);
    else hipLaunchKernelGGL((ln_bwd_wave<T, VEC, ITERS, 0, false, PF>), grid, block, 0, s, b);
  }
}

template <typename T, int VEC, int ITERS, int LPR = 64>
bool try_wave(const LnFwdArgs* f, const LnBwdArgs* b, int nblocks_bwd, hipStream_t s) {
  const int h = f ? f->h : b->h;
  if (h != LPR * VEC * ITERS) return false;
  const int nt = ew_nt_bits();
  if (f) {
    const int rows_per_block = 4 * (64 / LPR);
    const dim3 grid((f->rows + rows_per_block - 1) / rows_per_block);
    switch (nt) {
      case 3: hipLaunchKernelGGL((ln_fwd_wave<T, VEC, ITERS, LPR, 3>), grid, dim3(256), 0, s, *f); break;
      default: hipLaunchKernelGGL((ln_fwd_wave<T, VEC, ITERS, LPR, 0>), grid, dim3(256), 0, s, *f); break;
    }
  } else if (ln_bwd_prefetch()) {
    launch_bwd<T, VEC, ITERS, true>(*b, nblocks_bwd, nt, s);
  } else {
    launch_bwd<T, VEC, ITERS, false>(*b, nblocks_bwd, nt, s);
  }
  return true;
}

template <typename T>
void dispatch(const LnFwdArgs* f, const LnBwdArgs* b, int nblocks_bwd, hipStream_t s) {
  if (try_wave<T, 2, 1>(f, b, nblocks_bwd, s)) return;      // h = 128
  if (try_wave<T, 4, 1>(f, b, nblocks_bwd, s)) return;      // 256
  if (try_wave<T, 8, 1>(f, b, nblocks_bwd, s)) return;      // 512
  // h = 768 / 1280: the forward moves two rows per wave in 16-byte vectors (faster: 23.2 ->
  // 19.8 us at 16k x 768); the backward keeps one row per wave (8-byte vectors) because its
  // per-lane state (x-hat, g, 3 partial arrays) doubles with two rows and costs occupancy
  // (24.4 -> 31.3 us measured).
  if (f && try_wave<T, 8, 3, 32>(f, b, nblocks_bwd, s)) return;   // 768 fwd
  if (!f && try_wave<T, 4, 3>(f, b, nblocks_bwd, s)) return;      // 768 bwd
  if (try_wave<T, 8, 2>(f, b, nblocks_bwd, s)) return;            // 1024
  if (f && try_wave<T, 8, 5, 32>(f, b, nblocks_bwd, s)) return;   // 1280 fwd
  if (!f && try_wave<T, 4, 5>(f, b, nblocks_bwd, s)) return;      // 1280 bwd
  if (try_wave<T, 8, 3>(f, b, nblocks_bwd, s)) return;      // 1536
  if (try_wave<T, 8, 4>(f, b, nblocks_bwd, s)) return;      // 2048
  if (f) hipLaunchKernelGGL((ln_fwd_block<T>), dim3(f->rows), dim3(256), 0, s, *f);
  else hipLaunchKernelGGL((ln_bwd_block<T>), dim3(nblocks_bwd), dim3(256), 0, s, *b);
}

// Embedding forward in one pass (SURVEY.md K7 + K4 + K6; HF BertEmbeddings): z = word[id] +
// pos[s + offset] + type[type_id] (fp32 sum, stored as bf16 for the LayerNorm backward), x =
// LN(z) of the stored bf16 z, out = dropout(bf16(x)).  Bit-identical to dtd_embed_fwd ->
// dtd_ln_fwd (r = z) -> dtd_dropout: the same lane / column map and row reduction as ln_fwd_wave
// and the same keep-bit law and element index as dropout_kernel, with the two intermediate
// [rows, h] round trips through HBM (z re-read, x written and re-read) gone.
struct EmbLnArgs {
  const int64_t* ids; const int64_t* type_ids; const void* word; const void* pos; const void* type;
  const void* gamma; const void* beta; void* z; void* out; float* mean; float* rstd;
  int rows, h, seq, pos_offset; float eps, p; const uint64_t* rng; uint32_t stream_id;
};

template <int VEC, int ITERS, int LPR>
__global__ void __launch_bounds__(256) emb_ln_fwd_wave(EmbLnArgs a) {
  using T = bf16;
  constexpr int NPL = VEC * ITERS, RPW = 64 / LPR;
  const int lane = threadIdx.x & 63, sub = lane % LPR;
  const int row0 = (blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * RPW + lane / LPR;
  const bool valid = row0 < a.rows;
  const int row = valid ? row0 : a.rows - 1;     // keep every lane of the wave in the shuffles
  const int h = a.h;
  const size_t base = (size_t)row * h;
  const int64_t id = a.ids[row];
  const int64_t ty = a.type_ids ? a.type_ids[row] : 0;
  const T* w = (const T*)a.word + (size_t)id * h;
  const T* ps = a.pos ? (const T*)a.pos + (size_t)((row % a.seq) + a.pos_offset) * h : nullptr;
  const T* tp = a.type ? (const T*)a.type + (size_t)ty * h : nullptr;
  float z[NPL];
#pragma unroll
  for (int c = 0; c < ITERS; ++c) {
    const int col = (c * LPR + sub) * VEC;
    float t[VEC], u[VEC];
    vload<T, VEC>(w + col, t);
    if (ps) {
      vload<T, VEC>(ps + col, u);
#pragma unroll
      for (int j = 0; j < VEC; ++j) t[j] += u[j];
    }
    if (tp) {
      vload<T, VEC>(tp + col, u);
#pragma unroll
      for (int j = 0; j < VEC; ++j) t[j] += u[j];
    }
#pragma unroll
    for (int j = 0; j < VEC; ++j) t[j] = (float)(T)t[j];   // the stored bf16 z feeds the LN
    if (valid) vstore_nt<T, VEC>((T*)a.z + base + col, t);
#pragma unroll
    for (int j = 0; j < VEC; ++j) z[c * VEC + j] = t[j];
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NPL; ++i) s += z[i];
  const float mu = row_sum<LPR>(s) / h;
  float v = 0.f;
#pragma unroll
  for (int i = 0; i < NPL; ++i) { float d = z[i] - mu; v += d * d; }
  const float rs = rsqrtf(row_sum<LPR>(v) / h + a.eps);
  if (!valid) return;
  if (sub == 0) { a.mean[row] = mu; a.rstd[row] = rs; }
  const bool has_drop = a.p > 0.f;
  DropoutRng g(a.rng, a.stream_id);
  const uint32_t thr = keep_threshold(a.p);
  const float scale = has_drop ? 1.f / (1.f - a.p) : 1.f;
#pragma unroll
  for (int c = 0; c < ITERS; ++c) {
    const int col = (c * LPR + sub) * VEC;
    float gm[VEC], bt[VEC], o[VEC];
    vload<T, VEC>((const T*)a.gamma + col, gm);
    vload<T, VEC>((const T*)a.beta + col, bt);
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      o[j] = (float)(T)((z[c * VEC + j] - mu) * rs * gm[j] + bt[j]);   // x, rounded as stored
      if (has_drop) o[j] *= drop_factor(g, base + col + j, thr, scale);
    }
    vstore_nt<T, VEC>((T*)a.out + base + col, o);
  }
}

}  // namespace

// Number of partial rows the backward writes (callers size part_* as [n, h] fp32).
static bool wave_shape(int h) {
  return h == 128 || h == 256 || h == 512 || h == 768 || h == 1024 || h == 1280 || h == 1536 || h == 2048;
}
DTD_EXPORT int dtd_ln_bwd_num_partials(int rows, int h) {
  if (wave_shape(h)) {
    // up to 1024 blocks x 4 waves = 4 waves per SIMD on 256 CUs: the row loop is a serial chain
    // of loads -> wave reductions -> stores, so occupancy is what hides HBM latency
    // (the prefetching form holds 3 waves / SIMD: 768 blocks)
    const int cap = ln_bwd_prefetch() ? 768 : 1024;
    int blocks = (rows + 3) / 4;
    return blocks < cap ? blocks : cap;
  }
  return rows < 256 ? rows : 256;
}

DTD_EXPORT int dtd_ln_fwd(int dtype, const void* y, const void* r, const void* gamma, const void* beta,
                          void* z, void* out, float* mean, float* rstd, int rows, int h, float eps,
                          float p, const uint64_t* rng, uint32_t stream_id, hipStream_t s) {
  if (rows <= 0) return 0;
  LnFwdArgs a{y, r, gamma, beta, z, out, mean, rstd, rows, h, eps, p, rng, stream_id};
  if (dtype == kBF16) dispatch<bf16>(&a, nullptr, 0, s);
  else dispatch<float>(&a, nullptr, 0, s);
  DTD_LAUNCH_CHECK();
}

DTD_EXPORT int dtd_ln_bwd(int dtype, const void* dout, const void* dout2, const void* dz_extra, const void* z,
                          const float* mean, const float* rstd, const void* gamma, void* dz, void* dy,
                          float* part_gamma, float* part_beta, float* part_bias, int rows, int h,
                          float p, const uint64_t* rng, uint32_t stream_id, hipStream_t s) {
  if (rows <= 0) return 0;
  LnBwdArgs a{dout, dout2, dz_extra, z, mean, rstd, gamma, dz, dy, part_gamma, part_beta, part_bias,
              rows, h, p, rng, stream_id, nullptr, nullptr};
  const int nb = dtd_ln_bwd_num_partials(rows, h);
  if (dtype == kBF16) dispatch<bf16>(nullptr, &a, nb, s);
  else dispatch<float>(nullptr, &a, nb, s);
  DTD_LAUNCH_CHECK();
}

// Memory-efficient backward: x-hat recomputed from the LayerNorm output xo = x-hat * gamma + beta
// (the forward stored no z; Apex's memory_efficient LayerNorm form).  Same outputs as dtd_ln_bwd.
DTD_EXPORT int dtd_ln_bwd_fo(int dtype, const void* dout, const void* dout2, const void* dz_extra, const void* xo,
                             const void* beta, const float* rstd, const void* gamma, void* dz, void* dy,
                             float* part_gamma, float* part_beta, float* part_bias, int rows, int h, float p,
                             const uint64_t* rng, uint32_t stream_id, hipStream_t s) {
  if (rows <= 0) return 0;
  if (xo == nullptr || beta == nullptr) return (int)hipErrorInvalidValue;
  LnBwdArgs a{dout, dout2, dz_extra, nullptr, nullptr, rstd, gamma, dz, dy, part_gamma, part_beta, part_bias,
              rows, h, p, rng, stream_id, xo, beta};
  const int nb = dtd_ln_bwd_num_partials(rows, h);
  if (dtype == kBF16) dispatch<bf16>(nullptr, &a, nb, s);
  else dispatch<float>(nullptr, &a, nb, s);
  DTD_LAUNCH_CHECK();
}

// Fused embedding gather-sum + LayerNorm + dropout (bf16, h = 768 or 1024; else -1: the caller
// takes dtd_embed_fwd -> dtd_ln_fwd -> dtd_dropout).  z [rows, h] (LN input, for the backward),
// out [rows, h], mean / rstd [rows].
DTD_EXPORT int dtd_embed_ln_fwd(const int64_t* ids, const int64_t* type_ids, const void* word, const void* pos,
                                const void* type, const void* gamma, const void* beta, void* z, void* out, float* mean,
                                float* rstd, int rows, int h, int seq, int pos_offset, float eps, float p,
                                const uint64_t* rng, uint32_t stream_id, hipStream_t s) {
  if (rows <= 0) return 0;
  if (seq <= 0 || rng == nullptr) return (int)hipErrorInvalidValue;   // rng is read even at p = 0
  EmbLnArgs a{ids, type_ids, word, pos, type, gamma, beta, z, out, mean, rstd, rows, h, seq, pos_offset, eps, p,
              rng, stream_id};
  if (h == 768) {
    hipLaunchKernelGGL((emb_ln_fwd_wave<8, 3, 32>), dim3((rows + 7) / 8), dim3(256), 0, s, a);
  } else if (h == 1024) {
    hipLaunchKernelGGL((emb_ln_fwd_wave<8, 2, 64>), dim3((rows + 3) / 4), dim3(256), 0, s, a);
  } else {
    return -1;
  }
  DTD_LAUNCH_CHECK();
}
