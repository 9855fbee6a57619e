// MFMA GEMM with fused transformer epilogues for gfx950 (MI355X / CDNA4).
//
//   C[M, N] = A[M, K] . B[N, K]^T        bf16 in, fp32 accumulate, both operands K-contiguous
//
// A Linear layer's forward is exactly this product (B = the [out, in] weight); its input-gradient
// product uses B = W^T (a cached transposed copy, `dtd_transpose_bf16` below).  The epilogues fuse
// the elementwise passes that would otherwise re-read the GEMM output from HBM:
//   EPI_STORE      C = acc (+ bias[n])                          Linear forward / dgrad
//   EPI_BIAS_GELU  U = acc + bias; A = gelu(U); store U and A    FFN up-projection forward
//   EPI_GELU_BWD   dU = bf16(acc) * gelu'(U); store dU; column   FFN down-projection dgrad + GELU'
//                  partial sums of dU (the up-projection's bias gradient, finalised by colsum)
//   EPI_ADD        C = C + acc (in place)                       residual-branch dgrad (post-LN BERT)
//   EPI_BIAS_GELU_TANH / EPI_GELU_TANH_BWD, EPI_BIAS_RELU / EPI_RELU_BWD: the same two
//                  activation epilogues for tanh GELU (GPT-2 / BLOOM "gelu_new") and ReLU (OPT)
//   EPI_BIAS_GELU_G / EPI_BIAS_GELU_TANH_G   A = act(U) and G = act'(U) (U = acc + bias rounded
//                  to bf16, as above) from the same exponential; store G in place of U
//   EPI_MUL_BWD    dU = bf16(acc) * G (G = the stored derivative); column partials of dU.  The
//                  pair moves the derivative's transcendental math out of the backward epilogue
//                  (a multiply there) into the forward one, where it shares GELU's exp / rcp
//
// Main loop (cdna_hip_programming.md §5, "256² 8-phase template"): 256x256 output tile per
// 512-thread workgroup, 8 waves as 2 (M) x 4 (N), each wave 128 x 64 as 8 x 4 tiles of
// v_mfma_f32_16x16x32_bf16.  K-steps of 64 live in two 64 KiB LDS buffers (ONE __shared__ array);
// each K-step is four phases, one per 64x32 quadrant of the wave's output (16 MFMAs each), and
// every phase stages one quarter ("half-tile", 16 KiB) of the NEXT K-step by 16-byte LDS-DMA
// (global_load_lds_dwordx4): A-rows-lo, B-cols-lo, B-cols-hi, A-rows-hi -- the order the next
// K-step's phases read them.  A counted `s_waitcnt vmcnt(4)` per phase retires the DMA issued two
// phases earlier (never vmcnt(0) in the loop), and raw s_barriers order it for the readers.
// The two wave rows run one barrier apart (stagger): while one half of a SIMD's waves issues its
// MFMAs the other half reads its LDS fragments, so the matrix pipe sees back-to-back MFMA
// segments.  LDS rows are 128 B with the 16-byte chunk index XOR-swizzled by (row & 7): DMA
// destinations stay lane-linear, the SOURCE address carries the (involutive) swizzle, and every
// ds_read_b128 fragment read is bank-conflict free.  MFMAs take the B fragment as their first
// operand (the tile is computed transposed), so a lane's accumulator holds 4 consecutive columns
// of one row.
//
// Epilogue: the accumulators (with bias / residual added in fp32, one rounding) go to LDS as a
// 256 x 256 bf16 image (8-byte column slots XOR-swizzled by row & 15: conflict-free writes), and
// are read back row-major so every global store (and the GELU-backward U load) is a full 512-byte
// row segment of 16-byte vectors.  XCD-aware bijective tile order (T1).
#include <type_traits>

#ifndef DTD_GEMM_DIAG
#define DTD_GEMM_DIAG 0
#endif
// DTD_GEMM_ONEBAR=1 (variant build): one barrier per phase and no wave-row stagger in the
// persistent kernel -- both waves of a SIMD reach their MFMAs together and the matrix pipe
// arbitrates between them (4 barriers per K-step instead of 8)
#ifndef DTD_GEMM_ONEBAR
#define DTD_GEMM_ONEBAR 0
#endif
constexpr bool kOneBar = DTD_GEMM_ONEBAR != 0;

#include "common.h"

using namespace dtd;

namespace {

typedef __attribute__((address_space(3))) void lds_void;
typedef const __attribute__((address_space(1))) void gbl_void;

constexpr int BM = 256, BN = 256, BK = 64;
constexpr int A_BYTES = BM * BK * 2;             // 32 KiB
constexpr int TILE_BYTES = (BM + BN) * BK * 2;   // 64 KiB per K-step buffer
constexpr int LDS_BYTES = 2 * TILE_BYTES;        // 128 KiB

enum Epi : int { EPI_STORE = 0, EPI_BIAS_GELU = 1, EPI_GELU_BWD = 2, EPI_ADD = 3, EPI_BIAS_GELU_TANH = 4,
                 EPI_GELU_TANH_BWD = 5, EPI_BIAS_RELU = 6, EPI_RELU_BWD = 7, EPI_BIAS_GELU_G = 8,
                 EPI_BIAS_GELU_TANH_G = 9, EPI_MUL_BWD = 10, EPI_LAST = EPI_MUL_BWD };
// activation epilogues (the names keep "gelu" for the family: store U and act(U) / act'(U) . dA)
__host__ __device__ constexpr bool is_gelu_fwd(int e) {
  return e == EPI_BIAS_GELU || e == EPI_BIAS_GELU_TANH || e == EPI_BIAS_RELU || e == EPI_BIAS_GELU_G ||
         e == EPI_BIAS_GELU_TANH_G;
}
__host__ __device__ constexpr bool is_gelu_bwd(int e) {
  return e == EPI_GELU_BWD || e == EPI_GELU_TANH_BWD || e == EPI_RELU_BWD || e == EPI_MUL_BWD;
}
// forward activation epilogues that store the derivative G in place of U
__host__ __device__ constexpr bool stores_grad(int e) { return e == EPI_BIAS_GELU_G || e == EPI_BIAS_GELU_TANH_G; }

struct GemmArgs {
  const bf16* a; const bf16* b;          // A [M, K] (lda), B [N, K] (ldb)
  bf16* c;                               // STORE / ADD: C; BIAS_GELU: U; GELU_BWD: dU   (ldc)
  bf16* c2;                              // BIAS_GELU: A = gelu(U) (ldc)
  const bf16* u;                         // GELU_BWD: pre-activation U (ldu)
  const bf16* bias;                      // [N] or null (STORE, BIAS_GELU)
  float* part;                           // GELU_BWD: [M / 256][N] fp32 column partials (or null)
  int M, N, K, lda, ldb, ldc, ldu;
  unsigned long long* stamps;            // diagnostic builds only (-DDTD_GEMM_STAMPS), else null
  int* sched;                            // persistent form: dynamic tile queue (see below) or null
  int stagger;                           // persistent form: start delay (10 ns ticks) of odd members
  int nt;                                // persistent form: non-temporal epilogue stores (DTD_GEMM_NT_STORE)
};

// 16-byte epilogue store, non-temporal when `nt` (a wave-uniform flag)
__device__ __forceinline__ void st8(bf16* p, const bf16x8& v, int nt) {
  if (nt) __builtin_nontemporal_store(v, reinterpret_cast<bf16x8*>(p));
  else *reinterpret_cast<bf16x8*>(p) = v;
}

// Dynamic tile queue of the persistent form: sched[x] (x = 0..7) is the next unclaimed tile of XCD
// group x (after the 2 x 32 tiles per group the static order hands out first), sched[8] counts finished
// workgroups.  A workgroup starts with its first two static tiles; each tile's epilogue claims the
// tile after the next one (one device-scope atomic issued when the epilogue starts, its result handed to the
// other waves through LDS when it ends: the latency hides behind the epilogue and the main loop
// keeps the static form's registers and schedule), so workgroups that start late -- CUs held
// by an RCCL kernel on the comm stream, or by a side-stream kernel -- take fewer tiles instead of
// stretching the launch by their delay.  The last workgroup to finish zeroes the queue for the next
// launch on the same stream (one queue per stream: ops/gemm.py).
constexpr int SCHED_DONE = 8;

// In-kernel timing stamps (diagnostic build, scripts/gemm_stamps.py): lane 0 of wave 0 records
// s_memtime at fixed points of each tile, plus the CU / XCC ids, with plain vector stores.
#ifdef DTD_GEMM_STAMPS
#define STAMP(slot, iter)                                                                          \
  do {                                                                                             \
    if (g.stamps && tid == 0 && (iter) < 32)                                                       \
      g.stamps[((size_t)blockIdx.x * 32 + (iter)) * 8 + (slot)] = __builtin_amdgcn_s_memtime();    \
  } while (0)
#define STAMP_ID(iter)                                                                             \
  do {                                                                                             \
    if (g.stamps && tid == 0 && (iter) < 32)                                                       \
      g.stamps[((size_t)blockIdx.x * 32 + (iter)) * 8 + 7] =                                       \
          ((unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32) |                 \
          __builtin_amdgcn_s_getreg((31 << 11) | 4);                                               \
  } while (0)
#else
#define STAMP(slot, iter) do {} while (0)
#define STAMP_ID(iter) do {} while (0)
#endif

// raw workgroup barrier (no vmcnt drain: LDS-DMA may stay in flight across it) that the compiler
// also treats as a memory barrier, so no LDS access is hoisted or sunk across it
__device__ __forceinline__ void bar() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// GELU(erf) and its derivative from one exponential (the formulas of act.hip)
__device__ __forceinline__ float phi_cdf(float x, float e) {
  // t = 1 / (1 + p |x| / sqrt 2): one FMA with an |x| source modifier
  const float t = __builtin_amdgcn_rcpf(fmaf(fabsf(x), 0.3275911f * 0.70710678118654752f, 1.f));
  const float poly = t * fmaf(t, fmaf(t, fmaf(t, fmaf(t, 1.061405429f, -1.453152027f), 1.421413741f), -0.284496736f),
                              0.254829592f);
  return 0.5f + 0.5f * copysignf(1.f - poly * e, x);
}
// exp(-x^2 / 2) as v_exp_f32 (= 2^y) of y = x^2 * (-log2(e) / 2): two multiplies (packable)
__device__ __forceinline__ float gauss_e(float x) { return __builtin_amdgcn_exp2f((x * x) * -0.72134752044448170f); }
__device__ __forceinline__ float gelu(float x) { return x * phi_cdf(x, gauss_e(x)); }
// tanh GELU: 0.5 x (1 + tanh(k (x + 0.044715 x^3))), tanh from one v_exp + one v_rcp (saturates
// correctly at +-inf) -- the same formula as ops/csrc/act.hip
__device__ __forceinline__ float tanh_fast(float y) {
  return 1.f - 2.f * __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(y * 2.8853900817779268f));   // e^{2y}
}
__device__ __forceinline__ float gelu_tanh(float x) {
  return 0.5f * x * (1.f + tanh_fast(0.7978845608028654f * fmaf(0.044715f * x, x * x, x)));
}
__device__ __forceinline__ float gelu_tanh_grad(float x) {
  const float k = 0.7978845608028654f;
  const float t = tanh_fast(k * fmaf(0.044715f * x, x * x, x));
  return 0.5f * (1.f + t) + 0.5f * x * (1.f - t * t) * k * (1.f + 3.f * 0.044715f * x * x);
}
template <int EPI> __device__ __forceinline__ float epi_act(float x);
template <int EPI> __device__ __forceinline__ float epi_act_grad(float x);
__device__ __forceinline__ float gelu_grad(float x);
template <int EPI>
__device__ __forceinline__ float epi_act(float x) {
  if constexpr (EPI == EPI_BIAS_GELU_TANH || EPI == EPI_BIAS_GELU_TANH_G) return gelu_tanh(x);
  else if constexpr (EPI == EPI_BIAS_RELU) return x > 0.f ? x : 0.f;
  else return gelu(x);
}
template <int EPI>
__device__ __forceinline__ float epi_act_grad(float x) {
  if constexpr (EPI == EPI_GELU_TANH_BWD) return gelu_tanh_grad(x);
  else if constexpr (EPI == EPI_RELU_BWD) return x > 0.f ? 1.f : 0.f;
  else if constexpr (EPI == EPI_MUL_BWD) return x;   // the input already is the derivative
  else return gelu_grad(x);
}
// act(x) and act'(x) sharing the transcendental terms (EPI_BIAS_GELU_G / _TANH_G)
template <int EPI>
__device__ __forceinline__ void epi_act_and_grad(float x, float& a, float& d) {
  if constexpr (EPI == EPI_BIAS_GELU_TANH_G) {
    const float k = 0.7978845608028654f;
    const float t = tanh_fast(k * fmaf(0.044715f * x, x * x, x));
    const float h = 0.5f * (1.f + t);
    a = x * h;
    d = h + 0.5f * x * (1.f - t * t) * k * (1.f + 3.f * 0.044715f * x * x);
  } else {
    const float e = gauss_e(x);
    const float cdf = phi_cdf(x, e);
    a = x * cdf;
    d = fmaf(x * 0.3989422804014327f, e, cdf);
  }
}
__device__ __forceinline__ float gelu_grad(float x) {
  const float e = gauss_e(x);
  return fmaf(x * 0.3989422804014327f, e, phi_cdf(x, e));
}

// fp32 x 4 -> bf16 x 4 as two v_cvt_pk_bf16_f32 (element-wise casts of a vector make hipcc convert
// one element per instruction and re-pack with v_perm / v_alignbit)
__device__ __forceinline__ bf16x4 cvt4(f32x4 v) {
  typedef float f32x2_t __attribute__((ext_vector_type(2)));
  const bf16x2 lo = __builtin_convertvector(f32x2_t{v[0], v[1]}, bf16x2);
  const bf16x2 hi = __builtin_convertvector(f32x2_t{v[2], v[3]}, bf16x2);
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3);
}

// act(x) and act'(x) of 8 values stage by stage (each stage's 8 independent operations next to
// each other, so the dependent chain of one value never stalls on an instruction-latency hazard);
// the same arithmetic, operation for operation, as epi_act_and_grad
template <int EPI>
__device__ __forceinline__ void act_and_grad8(const bf16x8& v, float (&a)[8], float (&d)[8]) {
  float x[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) x[j] = (float)v[j];
  if constexpr (EPI == EPI_BIAS_GELU_TANH_G) {
#pragma unroll
    for (int j = 0; j < 8; ++j) epi_act_and_grad<EPI>(x[j], a[j], d[j]);
  } else {
    float e[8], t[8], p[8], c[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) e[j] = gauss_e(x[j]);
#pragma unroll
    for (int j = 0; j < 8; ++j) t[j] = __builtin_amdgcn_rcpf(fmaf(fabsf(x[j]), 0.3275911f * 0.70710678118654752f, 1.f));
#pragma unroll
    for (int j = 0; j < 8; ++j) p[j] = fmaf(t[j], 1.061405429f, -1.453152027f);
#pragma unroll
    for (int j = 0; j < 8; ++j) p[j] = fmaf(t[j], p[j], 1.421413741f);
#pragma unroll
    for (int j = 0; j < 8; ++j) p[j] = fmaf(t[j], p[j], -0.284496736f);
#pragma unroll
    for (int j = 0; j < 8; ++j) p[j] = t[j] * fmaf(t[j], p[j], 0.254829592f);
#pragma unroll
    for (int j = 0; j < 8; ++j) c[j] = 0.5f + 0.5f * copysignf(1.f - p[j] * e[j], x[j]);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      a[j] = x[j] * c[j];
      d[j] = fmaf(x[j] * 0.3989422804014327f, e[j], c[j]);
    }
  }
}
__device__ __forceinline__ bf16x8 cvt8(const float (&f)[8]) {
  const bf16x4 lo = cvt4(f32x4{f[0], f[1], f[2], f[3]}), hi = cvt4(f32x4{f[4], f[5], f[6], f[7]});
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}

// bijective XCD remap of the linear workgroup id (dispatch deals ids round-robin over 8 XCDs):
// each XCD gets a contiguous range of tiles, so tiles sharing an A panel share an L2
__device__ __forceinline__ int xcd_remap(int id, int n) {
  const int q = n / 8, r = n % 8, x = id % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + id / 8;
}

// buffer resource for a wave-uniform base pointer (readfirstlane makes the uniformity provable,
// so hipcc emits plain buffer ops instead of waterfall loops: cdna_hip_programming.md T20)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t uniform_rsrc(const void* p) {
  const uint64_t a = (uint64_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), (short)0, 0x7fffffff, 0x00020000);
}

// Per-lane byte offsets of this wave's 8 LDS-DMA rows within a tile's A / B panel (fixed for the
// whole kernel): DMA i of half-tile H fills 8 rows starting at r0, lane L -> row r0 + L/8, chunk
// slot L%8 <- global chunk (L%8) ^ (L/8)  (r0 is a multiple of 8, so (row & 7) == L/8).
// H = 0: A rows {0-63, 128-191}, 1: B rows {64j + 0..31}, 2: B rows {64j + 32..63},
// 3: A rows {64-127, 192-255}.
struct StageOffs {
  int a[2][2], b[2][2];   // [lo/hi half][dma]
  int la[2][2], lb[2][2]; // LDS byte offsets of the 8-row groups
};

__device__ __forceinline__ StageOffs stage_offsets(int w, int lane, int lda, int ldb) {
  StageOffs o;
  const int dr = lane >> 3;
  const int sc = ((lane & 7) ^ dr) * 8;
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int j = w * 2 + i;   // 8-row group 0..15 of the half-tile
      const int ra = (j >> 3) * 128 + (h ? 64 : 0) + 8 * (j & 7);
      const int rb = (j >> 2) * 64 + (h ? 32 : 0) + 8 * (j & 3);
      o.a[h][i] = ((ra + dr) * lda + sc) * 2;
      o.b[h][i] = ((rb + dr) * ldb + sc) * 2;
      o.la[h][i] = ra * 128;
      o.lb[h][i] = A_BYTES + rb * 128;
    }
  return o;
}

// One half-tile (16 KiB = 128 rows x 128 B) of K-step kt into LDS buffer `buf` by
// buffer_load_dwordx4 ... lds (32-bit lane offsets, the K-step as the scalar offset)
template <int H>
__device__ __forceinline__ void stage(const StageOffs& o, __amdgpu_buffer_rsrc_t ra, __amdgpu_buffer_rsrc_t rb,
                                      char* buf, int kt) {
#if DTD_GEMM_DIAG & 16   // diagnostic build: every K-step re-stages K-step 0 (L2-hot source)
  const int so = 0 * kt;
#else
  const int so = kt * BK * 2;
#endif
#if DTD_GEMM_DIAG & 32   // diagnostic build: only the A half-tiles are staged
  if constexpr (H == 1 || H == 2) return;
#endif
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    if constexpr (H == 0 || H == 3) {
      constexpr int h = H == 3 ? 1 : 0;
      dma16(ra, buf + o.la[h][i], o.a[h][i], so);
    } else {
      constexpr int h = H == 2 ? 1 : 0;
      dma16(rb, buf + o.lb[h][i], o.b[h][i], so);
    }
  }
}

template <int EPI>
__global__ void __launch_bounds__(512, 2) gemm_bt_kernel(GemmArgs g) {
  __shared__ __attribute__((aligned(1024))) char smem[LDS_BYTES];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int li = lane & 15, lq = lane >> 4, sw = li & 7;
  const int wm = w >> 2, wn = w & 3;
  const int ntn = g.N / BN, ntiles = (g.M / BM) * ntn;
  const int t = xcd_remap(blockIdx.x, ntiles);
  const int bm = t / ntn, bn = t % ntn;   // N-minor: consecutive tiles share the A panel
  const int m0 = bm * BM, n0 = bn * BN;
  const int nk = g.K / BK;

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  STAMP_ID(0);
  STAMP(0, 0);

  // prologue: K-step 0 complete in buffer 0
  const StageOffs so = stage_offsets(w, lane, g.lda, g.ldb);
  const auto rsa = uniform_rsrc(g.a + (size_t)m0 * g.lda), rsb = uniform_rsrc(g.b + (size_t)n0 * g.ldb);
  stage<0>(so, rsa, rsb, smem, 0);
  stage<1>(so, rsa, rsb, smem, 0);
  stage<2>(so, rsa, rsb, smem, 0);
  stage<3>(so, rsa, rsb, smem, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  STAMP(1, 0);
  if (__builtin_amdgcn_readfirstlane(wm) == 1) bar();   // stagger wave row 1

  // fragment byte offsets within a buffer (row r, chunk c) -> r*128 + ((c ^ (r&7)) * 16)
  const int arow = (wm * 128 + li) * 128;            // + mi*16 rows
  const int brow = A_BYTES + (wn * 64 + li) * 128;   // + ni*16 rows
  const int ch0 = ((0 * 4 + lq) ^ sw) * 16, ch1 = ((1 * 4 + lq) ^ sw) * 16;

  bf16x8 af[4][2], b0[2][2], b1[2][2];

  for (int kt = 0; kt < nk; ++kt) {
    const char* cur = smem + (kt & 1) * TILE_BYTES;
    char* nxt = smem + ((kt & 1) ^ 1) * TILE_BYTES;
    const bool more = kt + 1 < nk;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      // ---- this phase's LDS fragments (quadrant order (0,0) (0,1) (1,1) (1,0))
      if (p == 0 || p == 2) {
        const int qm = p == 0 ? 0 : 1;
#pragma unroll
        for (int mi = 0; mi < 4; ++mi) {
          const char* r = cur + arow + (qm * 4 + mi) * 16 * 128;
          af[mi][0] = *reinterpret_cast<const bf16x8*>(r + ch0);
          af[mi][1] = *reinterpret_cast<const bf16x8*>(r + ch1);
        }
      }
      if (p == 0 || p == 1) {
#pragma unroll
        for (int ni = 0; ni < 2; ++ni) {
          const char* r = cur + brow + (p * 2 + ni) * 16 * 128;
          bf16x8 x0 = *reinterpret_cast<const bf16x8*>(r + ch0);
          bf16x8 x1 = *reinterpret_cast<const bf16x8*>(r + ch1);
          if (p == 0) { b0[ni][0] = x0; b0[ni][1] = x1; } else { b1[ni][0] = x0; b1[ni][1] = x1; }
        }
      }
      // ---- stage quarter p of the next K-step; retire the DMA of two phases ago
      if (more) {
        if (p == 0) stage<0>(so, rsa, rsb, nxt, kt + 1);
        if (p == 1) stage<1>(so, rsa, rsb, nxt, kt + 1);
        if (p == 2) stage<2>(so, rsa, rsb, nxt, kt + 1);
        if (p == 3) stage<3>(so, rsa, rsb, nxt, kt + 1);
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
      } else if (p == 0) {
        asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      bar();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
      const int qm = (p == 2 || p == 3) ? 1 : 0;
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
#pragma unroll
          for (int ks = 0; ks < 2; ++ks) {
            const bf16x8 bb = (p == 1 || p == 2) ? b1[ni][ks] : b0[ni][ks];
            const int nn = ((p == 1 || p == 2) ? 2 : 0) + ni;
            acc[qm * 4 + mi][nn] = mfma16(bb, af[mi][ks], acc[qm * 4 + mi][nn]);
          }
      __builtin_amdgcn_s_setprio(0);
      bar();
    }
  }
  if (__builtin_amdgcn_readfirstlane(wm) == 0) bar();   // close the stagger
  __syncthreads();
  STAMP(2, 0);

  // ---- epilogue 1 (accumulator layout): lane holds C[m][n .. n+3], m = wm*128 + mi*16 + li,
  //      n = wn*64 + ni*16 + 4*lq (tile-local).  fp32 bias / residual, one bf16 rounding, -> LDS.
  char* img = smem;   // [256][512 B] bf16, 8-byte slot s of row r at slot s ^ (r & 15)
#pragma unroll
  for (int ni = 0; ni < 4; ++ni) {
    const int n = wn * 64 + ni * 16 + 4 * lq;
    float bv[4] = {0.f, 0.f, 0.f, 0.f};
    if constexpr (EPI == EPI_STORE || is_gelu_fwd(EPI)) {
      if (g.bias) {
        const bf16x4 b4 = *reinterpret_cast<const bf16x4*>(g.bias + n0 + n);
#pragma unroll
        for (int r = 0; r < 4; ++r) bv[r] = (float)b4[r];
      }
    }
#pragma unroll
    for (int mi = 0; mi < 8; ++mi) {
      const int m = wm * 128 + mi * 16 + li;
      float v[4];
      if constexpr (EPI == EPI_ADD) {
        const bf16x4 c4 = *reinterpret_cast<const bf16x4*>(g.c + (size_t)(m0 + m) * g.ldc + n0 + n);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = acc[mi][ni][r] + (float)c4[r];
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = acc[mi][ni][r] + bv[r];
      }
      bf16x4 o;
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] = (bf16)v[r];
      *reinterpret_cast<bf16x4*>(img + m * 512 + (((n >> 2) ^ (m & 15)) << 3)) = o;
    }
  }
  __syncthreads();
  STAMP(3, 0);

  // ---- epilogue 2 (row layout): wave w stores rows w*32 .. w*32+31, two rows per instruction,
  //      lane -> row r = w*32 + 2i + (lane >> 5), 16-byte chunk c = lane & 31 (8 columns)
  const int c = lane & 31;
  float colsum[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) colsum[j] = 0.f;
#pragma unroll 4
  for (int i = 0; i < 16; ++i) {
    const int r = w * 32 + 2 * i + (lane >> 5);
    const int x = r & 15;
    bf16x8 v = *reinterpret_cast<const bf16x8*>(img + r * 512 + ((c ^ (x >> 1)) << 4));
    if (x & 1) v = __builtin_shufflevector(v, v, 4, 5, 6, 7, 0, 1, 2, 3);   // halves stored swapped
    const size_t off = (size_t)(m0 + r) * g.ldc + n0 + c * 8;
    if constexpr (EPI == EPI_STORE || EPI == EPI_ADD) {
      *reinterpret_cast<bf16x8*>(g.c + off) = v;
    } else if constexpr (stores_grad(EPI)) {
      float a[8], d[8];
      act_and_grad8<EPI>(v, a, d);
      *reinterpret_cast<bf16x8*>(g.c + off) = cvt8(d);
      *reinterpret_cast<bf16x8*>(g.c2 + off) = cvt8(a);
    } else if constexpr (is_gelu_fwd(EPI)) {
      bf16x8 a;
#pragma unroll
      for (int j = 0; j < 8; ++j) a[j] = (bf16)epi_act<EPI>((float)v[j]);   // GELU of the stored (bf16) U
      *reinterpret_cast<bf16x8*>(g.c + off) = v;
      *reinterpret_cast<bf16x8*>(g.c2 + off) = a;
    } else {   // EPI_GELU_BWD: v = bf16(dA)
      const bf16x8 u8 = *reinterpret_cast<const bf16x8*>(g.u + (size_t)(m0 + r) * g.ldu + n0 + c * 8);
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float du = (float)v[j] * epi_act_grad<EPI>((float)u8[j]);
        o[j] = (bf16)du;
        colsum[j] += du;
      }
      *reinterpret_cast<bf16x8*>(g.c + off) = o;
    }
  }
  STAMP(4, 0);
#ifdef DTD_GEMM_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  STAMP(5, 0);
#endif
  if constexpr (is_gelu_bwd(EPI)) {
    if (!g.part) return;
    // lanes c and c+32 hold the same columns; then the 8 waves combine through LDS
#pragma unroll
    for (int j = 0; j < 8; ++j) colsum[j] += __shfl_xor(colsum[j], 32, 64);
    __syncthreads();   // the image is fully consumed
    float* red = reinterpret_cast<float*>(smem);   // [8 waves][256 columns]
    if (lane < 32) {
      *reinterpret_cast<f32x4*>(red + w * 256 + c * 8) = f32x4{colsum[0], colsum[1], colsum[2], colsum[3]};
      *reinterpret_cast<f32x4*>(red + w * 256 + c * 8 + 4) = f32x4{colsum[4], colsum[5], colsum[6], colsum[7]};
    }
    __syncthreads();
    if (tid < 256) {
      float s = 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) s += red[k * 256 + tid];
      g.part[(size_t)bm * g.N + n0 + tid] = s;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Persistent form: one 512-thread workgroup per CU walks its tiles (XCD group x = blockIdx % 8
// owns a contiguous tile range, its 32 workgroups take every 32nd tile of it, so the tiles in
// flight on one XCD share A panels).  The K-step stream never drains between tiles: the last
// K-step of a tile stages K-step 0 of the workgroup's NEXT tile into the other LDS buffer, so the
// epilogue (two rounds through the free buffer, the stores as full row segments) runs while that
// DMA lands, and there is no prologue or workgroup dispatch between tiles.  The first two phases
// of a tile wait with vmcnt(4 + S) (S = the epilogue's vector-memory count): the DMA they retire
// is older than the epilogue's stores, which may stay in flight.  (An epilogue storing straight
// from the accumulators, 8-byte pieces, measured slower: scripts/gemm_stamps.py.)
// vector-memory instructions every wave issues in one epilogue (loads + stores): the lower
// bound of what sits between a K-step-0 DMA and the next tile's first waits
constexpr int kStores(int epi) {
  return is_gelu_fwd(epi) ? 32 : is_gelu_bwd(epi) ? 32 : epi == EPI_ADD ? 48 : 16;
}

__device__ __forceinline__ void tile_of(int t, int ntn, int& m0, int& n0) {
  m0 = (t / ntn) * BM;
  n0 = (t % ntn) * BN;
}

// end of a workgroup's claims: the last one to finish zeroes the queue (every claim of this
// launch has returned by then: each workgroup's final claim precedes its finish count)
__device__ __forceinline__ void sched_finish(int* q, int nwg, int tid) {
  if (q == nullptr || tid != 0) return;
  if (atomicAdd(&q[SCHED_DONE], 1) == nwg - 1) {
#pragma unroll
    for (int i = 0; i <= SCHED_DONE; ++i) atomicExch(&q[i], 0);
  }
}

template <int EPI, bool DYN>
__global__ void __launch_bounds__(512, 2) gemm_bt_persistent(GemmArgs g) {
  __shared__ __attribute__((aligned(1024))) char smem[LDS_BYTES];
  // the wave index through readfirstlane: provably uniform, so the LDS-DMA destinations (M0) are
  // formed with scalar adds instead of a v_readfirstlane per DMA (-11 % VALU; +2-3 % vs hipBLASLt
  // on the BERT projection shapes, profiles/r3_gemm_u2_experiment.jsonl)
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 15, lq = lane >> 4, sw = li & 7;
  const int wm = w >> 2, wn = w & 3;
  const int ntn = g.N / BN, ntiles = (g.M / BM) * ntn;
  const int nk = g.K / BK;
  // tile sequence of this workgroup: XCD group x gets tiles [beg, end), member l takes beg + l + 32 i
  const int nwg = gridDim.x, x = blockIdx.x % 8, l = blockIdx.x / 8, per = nwg / 8;
  const int q = ntiles / 8, r = ntiles % 8;
  const int beg = x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q;
  const int end = beg + q + (x < r ? 1 : 0);
  constexpr bool dyn = DYN;   // g.sched != null (a separate instantiation keeps SGPR pressure)
  // dynamic queue: a workgroup's first two tiles are the static order's (no claims at launch,
  // where 256 workgroups would contend for 8 counters); queue entry c is tile beg + 2 per + c.
  // Iteration j >= 1 reads the tile of iteration j + 1 from qslot[j & 1].
  __shared__ int qslot[2];
  int t = beg + l;
  if (t >= end) {   // more workgroups than tiles in this group (small problems) / queue drained
    if constexpr (DYN) sched_finish(g.sched, nwg, tid);
    return;
  }
  // Start stagger (DTD_GEMM_STAGGER_US, experiment): the odd members of each XCD group start
  // later, so the CUs' epilogue store bursts (128 KiB a tile) fall under other CUs' main loops
  // instead of all CUs writing at once with their MFMA pipes idle.  Bounded wait on the real-time
  // counter; the dynamic queue re-balances the tiles.
  if (g.stagger > 0 && (l & 1)) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < (unsigned long long)g.stagger) __builtin_amdgcn_s_sleep(8);
  }
  int m0, n0;
  tile_of(t, ntn, m0, n0);
  const StageOffs so = stage_offsets(w, lane, g.lda, g.ldb);
  auto rsa = uniform_rsrc(g.a + (size_t)m0 * g.lda), rsb = uniform_rsrc(g.b + (size_t)n0 * g.ldb);
  stage<0>(so, rsa, rsb, smem, 0);
  stage<1>(so, rsa, rsb, smem, 0);
  stage<2>(so, rsa, rsb, smem, 0);
  stage<3>(so, rsa, rsb, smem, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (!kOneBar && __builtin_amdgcn_readfirstlane(wm) == 1) bar();   // stagger wave row 1

  const int arow = (wm * 128 + li) * 128;
  const int brow = A_BYTES + (wn * 64 + li) * 128;
  const int ch0 = ((0 * 4 + lq) ^ sw) * 16, ch1 = ((1 * 4 + lq) ^ sw) * 16;
  constexpr int S = kStores(EPI);
  constexpr int WAIT_FIRST = 4 + S > 63 ? 63 : 4 + S;

  bf16x8 af[4][2], b0[2][2], b1[2][2];
  f32x4 acc[8][4];
  int buf = 0;
  int it = 0;
  STAMP_ID(0);
  while (true) {
    STAMP(0, it);
    const int tn = dyn && it > 0 ? __builtin_amdgcn_readfirstlane(qslot[it & 1]) : t + per;
    const bool has_next = tn < end;
    int m1 = 0, n1 = 0;
    if (has_next) tile_of(tn, ntn, m1, n1);
    const auto rsa1 = uniform_rsrc(g.a + (size_t)m1 * g.lda), rsb1 = uniform_rsrc(g.b + (size_t)n1 * g.ldb);
    // K-step 0 is peeled: its first MFMA per accumulator takes an inline-zero C operand, so the
    // 128 accumulators need no v_mov zeroing per tile (the MFMA pipe idles during that block)
    auto kstep = [&](auto first_c, int kt) {
      constexpr bool first = decltype(first_c)::value;
      const char* cur = smem + buf * TILE_BYTES;
      char* nxt = smem + (buf ^ 1) * TILE_BYTES;
      buf ^= 1;
      // what the phases of this K-step stage: the next K-step of this tile, else K-step 0 of the
      // next tile, else nothing (the very last K-step)
      const bool more_here = kt + 1 < nk;
      const bool more = more_here || has_next;
      const auto sra = more_here ? rsa : rsa1, srb = more_here ? rsb : rsb1;
      const int skt = more_here ? kt + 1 : 0;
#pragma unroll
      for (int p = 0; p < 4; ++p) {
#if DTD_GEMM_DIAG & 2   // diagnostic build: fragments read in the first K-step only
        if (first)
#endif
        if (p == 0 || p == 2) {
          const int qm = p == 0 ? 0 : 1;
#pragma unroll
          for (int mi = 0; mi < 4; ++mi) {
            const char* rr = cur + arow + (qm * 4 + mi) * 16 * 128;
            af[mi][0] = *reinterpret_cast<const bf16x8*>(rr + ch0);
            af[mi][1] = *reinterpret_cast<const bf16x8*>(rr + ch1);
          }
        }
#if DTD_GEMM_DIAG & 2
        if (first)
#endif
        if (p == 0 || p == 1) {
#pragma unroll
          for (int ni = 0; ni < 2; ++ni) {
            const char* rr = cur + brow + (p * 2 + ni) * 16 * 128;
            bf16x8 x0 = *reinterpret_cast<const bf16x8*>(rr + ch0);
            bf16x8 x1 = *reinterpret_cast<const bf16x8*>(rr + ch1);
            if (p == 0) { b0[ni][0] = x0; b0[ni][1] = x1; } else { b1[ni][0] = x0; b1[ni][1] = x1; }
          }
        }
        if (more) {
#if DTD_GEMM_DIAG & 1   // diagnostic build (timing only, wrong results): no main-loop LDS-DMA
          if (first) {
#endif
          if (p == 0) stage<0>(so, sra, srb, nxt, skt);
          if (p == 1) stage<1>(so, sra, srb, nxt, skt);
          if (p == 2) stage<2>(so, sra, srb, nxt, skt);
          if (p == 3) stage<3>(so, sra, srb, nxt, skt);
#if DTD_GEMM_DIAG & 1
          }
#endif
#if !(DTD_GEMM_DIAG & 8)   // diagnostic build: LDS-DMA issued but never waited for in the loop
          if (first && p < 2) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(WAIT_FIRST) : "memory");
          else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
#endif
        } else if (p == 0) {
          if (first) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(WAIT_FIRST - 2) : "memory");
          else asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
        } else {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
#if !(DTD_GEMM_DIAG & 4)   // diagnostic build: no barriers in the main loop
        bar();
#endif
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(1);
        const int qm = (p == 2 || p == 3) ? 1 : 0;
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
#pragma unroll
          for (int ni = 0; ni < 2; ++ni)
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) {
              const bf16x8 bb = (p == 1 || p == 2) ? b1[ni][ks] : b0[ni][ks];
              const int nn = ((p == 1 || p == 2) ? 2 : 0) + ni;
              acc[qm * 4 + mi][nn] =
                  mfma16(bb, af[mi][ks], (first && ks == 0) ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[qm * 4 + mi][nn]);
            }
        __builtin_amdgcn_s_setprio(0);
#if !(DTD_GEMM_DIAG & 4) && !DTD_GEMM_ONEBAR
        bar();
#endif
      }
    };
    kstep(std::true_type{}, 0);
    for (int kt = 1; kt < nk; ++kt) kstep(std::false_type{}, kt);

    STAMP(2, it);
    // ---- epilogue through the free LDS buffer (the last K-step's; the other one holds the
    //      next tile's K-step 0), in two rounds of 128 rows: the wave row r writes its
    //      accumulators (fp32 bias / residual, one bf16 rounding) as a [128][512 B] image
    //      (8-byte slots XOR-swizzled by row & 15), then all 8 waves store 16 rows each as
    //      512-byte row segments of 16-byte vectors.
    // accumulators -> packed bf16 first (fp32 bias / residual, one rounding): halves the live
    // registers for the rest of the epilogue
    bf16x4 pk[8][4];
    if constexpr (EPI == EPI_ADD) {
      const auto rs = uniform_rsrc(g.c + (size_t)(m0 + wm * 128) * g.ldc + n0 + wn * 64);
      const int voff = (li * g.ldc + 4 * lq) * 2;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        bf16x4 cin[4][4];
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
#pragma unroll
          for (int ni = 0; ni < 4; ++ni)
            cin[mi][ni] = __builtin_bit_cast(bf16x4, __builtin_amdgcn_raw_buffer_load_b64(
                                                         rs, voff + ni * 32, (h * 4 + mi) * 16 * g.ldc * 2, 0));
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
#pragma unroll
          for (int ni = 0; ni < 4; ++ni)
            pk[h * 4 + mi][ni] = cvt4(acc[h * 4 + mi][ni] + __builtin_convertvector(cin[mi][ni], f32x4));
      }
    } else {
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        float bv[4] = {0.f, 0.f, 0.f, 0.f};
        if constexpr (EPI == EPI_STORE || is_gelu_fwd(EPI)) {
          if (g.bias) {
            const bf16x4 b4 = *reinterpret_cast<const bf16x4*>(g.bias + n0 + wn * 64 + ni * 16 + 4 * lq);
#pragma unroll
            for (int k = 0; k < 4; ++k) bv[k] = (float)b4[k];
          }
        }
        const f32x4 bv4{bv[0], bv[1], bv[2], bv[3]};
#pragma unroll
        for (int mi = 0; mi < 8; ++mi) pk[mi][ni] = cvt4(acc[mi][ni] + bv4);
      }
    }
    if (!kOneBar && __builtin_amdgcn_readfirstlane(wm) == 0) bar();   // close the stagger
    bar();                                                // every wave is done with `img`
    char* img = smem + (buf ^ 1) * TILE_BYTES;            // = the last K-step's buffer
    const int c = lane & 31;
    // row-phase inputs first (GELU_BWD: U), so no later load wait holds back a store
    bf16x8 uin[2][8];
    if constexpr (is_gelu_bwd(EPI)) {
      const auto rs = uniform_rsrc(g.u + (size_t)m0 * g.ldu + n0);
      const int voff = ((w * 16 + (lane >> 5)) * g.ldu + c * 8) * 2;
#pragma unroll
      for (int rr = 0; rr < 2; ++rr)
#pragma unroll
        for (int i = 0; i < 8; ++i)
          uin[rr][i] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(
                                                      rs, voff, (rr * 128 + 2 * i) * g.ldu * 2, 0));
    }
    float colsum[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) colsum[j] = 0.f;
    int claim = 0;
#pragma unroll
    for (int rr = 0; rr < 2; ++rr) {
      // dynamic queue: claim the tile after the next one when the second round starts (every load
      // of the epilogue is older, so no counted wait for them waits for the atomic as well);
      // publish it when the round ends
      if (dyn && rr == 1 && has_next && tid == 0) claim = atomicAdd(&g.sched[x], 1);
      if (__builtin_amdgcn_readfirstlane(wm) == rr) {
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) {
          const int n = wn * 64 + ni * 16 + 4 * lq;
#pragma unroll
          for (int mi = 0; mi < 8; ++mi) {
            const int m = mi * 16 + li;   // row within the round's 128
            *reinterpret_cast<bf16x4*>(img + m * 512 + (((n >> 2) ^ ((m & 15) << 1)) << 3)) = pk[mi][ni];
          }
        }
      }
      bar();
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int r = w * 16 + 2 * i + (lane >> 5);   // row within the round
        const bf16x8 v = *reinterpret_cast<const bf16x8*>(img + r * 512 + ((c ^ (r & 15)) << 4));
        const size_t off = (size_t)(m0 + rr * 128 + r) * g.ldc + n0 + c * 8;
        if constexpr (EPI == EPI_STORE || EPI == EPI_ADD) {
          st8(g.c + off, v, g.nt);
        } else if constexpr (stores_grad(EPI)) {
          float av[8], dv[8];
          act_and_grad8<EPI>(v, av, dv);
          st8(g.c + off, cvt8(dv), g.nt);
          st8(g.c2 + off, cvt8(av), g.nt);
        } else if constexpr (is_gelu_fwd(EPI)) {
          bf16x8 av;
#pragma unroll
          for (int j = 0; j < 8; ++j) av[j] = (bf16)epi_act<EPI>((float)v[j]);
          st8(g.c + off, v, g.nt);
          st8(g.c2 + off, av, g.nt);
        } else {
          float o[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            o[j] = (float)v[j] * epi_act_grad<EPI>((float)uin[rr][i][j]);
            colsum[j] += o[j];
          }
          st8(g.c + off, cvt8(o), g.nt);
        }
      }
      if (dyn && rr == 1 && tid == 0) qslot[(it + 1) & 1] = has_next ? beg + 2 * per + claim : end;
      bar();   // the image is consumed before it is rewritten / restaged
    }
    if constexpr (is_gelu_bwd(EPI)) {
      // lanes c and c+32 hold the same columns; the 8 waves combine through LDS: one fp32
      // partial row per 256-row tile
#pragma unroll
      for (int j = 0; j < 8; ++j) colsum[j] += __shfl_xor(colsum[j], 32, 64);
      float* red = reinterpret_cast<float*>(img);
      if (lane < 32) {
        *reinterpret_cast<f32x4*>(red + w * 256 + c * 8) = f32x4{colsum[0], colsum[1], colsum[2], colsum[3]};
        *reinterpret_cast<f32x4*>(red + w * 256 + c * 8 + 4) = f32x4{colsum[4], colsum[5], colsum[6], colsum[7]};
      }
      bar();
      if (tid < 256 && g.part) {
        float sum = 0.f;
#pragma unroll
        for (int k = 0; k < 8; ++k) sum += red[k * 256 + tid];
        g.part[(size_t)(m0 >> 8) * g.N + n0 + tid] = sum;
      }
      bar();
    }
    if (!kOneBar && has_next && __builtin_amdgcn_readfirstlane(wm) == 1) bar();   // reopen the stagger
    STAMP(4, it);
    ++it;
    if (!has_next) break;
    t = tn;
    m0 = m1;
    n0 = n1;
    rsa = rsa1;
    rsb = rsb1;
  }
  if constexpr (DYN) sched_finish(g.sched, nwg, tid);
}


// W [rows][cols] -> WT [cols][rows], bf16, 64 x 64 tiles through LDS (padded rows).  Vector form
// (rows, cols multiples of 8): 16-byte global loads and stores; otherwise element-wise.
__global__ void __launch_bounds__(256) transpose_bf16_kernel(const bf16* __restrict__ in, bf16* __restrict__ out,
                                                             int rows, int cols) {
  __shared__ bf16 tile[64][66];
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int i = ty; i < 64; i += 4) {
    const int r = r0 + i, cc = c0 + tx;
    if (r < rows && cc < cols) tile[i][tx] = in[(size_t)r * cols + cc];
  }
  __syncthreads();
  for (int i = ty; i < 64; i += 4) {
    const int cc = c0 + i, r = r0 + tx;
    if (cc < cols && r < rows) out[(size_t)cc * rows + r] = tile[tx][i];
  }
}

// one 64 x 64 tile (rows r0.., columns c0..) of the vector form
__device__ __forceinline__ void transpose_tile_vec(const bf16* __restrict__ in, bf16* __restrict__ out, int rows,
                                                   int cols, int r0, int c0) {
  __shared__ bf16 tile[64][72];
  const int t = threadIdx.x, cv = (t & 7) * 8, rv = t >> 3;   // 8 vectors per 64-wide row
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int r = rv + 32 * h;
    if (r0 + r < rows && c0 + cv < cols) {
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(in + (size_t)(r0 + r) * cols + c0 + cv);
#pragma unroll
      for (int j = 0; j < 8; ++j) tile[cv + j][r] = v[j];
    }
  }
  __syncthreads();
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int cc = rv + 32 * h;   // output row = input column
    if (c0 + cc < cols && r0 + cv < rows) {
      bf16x8 v;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = tile[cc][cv + j];
      *reinterpret_cast<bf16x8*>(out + (size_t)(c0 + cc) * rows + r0 + cv) = v;
    }
  }
}

__global__ void __launch_bounds__(256) transpose_bf16_vec_kernel(const bf16* __restrict__ in, bf16* __restrict__ out,
                                                                 int rows, int cols) {
  transpose_tile_vec(in, out, rows, cols, blockIdx.y * 64, blockIdx.x * 64);
}

// Many weights transposed in one launch (the NT input-gradient operands of a whole model at the
// start of its backward, instead of one small launch per weight per layer): workgroup b takes
// tile b - tile0[e] of entry e, tile0 the entries' running tile counts (kernel-argument arrays,
// indexed wave-uniformly).
constexpr int kMaxTranspose = 64;
struct TransposeSet {
  const bf16* in[kMaxTranspose];
  bf16* out[kMaxTranspose];
  int rows[kMaxTranspose], cols[kMaxTranspose], tile0[kMaxTranspose + 1];
  int n;
};
__global__ void __launch_bounds__(256) transpose_many_kernel(TransposeSet s) {
  const int b = blockIdx.x;
  int e = 0;
  while (e + 1 < s.n && s.tile0[e + 1] <= b) ++e;
  const int ntc = (s.cols[e] + 63) / 64, t = b - s.tile0[e];
  transpose_tile_vec(s.in[e], s.out[e], s.rows[e], s.cols[e], (t / ntc) * 64, (t % ntc) * 64);
}

}  // namespace

// Kernel form: 1 = persistent (default), 0 = one tile per workgroup with the LDS-image epilogue
// (DTD_GEMM_VARIANT; kept for same-box A/B runs).
static int g_gemm_variant = -1;
static int gemm_variant() {
  if (g_gemm_variant < 0) {
    const char* e = getenv("DTD_GEMM_VARIANT");
    g_gemm_variant = e ? atoi(e) : 1;
  }
  return g_gemm_variant;
}

// same-process A/B of the kernel forms (scripts/bench_gemm8.py); returns the previous form
DTD_EXPORT int dtd_gemm_set_variant(int v) {
  const int old = gemm_variant();
  g_gemm_variant = v;
  return old;
}

static int num_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0, c = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                 hipSuccess || c < 8)
      c = 256;
    n = c;
  }
  return n;
}

// persistent-form non-temporal epilogue stores (default; DTD_GEMM_NT_STORE=0 turns them off, read
// per call): the fused FFN kernels write two T x 3072 tensors per layer that nothing reads from
// cache -- +0.13 % step at b1024, the same in both interleaved rounds (profiles/r6_ntstore.jsonl)
static int gemm_nt_store() {
  const char* e = getenv("DTD_GEMM_NT_STORE");
  return !(e && e[0] == '0');
}

// persistent-form start stagger in 10 ns ticks (DTD_GEMM_STAGGER_US; dtd_gemm_set_stagger)
static int g_stagger = -1;
static int gemm_stagger() {
  if (g_stagger < 0) {
    const char* e = getenv("DTD_GEMM_STAGGER_US");
    g_stagger = e ? (int)(atof(e) * 100.0) : 0;
  }
  return g_stagger;
}
DTD_EXPORT int dtd_gemm_set_stagger(double us) {
  g_stagger = us > 0 ? (int)(us * 100.0) : 0;
  return 0;
}

static unsigned long long* g_stamps = nullptr;
// diagnostic builds: device buffer of [workgroups][32 tiles][8] u64 stamps (null: off)
DTD_EXPORT int dtd_gemm_set_stamps(void* p) {
  g_stamps = (unsigned long long*)p;
  return 0;
}

// Shape contract (checked): M % 256 == 0, N % 256 == 0, K % 64 == 0, leading dimensions % 8 == 0,
// 16-byte aligned base pointers (checked on the Python side).
DTD_EXPORT int dtd_gemm_bt_supported(int M, int N, int K) {
  return M > 0 && N > 0 && K > 0 && M % BM == 0 && N % BN == 0 && K % BK == 0;
}

// GELU_BWD column partials: one fp32 row per 256 rows of M
DTD_EXPORT int dtd_gemm_bt_part_rows(int M) { return M / BM; }

// sched: the stream's dynamic tile queue (9 zero-initialised ints, ops/gemm.py) or null for the
// static tile order
DTD_EXPORT int dtd_gemm_bt(int epi, const void* a, int lda, const void* b, int ldb, void* c, int ldc, void* c2,
                           const void* u, int ldu, const void* bias, float* part, int M, int N, int K,
                           int* sched, hipStream_t s) {
  if (!dtd_gemm_bt_supported(M, N, K)) return (int)hipErrorInvalidValue;
  if ((lda | ldb | ldc) % 8 || (u && ldu % 8)) return (int)hipErrorInvalidValue;
  if (lda < K || ldb < K || ldc < N) return (int)hipErrorInvalidValue;
  if (epi < EPI_STORE || epi > EPI_LAST) return (int)hipErrorInvalidValue;
  if (is_gelu_fwd(epi) && !c2) return (int)hipErrorInvalidValue;
  if (is_gelu_bwd(epi) && !u) return (int)hipErrorInvalidValue;
  GemmArgs g{(const bf16*)a, (const bf16*)b, (bf16*)c, (bf16*)c2, (const bf16*)u, (const bf16*)bias, part,
             M, N, K, lda, ldb, ldc, ldu, g_stamps, nullptr, gemm_stagger(), gemm_nt_store()};
  const int ntiles = (M / BM) * (N / BN);
  if (gemm_variant() >= 1) {
    const int cus = num_cus() / 8 * 8;
    const int nwg = ntiles >= cus ? cus : (ntiles + 7) / 8 * 8;
    g.sched = sched;
#define DTD_GEMM_P(E)                                                                       \
  if (sched) hipLaunchKernelGGL((gemm_bt_persistent<E, true>), dim3(nwg), dim3(512), 0, s, g);   \
  else hipLaunchKernelGGL((gemm_bt_persistent<E, false>), dim3(nwg), dim3(512), 0, s, g)
    switch (epi) {
      case EPI_STORE: DTD_GEMM_P(EPI_STORE); break;
      case EPI_BIAS_GELU: DTD_GEMM_P(EPI_BIAS_GELU); break;
      case EPI_GELU_BWD: DTD_GEMM_P(EPI_GELU_BWD); break;
      case EPI_ADD: DTD_GEMM_P(EPI_ADD); break;
      case EPI_BIAS_GELU_TANH: DTD_GEMM_P(EPI_BIAS_GELU_TANH); break;
      case EPI_GELU_TANH_BWD: DTD_GEMM_P(EPI_GELU_TANH_BWD); break;
      case EPI_BIAS_RELU: DTD_GEMM_P(EPI_BIAS_RELU); break;
      case EPI_RELU_BWD: DTD_GEMM_P(EPI_RELU_BWD); break;
      case EPI_BIAS_GELU_G: DTD_GEMM_P(EPI_BIAS_GELU_G); break;
      case EPI_BIAS_GELU_TANH_G: DTD_GEMM_P(EPI_BIAS_GELU_TANH_G); break;
      case EPI_MUL_BWD: DTD_GEMM_P(EPI_MUL_BWD); break;
      default: return (int)hipErrorInvalidValue;
    }
#undef DTD_GEMM_P
    DTD_LAUNCH_CHECK();
  }
  const dim3 grid(ntiles);
  switch (epi) {
    case EPI_STORE: hipLaunchKernelGGL(gemm_bt_kernel<EPI_STORE>, grid, dim3(512), 0, s, g); break;
    case EPI_BIAS_GELU: hipLaunchKernelGGL(gemm_bt_kernel<EPI_BIAS_GELU>, grid, dim3(512), 0, s, g); break;
    case EPI_GELU_BWD: hipLaunchKernelGGL(gemm_bt_kernel<EPI_GELU_BWD>, grid, dim3(512), 0, s, g); break;
    case EPI_ADD: hipLaunchKernelGGL(gemm_bt_kernel<EPI_ADD>, grid, dim3(512), 0, s, g); break;
    case EPI_BIAS_GELU_TANH: hipLaunchKernelGGL(gemm_bt_kernel<EPI_BIAS_GELU_TANH>, grid, dim3(512), 0, s, g); break;
    case EPI_GELU_TANH_BWD: hipLaunchKernelGGL(gemm_bt_kernel<EPI_GELU_TANH_BWD>, grid, dim3(512), 0, s, g); break;
    case EPI_BIAS_RELU: hipLaunchKernelGGL(gemm_bt_kernel<EPI_BIAS_RELU>, grid, dim3(512), 0, s, g); break;
    case EPI_RELU_BWD: hipLaunchKernelGGL(gemm_bt_kernel<EPI_RELU_BWD>, grid, dim3(512), 0, s, g); break;
    case EPI_BIAS_GELU_G: hipLaunchKernelGGL(gemm_bt_kernel<EPI_BIAS_GELU_G>, grid, dim3(512), 0, s, g); break;
    case EPI_BIAS_GELU_TANH_G: hipLaunchKernelGGL(gemm_bt_kernel<EPI_BIAS_GELU_TANH_G>, grid, dim3(512), 0, s, g); break;
    case EPI_MUL_BWD: hipLaunchKernelGGL(gemm_bt_kernel<EPI_MUL_BWD>, grid, dim3(512), 0, s, g); break;
    default: return (int)hipErrorInvalidValue;
  }
  DTD_LAUNCH_CHECK();
}

// Diagnostic (scripts/bench_gemm_sched.py): `nwg` workgroups that each hold a whole CU for the
// persistent GEMM's purposes (96 KiB of LDS: no 128 KiB GEMM workgroup fits beside one) and wait
// `ticks` of the 100 MHz real-time counter -- a stand-in for an RCCL kernel that occupies CUs on
// the comm stream while the compute stream launches a GEMM.  Every workgroup exits on its own
// clock; nothing is written unless the (never true) sink condition holds.
__global__ void __launch_bounds__(256) spin_occupy_kernel(unsigned long long ticks, int* sink) {
  __shared__ int hold[24576];
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  hold[threadIdx.x] = (int)threadIdx.x;
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
  __syncthreads();
  if (sink && hold[threadIdx.x ^ 1] < 0) sink[0] = 1;
}

DTD_EXPORT int dtd_spin_occupy(int nwg, double us, hipStream_t s) {
  if (nwg < 1 || nwg > 4096 || !(us >= 0.0) || us > 1e6) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(spin_occupy_kernel, dim3(nwg), dim3(256), 0, s, (unsigned long long)(us * 100.0), nullptr);
  DTD_LAUNCH_CHECK();
}


// ins[i] [rows[i]][cols[i]] -> outs[i] [cols[i]][rows[i]] for i < n in one launch (vector form only:
// rows, cols multiples of 8, 16-byte aligned pointers; n <= 64)
DTD_EXPORT int dtd_transpose_many(const void* const* ins, void* const* outs, const int* rows, const int* cols, int n,
                                  hipStream_t s) {
  if (n <= 0) return 0;
  if (n > kMaxTranspose) return (int)hipErrorInvalidValue;
  TransposeSet set{};
  int tiles = 0;
  for (int i = 0; i < n; ++i) {
    if (rows[i] <= 0 || cols[i] <= 0 || rows[i] % 8 || cols[i] % 8 || ((uintptr_t)ins[i] | (uintptr_t)outs[i]) % 16)
      return (int)hipErrorInvalidValue;
    set.in[i] = (const bf16*)ins[i];
    set.out[i] = (bf16*)outs[i];
    set.rows[i] = rows[i];
    set.cols[i] = cols[i];
    set.tile0[i] = tiles;
    tiles += ((rows[i] + 63) / 64) * ((cols[i] + 63) / 64);
  }
  set.tile0[n] = tiles;
  set.n = n;
  hipLaunchKernelGGL(transpose_many_kernel, dim3(tiles), dim3(256), 0, s, set);
  DTD_LAUNCH_CHECK();
}

DTD_EXPORT int dtd_transpose_bf16(const void* in, void* out, int rows, int cols, hipStream_t s) {
  if (rows <= 0 || cols <= 0) return (int)hipErrorInvalidValue;
  const dim3 grid((cols + 63) / 64, (rows + 63) / 64);
  if (rows % 8 == 0 && cols % 8 == 0 && ((uintptr_t)in | (uintptr_t)out) % 16 == 0)
    hipLaunchKernelGGL(transpose_bf16_vec_kernel, grid, dim3(256), 0, s, (const bf16*)in, (bf16*)out, rows, cols);
  else
    hipLaunchKernelGGL(transpose_bf16_kernel, grid, dim3(256), 0, s, (const bf16*)in, (bf16*)out, rows, cols);
  DTD_LAUNCH_CHECK();
}
