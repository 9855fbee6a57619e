// MFMA GEMM with fused epilogues for the transformer FFN (gfx950).
//
//   C[M, N] = A[M, K] . B[N, K]^T        bf16 in, fp32 accumulate, both operands K-contiguous
//
// hipBLASLt runs the plain projections; this kernel exists for the products whose OUTPUT feeds an
// elementwise pass that would otherwise re-read it from HBM:
//   EPI_STORE      C (+ bias[n])                         plain / bias GEMM (tests, reference point)
//   EPI_BIAS_GELU  U = C + bias; A = gelu(U); store U, A    FFN up-projection forward (fc1 + GELU):
//                                                         the activation pass's U re-read disappears
//   EPI_GELU_BWD   dU = C * gelu'(U[m, n]); store dU;     FFN backward (fc2 dgrad + GELU'): the
//                  column partial sums of dU (fc1 bias)   da round trip through HBM disappears
//
// Structure (cdna_hip_programming.md §5): 256x256 output tile per 512-thread workgroup, 8 waves as
// 2 (M) x 4 (N), each wave 128 x 64; K-steps of 64 staged global -> LDS with 16-byte LDS-DMA
// (global_load_lds_dwordx4, no VGPR staging) into two LDS stages (2 x 64 KiB in ONE __shared__
// array); the next K-step's DMA is in flight while the current one is multiplied, ordered by a
// counted `s_waitcnt vmcnt` and raw s_barrier (no vmcnt(0) drain).  LDS rows are 128 B with the
// 16-byte chunk index XOR-swizzled by (row & 7): DMA destinations stay lane-linear (the SOURCE
// address carries the inverse swizzle, an involution) and every ds_read_b128 fragment read is
// bank-conflict free.  MFMA v_mfma_f32_16x16x32_bf16 computes the transposed tile (B fragment as
// the A operand), so each lane's accumulator holds 4 CONSECUTIVE columns of one row: epilogue
// loads/stores are 8-byte bf16x4 row segments.  XCD-aware bijective tile order.
#include "common.h"

using namespace dtd;

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;
typedef const __attribute__((address_space(1))) void gbl_void;

constexpr int BM = 256, BK = 64;

enum Epi : int { EPI_STORE = 0, EPI_BIAS_GELU = 1, EPI_GELU_BWD = 2 };

struct GemmArgs {
  const bf16* a; const bf16* b;          // A [M, K] (lda), B [N, K] (ldb)
  bf16* c; int ldc;                      // output (STORE: C, BIAS_GELU: U, GELU_BWD: dU)
  bf16* c2;                              // BIAS_GELU: A = gelu(U) (ldc)
  const bf16* u; int ldu;                // GELU_BWD: pre-activation U
  const bf16* bias;                      // [N] or null
  float* part;                           // GELU_BWD: [M/128][N] column partials of dU (or null)
  int M, N, K, lda, ldb;
};

__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// GELU(erf) and its derivative from one exponential (same formulas as act.hip)
__device__ __forceinline__ float phi_cdf(float x, float e) {
  const float a = fabsf(x) * 0.70710678118654752f;
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, a, 1.f));
  const float poly = t * fmaf(t, fmaf(t, fmaf(t, fmaf(t, 1.061405429f, -1.453152027f), 1.421413741f), -0.284496736f),
                              0.254829592f);
  return 0.5f + 0.5f * copysignf(1.f - poly * e, x);
}
__device__ __forceinline__ float gelu(float x) { return x * phi_cdf(x, __expf(-0.5f * x * x)); }
__device__ __forceinline__ float gelu_grad(float x) {
  const float e = __expf(-0.5f * x * x);
  return fmaf(x * 0.3989422804014327f, e, phi_cdf(x, e));
}

// bijective XCD remap of the linear workgroup id (dispatch deals ids round-robin over 8 XCDs)
__device__ __forceinline__ int xcd_remap(int id, int n) {
  const int q = n / 8, r = n % 8, x = id % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + id / 8;
}

// BN = 256: 8 waves as 2 (M) x 4 (N), 2 LDS stages of 64 KiB (one K-step in flight).
// BN = 128: 8 waves as 4 (M) x 2 (N), 3 LDS stages of 48 KiB (two K-steps in flight).
template <int EPI, int BN, int STAGES>
__global__ void __launch_bounds__(512, 1) gemm_bt_kernel(GemmArgs g) {
  constexpr int STAGE_BYTES = (BM + BN) * BK * 2;   // A rows then B rows, 128 B each
  constexpr int WAVES_N = BN / 64, WAVES_M = 8 / WAVES_N;
  constexpr int WM = BM / WAVES_M;                  // rows per wave (128 or 64)
  constexpr int MI = WM / 16;                       // 16-row MFMA sub-tiles per wave
  constexpr int A_DMA = BM / 64, B_DMA = BN / 64;   // 1 KiB DMA instructions per wave per K-step
  constexpr int DMA = A_DMA + B_DMA;
  __shared__ __attribute__((aligned(1024))) char smem[STAGES * STAGE_BYTES];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int li = lane & 15, lq = lane >> 4;
  const int wm = w / WAVES_N, wn = w % WAVES_N;
  const int ntn = g.N / BN, ntiles = (g.M / BM) * ntn;
  const int t = xcd_remap(blockIdx.x, ntiles);
  // M-major within an XCD's range: consecutive tiles share the B panel (the weight, L2 resident)
  const int bm = t / ntn, bn = t % ntn;
  const int m0 = bm * BM, n0 = bn * BN;
  const int nk = g.K / BK;

  // LDS-DMA of one K-step into stage s: each wave moves BM/8 rows of A and BN/8 rows of B, 8 rows
  // (1 KiB) per instruction; lane L fills row row0 + L/8, chunk slot L%8 <- global chunk
  // (L%8) ^ (row & 7).
  const int drow = lane >> 3, dpos = lane & 7;
  auto issue = [&](int kt, int s) {
    char* base = smem + s * STAGE_BYTES;
    const int k0 = kt * BK;
#pragma unroll
    for (int i = 0; i < A_DMA; ++i) {
      const int row0 = (w * A_DMA + i) * 8, r = row0 + drow;
      const bf16* src = g.a + (size_t)(m0 + r) * g.lda + k0 + ((dpos ^ (r & 7)) * 8);
      __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)(base + row0 * 128), 16, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < B_DMA; ++i) {
      const int row0 = (w * B_DMA + i) * 8, r = row0 + drow;
      const bf16* src = g.b + (size_t)(n0 + r) * g.ldb + k0 + ((dpos ^ (r & 7)) * 8);
      __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)(base + BM * 128 + row0 * 128), 16, 0, 0);
    }
  };

  f32x4 acc[MI][4];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // STAGES-1 K-steps in flight: prologue issues them, each iteration issues kt+STAGES-1 and
  // waits (counted) for kt's DMAs only
#pragma unroll
  for (int p = 0; p < STAGES - 1; ++p)
    if (p < nk) issue(p, p);
  for (int kt = 0; kt < nk; ++kt) {
    const int s = kt % STAGES;
    const int ahead = nk - 1 - kt < STAGES - 1 ? nk - 1 - kt : STAGES - 1;   // K-steps issued beyond kt
    if (kt + STAGES - 1 < nk) {
      issue(kt + STAGES - 1, (kt + STAGES - 1) % STAGES);
      if constexpr (STAGES == 2) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(DMA) : "memory");
      else asm volatile("s_waitcnt vmcnt(%0)" :: "n"(2 * DMA) : "memory");
    } else if (ahead >= 1 && STAGES == 3) {
      asm volatile("s_waitcnt vmcnt(%0)" :: "n"(DMA) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __builtin_amdgcn_s_barrier();
    const char* As = smem + s * STAGE_BYTES;
    const char* Bs = As + BM * 128;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int chunk = ks * 4 + lq;
      bf16x8 af[MI], bfr[4];
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        const int row = wn * 64 + ni * 16 + li;
        bfr[ni] = *reinterpret_cast<const bf16x8*>(Bs + row * 128 + ((chunk ^ (row & 7)) * 16));
      }
#pragma unroll
      for (int mi = 0; mi < MI; ++mi) {
        const int row = wm * WM + mi * 16 + li;
        af[mi] = *reinterpret_cast<const bf16x8*>(As + row * 128 + ((chunk ^ (row & 7)) * 16));
      }
#pragma unroll
      for (int mi = 0; mi < MI; ++mi)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = mfma16(bfr[ni], af[mi], acc[mi][ni]);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();   // stage s fully read before it is refilled
  }

  // ---- epilogue: lane holds rows m = m0 + wm*WM + mi*16 + li, columns n = n0 + wn*64 + ni*16 + 4*lq + r
  float colsum[4][4];
  if constexpr (EPI == EPI_GELU_BWD) {
#pragma unroll
    for (int ni = 0; ni < 4; ++ni)
#pragma unroll
      for (int r = 0; r < 4; ++r) colsum[ni][r] = 0.f;
  }
#pragma unroll
  for (int ni = 0; ni < 4; ++ni) {
    const int n = n0 + wn * 64 + ni * 16 + 4 * lq;
    float bv[4] = {0.f, 0.f, 0.f, 0.f};
    if (EPI != EPI_GELU_BWD && g.bias) {
      const bf16x4 b4 = *reinterpret_cast<const bf16x4*>(g.bias + n);
#pragma unroll
      for (int r = 0; r < 4; ++r) bv[r] = (float)b4[r];
    }
#pragma unroll
    for (int mi = 0; mi < MI; ++mi) {
      const int m = m0 + wm * WM + mi * 16 + li;
      const size_t off = (size_t)m * g.ldc + n;
      bf16x4 o;
      if constexpr (EPI == EPI_STORE) {
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = (bf16)(acc[mi][ni][r] + bv[r]);
        *reinterpret_cast<bf16x4*>(g.c + off) = o;
      } else if constexpr (EPI == EPI_BIAS_GELU) {
        bf16x4 o2;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const bf16 uq = (bf16)(acc[mi][ni][r] + bv[r]);   // GELU of the STORED (bf16) U, as the
          o[r] = uq;                                        // unfused path computes it
          o2[r] = (bf16)gelu((float)uq);
        }
        *reinterpret_cast<bf16x4*>(g.c + off) = o;
        *reinterpret_cast<bf16x4*>(g.c2 + off) = o2;
      } else {
        const bf16x4 u4 = *reinterpret_cast<const bf16x4*>(g.u + (size_t)m * g.ldu + n);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          // dA rounded to bf16 first: bit-compatible with the unfused (GEMM -> act_bwd) path
          const float da = (float)(bf16)acc[mi][ni][r];
          const float du = da * gelu_grad((float)u4[r]);
          o[r] = (bf16)du;
          colsum[ni][r] += du;
        }
        *reinterpret_cast<bf16x4*>(g.c + off) = o;
      }
    }
  }
  if constexpr (EPI == EPI_GELU_BWD) {
    if (!g.part) return;
    // sum over the 16 lanes sharing lq (16 rows each already summed over mi): xor 1,2,4,8
#pragma unroll
    for (int ni = 0; ni < 4; ++ni)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = colsum[ni][r];
        v += __shfl_xor(v, 1, 64);
        v += __shfl_xor(v, 2, 64);
        v += __shfl_xor(v, 4, 64);
        v += __shfl_xor(v, 8, 64);
        colsum[ni][r] = v;
      }
    if (li == 0) {
      float* prow = g.part + (size_t)((m0 + wm * WM) / WM) * g.N + n0 + wn * 64 + 4 * lq;
#pragma unroll
      for (int ni = 0; ni < 4; ++ni)
        *reinterpret_cast<f32x4*>(prow + ni * 16) = f32x4{colsum[ni][0], colsum[ni][1], colsum[ni][2], colsum[ni][3]};
    }
  }
}

}  // namespace

// Tile width: 256 (2 LDS stages) or 128 (3 stages, two K-steps in flight); DTD_GEMM_BN overrides.
static int gemm_bn() {
  static int bn = -1;
  if (bn < 0) {
    const char* e = getenv("DTD_GEMM_BN");
    bn = e ? atoi(e) : 128;
    if (bn != 128 && bn != 256) bn = 128;
  }
  return bn;
}

// Shape contract (checked): M % 256 == 0, N % gemm_bn() == 0, K % 64 == 0, lda/ldb/ldc/ldu % 8
// == 0, 16-byte aligned base pointers.  part: [dtd_gemm_bt_part_rows(M)][N] fp32 (GELU_BWD
// column partials, one row per wave row-block) or null.
DTD_EXPORT int dtd_gemm_bt_supported(int M, int N, int K) {
  return M > 0 && N > 0 && K > 0 && M % BM == 0 && N % gemm_bn() == 0 && K % BK == 0;
}

DTD_EXPORT int dtd_gemm_bt_part_rows(int M) { return M / (gemm_bn() == 256 ? 128 : 64); }

DTD_EXPORT int dtd_gemm_bt(int epi, const void* a, int lda, const void* b, int ldb, void* c, int ldc, void* c2,
                           const void* u, int ldu, const void* bias, float* part, int M, int N, int K,
                           hipStream_t s) {
  if (!dtd_gemm_bt_supported(M, N, K)) return (int)hipErrorInvalidValue;
  if ((lda | ldb | ldc) % 8 || (u && ldu % 8)) return (int)hipErrorInvalidValue;
  if (epi == EPI_BIAS_GELU && !c2) return (int)hipErrorInvalidValue;
  if (epi == EPI_GELU_BWD && !u) return (int)hipErrorInvalidValue;
  GemmArgs g{(const bf16*)a, (const bf16*)b, (bf16*)c, ldc, (bf16*)c2, (const bf16*)u, ldu, (const bf16*)bias, part,
             M, N, K, lda, ldb};
  const int bn = gemm_bn();
  const dim3 grid((M / BM) * (N / bn));
#define DTD_GEMM_LAUNCH(E)                                                                        \
  if (bn == 256) hipLaunchKernelGGL((gemm_bt_kernel<E, 256, 2>), grid, dim3(512), 0, s, g);     \
  else hipLaunchKernelGGL((gemm_bt_kernel<E, 128, 3>), grid, dim3(512), 0, s, g)
  switch (epi) {
    case EPI_STORE: DTD_GEMM_LAUNCH(EPI_STORE); break;
    case EPI_BIAS_GELU: DTD_GEMM_LAUNCH(EPI_BIAS_GELU); break;
    case EPI_GELU_BWD: DTD_GEMM_LAUNCH(EPI_GELU_BWD); break;
    default: return (int)hipErrorInvalidValue;
  }
#undef DTD_GEMM_LAUNCH
  DTD_LAUNCH_CHECK();
}
