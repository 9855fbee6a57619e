// fp32 GEMM on the gfx950 f32 MFMA (v_mfma_f32_32x32x2_f32): the reference-precision path.
//
// The reference trains in fp32 (reference model/transformer.py:37-40,50-51 Linears,
// HF BertForMaskedLM).  On MI355X there is no TF32-like shortcut: the f32-input MFMA is an exact
// fp32 FMA chain at 64 FLOP/clk/SIMD, the same rate as the f32 VALU (cdna_hip_programming.md §3
// "FP32-input MFMA").  At that rate one 32x32x2 MFMA (4096 FLOP) takes 64 cycles and consumes
// 512 B of operands, so the kernel is MFMA-bound by a wide margin: LDS bandwidth, load latency and
// the epilogue are secondary, and a plain structure reaches the pipe -- 128x128 tiles, 4 waves of
// 64x64 (2x2 blocks of 32x32, 64 accumulator registers per lane), 16-deep K-steps double-buffered
// in LDS, up to 3 workgroups per CU so one workgroup's loads and barrier hide under another's MFMAs.
//
//   NT: C[M, N] = A[M, K] . B[N, K]^T (+ bias[n])   Linear forward; input gradient with B = W^T
//   TN: C[M, N] = A[K, M]^T . B[K, N]              weight gradient dW = dY^T X (K = tokens), with
//       an optional split over K into fp32 partial slices (summed by ops/csrc/reduce.hip)
//
// Fragment k order: a 16-deep K-step is 8 MFMA steps; lane half h takes k = 8h + s in step s, so an
// NT operand row is read as two float4 (rows padded to 20 floats: the 16 rows of a ds_read_b128
// lane group land on distinct 4-bank slots).  TN operands are staged as [k][m] rows (pitch 132
// floats) and read one float per step, 32 consecutive m per half-wave (conflict-free).
// C/D map: register i of lane l is row crow(i, l >> 5), column l & 31 of a 32x32 block.
#include "common.h"

using namespace dtd;

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int BM = 128, BN = 128, BK = 16;
constexpr int NT_PITCH = BK + 4;          // floats per staged row, NT layout
constexpr int TN_PITCH = BM + 4;          // floats per staged k-row, TN layout (BM == BN)
constexpr int STAGE_FLOATS = 2 * BM * NT_PITCH > 2 * BK * TN_PITCH ? 2 * BM * NT_PITCH : 2 * BK * TN_PITCH;

__device__ __forceinline__ f32x16 mfma_f32(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ int crow(int i, int h) { return (i & 3) + 8 * (i >> 2) + 4 * h; }
__device__ __forceinline__ float comp(const float4& v, int c) { return c == 0 ? v.x : c == 1 ? v.y : c == 2 ? v.z : v.w; }

struct F32GemmArgs {
  const float* a; const float* b; float* c; const float* bias;
  int M, N, K, lda, ldb, ldc;
  int ksplit;          // K-steps per split (TN split-K), grid.z = splits
  long long cstride;   // floats between split slices of C
};

// XCD-aware bijective tile order (each XCD a contiguous range of tiles, N-minor)
__device__ __forceinline__ void tile_xy(int& bm, int& bn, int ntn) {
  const int n = gridDim.x, id = blockIdx.x;
  const int q = n / 8, r = n % 8, x = id % 8;
  const int t = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + id / 8;
  bm = t / ntn;
  bn = t % ntn;
}

template <bool TN>
__global__ void __launch_bounds__(256, 3) gemm_f32_kernel(F32GemmArgs g) {
  __shared__ __attribute__((aligned(16))) float sm[2][STAGE_FLOATS];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 31, hh = lane >> 5;
  const int wm = w >> 1, wn = w & 1;
  const int ntn = g.N / BN;
  int bm, bn;
  tile_xy(bm, bn, ntn);
  const int m0 = bm * BM, n0 = bn * BN;
  const int nk_all = g.K / BK;
  const int kb = blockIdx.z * g.ksplit;
  const int nk = min(g.ksplit, nk_all - kb);
  float* cbase = g.c + (size_t)blockIdx.z * g.cstride;

  // global -> registers: 2 float4 of A and 2 of B per thread per K-step (named, not an array: a
  // runtime-indexed array lands in scratch).
  // NT: 128 rows x 16 floats per operand = 512 float4: thread t takes rows t/4 and t/4 + 64, chunk t%4
  // TN: 16 k-rows x 128 floats = 512 float4: thread t takes k-rows t/32 and t/32 + 8, chunk t%32
  float4 ra0, ra1, rb0, rb1;
  const int q_row = TN ? tid / 32 : tid / 4, q_ch = TN ? tid % 32 : tid % 4, q_step = TN ? 8 : 64;
  auto gload = [&](int kt) {
    const int k0 = (kb + kt) * BK;
    if constexpr (!TN) {
      const float* pa = g.a + (size_t)(m0 + q_row) * g.lda + k0 + 4 * q_ch;
      const float* pb = g.b + (size_t)(n0 + q_row) * g.ldb + k0 + 4 * q_ch;
      ra0 = *reinterpret_cast<const float4*>(pa);
      ra1 = *reinterpret_cast<const float4*>(pa + (size_t)q_step * g.lda);
      rb0 = *reinterpret_cast<const float4*>(pb);
      rb1 = *reinterpret_cast<const float4*>(pb + (size_t)q_step * g.ldb);
    } else {
      const float* pa = g.a + (size_t)(k0 + q_row) * g.lda + m0 + 4 * q_ch;
      const float* pb = g.b + (size_t)(k0 + q_row) * g.ldb + n0 + 4 * q_ch;
      ra0 = *reinterpret_cast<const float4*>(pa);
      ra1 = *reinterpret_cast<const float4*>(pa + (size_t)q_step * g.lda);
      rb0 = *reinterpret_cast<const float4*>(pb);
      rb1 = *reinterpret_cast<const float4*>(pb + (size_t)q_step * g.ldb);
    }
  };
  auto swrite = [&](float* s) {
    constexpr int P = TN ? TN_PITCH : NT_PITCH;
    constexpr int BOFF = TN ? BK * TN_PITCH : BM * NT_PITCH;
    float* d = s + q_row * P + 4 * q_ch;
    *reinterpret_cast<float4*>(d) = ra0;
    *reinterpret_cast<float4*>(d + q_step * P) = ra1;
    *reinterpret_cast<float4*>(d + BOFF) = rb0;
    *reinterpret_cast<float4*>(d + BOFF + q_step * P) = rb1;
  };

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};

  if (nk > 0) {
    gload(0);
    swrite(sm[0]);
    __syncthreads();
  }
  for (int kt = 0; kt < nk; ++kt) {
    const float* s = sm[kt & 1];
    if (kt + 1 < nk) gload(kt + 1);   // lands under this K-step's MFMAs
    if constexpr (!TN) {
      // A / B fragments: rows (block * 32 + r), k = 8 hh .. 8 hh + 7 as two float4
      float4 fa[2][2], fb[2][2];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          fa[i][c] = *reinterpret_cast<const float4*>(s + (wm * 64 + i * 32 + r) * NT_PITCH + 8 * hh + 4 * c);
          fb[i][c] = *reinterpret_cast<const float4*>(s + BM * NT_PITCH + (wn * 64 + i * 32 + r) * NT_PITCH + 8 * hh + 4 * c);
        }
#pragma unroll
      for (int st = 0; st < 8; ++st)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            // transposed tile (B operand first): lane column = m, register rows = n
            acc[i][j] = mfma_f32(comp(fb[j][st >> 2], st & 3), comp(fa[i][st >> 2], st & 3), acc[i][j]);
    } else {
#pragma unroll
      for (int st = 0; st < 8; ++st) {
        const int k = 8 * hh + st;
        float fa[2], fb[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          fa[i] = s[k * TN_PITCH + wm * 64 + i * 32 + r];
          fb[i] = s[BK * TN_PITCH + k * TN_PITCH + wn * 64 + i * 32 + r];
        }
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[i][j] = mfma_f32(fb[j], fa[i], acc[i][j]);
      }
    }
    if (kt + 1 < nk) {
      swrite(sm[(kt + 1) & 1]);
      __syncthreads();
    }
  }
  // lane holds C[m = m0 + wm*64 + i*32 + r][n = n0 + wn*64 + j*32 + crow(reg, hh)]; registers
  // 4g .. 4g+3 are 4 consecutive n of one row: one float4 store each (the epilogue is a rounding
  // error next to the f32-MFMA main loop)
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int m = m0 + wm * 64 + i * 32 + r;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        const int n = n0 + wn * 64 + j * 32 + 8 * gq + 4 * hh;
        float4 v = make_float4(acc[i][j][4 * gq], acc[i][j][4 * gq + 1], acc[i][j][4 * gq + 2], acc[i][j][4 * gq + 3]);
        if (!TN && g.bias) {
          const float4 bv = *reinterpret_cast<const float4*>(g.bias + n);
          v.x += bv.x; v.y += bv.y; v.z += bv.z; v.w += bv.w;
        }
        *reinterpret_cast<float4*>(cbase + (size_t)m * g.ldc + n) = v;
      }
  }
}

int f32_num_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0, cu = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cu < 8)
      cu = 256;
    n = cu;
  }
  return n;
}

}  // namespace

DTD_EXPORT int dtd_gemm_f32_supported(int M, int N, int K) {
  return M > 0 && N > 0 && K > 0 && M % BM == 0 && N % BN == 0 && K % BK == 0;
}

// NT: a [M, K] (lda), b [N, K] (ldb) -> c [M, N] (ldc) (+ bias [N])
DTD_EXPORT int dtd_gemm_f32_nt(const float* a, int lda, const float* b, int ldb, float* c, int ldc, const float* bias,
                               int M, int N, int K, hipStream_t s) {
  if (!dtd_gemm_f32_supported(M, N, K) || lda % 4 || ldb % 4 || ldc % 4 || lda < K || ldb < K || ldc < N)
    return (int)hipErrorInvalidValue;
  F32GemmArgs g{a, b, c, bias, M, N, K, lda, ldb, ldc, K / BK, 0};
  hipLaunchKernelGGL((gemm_f32_kernel<false>), dim3((M / BM) * (N / BN), 1, 1), dim3(256), 0, s, g);
  DTD_LAUNCH_CHECK();
}

// split count for a TN product: about two workgroups per CU over all splits
DTD_EXPORT int dtd_gemm_f32_tn_splits(int M, int N, int K) {
  const int tiles = (M / BM) * (N / BN), nk = K / BK;
  int sp = (2 * f32_num_cus() + tiles - 1) / tiles;
  if (sp < 1) sp = 1;
  if (sp > nk) sp = nk;
  return sp;
}

// TN: a [K, M] (lda), b [K, N] (ldb) -> part [splits][M][N] fp32 partial products over contiguous
// K ranges (splits == 1: the product itself)
DTD_EXPORT int dtd_gemm_f32_tn(const float* a, int lda, const float* b, int ldb, float* part, int M, int N, int K,
                               int splits, hipStream_t s) {
  if (!dtd_gemm_f32_supported(M, N, K) || lda % 4 || ldb % 4 || lda < M || ldb < N || splits < 1)
    return (int)hipErrorInvalidValue;
  const int nk = K / BK, ks = (nk + splits - 1) / splits;
  F32GemmArgs g{a, b, part, nullptr, M, N, K, lda, ldb, N, ks, (long long)M * N};
  hipLaunchKernelGGL((gemm_f32_kernel<true>), dim3((M / BM) * (N / BN), 1, splits), dim3(256), 0, s, g);
  DTD_LAUNCH_CHECK();
}
