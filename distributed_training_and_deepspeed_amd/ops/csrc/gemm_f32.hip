// fp32 GEMM on the gfx950 f32 MFMA (v_mfma_f32_32x32x2_f32): the reference-precision path.
//
// The reference trains in fp32 (reference model/transformer.py:37-40,50-51 Linears,
// HF BertForMaskedLM).  On MI355X there is no TF32-like shortcut: the f32-input MFMA is an exact
// fp32 FMA chain at 64 FLOP/clk/SIMD, the same rate as the f32 VALU (cdna_hip_programming.md §3
// "FP32-input MFMA").  At that rate one 32x32x2 MFMA (4096 FLOP) takes 64 cycles and consumes
// 512 B of operands, so the kernel is MFMA-bound by a wide margin: LDS bandwidth, load latency and
// the epilogue are secondary -- 128x128 tiles, 4 waves of 64x64 (2x2 blocks of 32x32, 64
// accumulator registers per lane), 32-deep K-steps double-buffered in LDS (72 KiB), 2 workgroups
// per CU so one workgroup's loads and barrier hide under the other's MFMAs.
//
//   NT: C[M, N] (+)= A[M, K] . B[N, K]^T (+ bias[n])   Linear forward
//   NN: C[M, N] (+)= A[M, K] . B[K, N]                 input gradient dY W (register form below)
//   TN: C[M, N] = A[K, M]^T . B[K, N]                weight gradient dW = dY^T X (K = tokens), with
//       an optional split over K into fp32 partial slices (summed by ops/csrc/reduce.hip)
// Two implementations: the LDS-staged workgroup kernel right below (small grids) and the
// register-direct one-wave kernel further down (the default wherever its grid fills a round).
//
// One LDS layout for both forms: each operand tile is staged as [row][k] (128 rows x 32 k, row
// pitch 36 floats), so the fragment reads are ds_read_b128 of 4 consecutive k in either form; the
// TN form transposes while writing LDS (4 scalar writes per global float4).  A 32-deep K-step is 16
// MFMA steps: lane half h takes k = 16h + s in step s, i.e. 4 float4 per fragment row (the 16 rows
// of a ds_read_b128 lane group land on distinct 4-bank slots: pitch / 4 is odd).
// Round 5 (profiles/r5_s49_f32_gemm.jsonl): the 16-deep form with 3 workgroups per CU kept the f32
// MFMA pipe 78 % (NT) / 61 % (TN) busy against hipBLASLt's 83-91 % at the same 2.4 GHz clock --
// one barrier per 2048 MFMA cycles and, in TN, 32 scalar LDS reads per K-step; 32-deep steps at 2
// workgroups per CU halve the barriers and give TN the NT read path.
// C/D map: register i of lane l is row crow(i, l >> 5), column l & 31 of a 32x32 block.
#include <algorithm>
#include <cmath>
#include <cstdlib>

#include "common.h"

using namespace dtd;

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int BM = 128, BN = 128, BK = 32;
constexpr int PITCH = BK + 4;             // floats per staged row ([row][k], both forms)
constexpr int OP_FLOATS = BM * PITCH;     // one operand tile (BM == BN)

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
  int accumulate;      // C += product (NT)
};

// XCD-aware bijective tile order (each XCD a contiguous range of tiles, N-minor)
__device__ __forceinline__ void tile_xy(int& bm, int& bn, int ntn) {
  const int n = gridDim.x, id = blockIdx.x;
  const int q = n / 8, r = n % 8, x = id % 8;
  const int t = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + id / 8;
  bm = t / ntn;
  bn = t % ntn;
}

// BNT: N-width of the workgroup tile, 128 (waves 2 x 2 of 64 x 64) or 64 (waves 2 x 2 of 64 x 32:
// twice the tiles, for shapes whose 128-wide grid leaves the last round of 2 workgroups per CU
// half empty -- N = 768 at 16k tokens is 1.5 rounds).  The TN form uses 128 only.
template <bool TN, int BNT>
__global__ void __launch_bounds__(256, 2) gemm_f32_kernel(F32GemmArgs g) {
  static_assert(BNT == 128 || (BNT == 64 && !TN), "tile width");
  constexpr int NJ = BNT / 64;            // 32-column B blocks per wave
  constexpr int NB = BNT / 32;            // B float4 loads per thread per K-step (NT)
  __shared__ __attribute__((aligned(16))) float sm[2][OP_FLOATS + BNT * PITCH];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r = lane & 31, hh = lane >> 5;
  const int wm = w >> 1, wn = w & 1;
  const int ntn = g.N / BNT;
  int bm, bn;
  tile_xy(bm, bn, ntn);
  const int m0 = bm * BM, n0 = bn * BNT;
  const int nk_all = g.K / BK;
  const int kb = blockIdx.z * g.ksplit;
  const int nk = min(g.ksplit, nk_all - kb);
  float* cbase = g.c + (size_t)blockIdx.z * g.cstride;

  // global -> registers: 4 float4 of A and 4 of B per thread per K-step (named, not an array: a
  // runtime-indexed array lands in scratch).  Each operand tile is 1024 float4.
  // NT ([row][k] in memory): thread t takes rows t/8 + 32j, k-chunk t%8 (8 lanes = one 128-B row run)
  // TN ([k][row] in memory): thread t takes k-rows t%8 + 8j, row-chunk t/8 (8 lanes = 8 k-rows of
  //   one 16-B column run; the wave covers 8 k-rows x 128 B)
  float4 ra0, ra1, ra2, ra3, rb0, rb1, rb2, rb3;
  const int q_lo = tid & 7, q_hi = tid >> 3;
  auto gload = [&](int kt) {
    const int k0 = (kb + kt) * BK;
    if constexpr (!TN) {
      const float* pa = g.a + (size_t)(m0 + q_hi) * g.lda + k0 + 4 * q_lo;
      const float* pb = g.b + (size_t)(n0 + q_hi) * g.ldb + k0 + 4 * q_lo;
      const size_t sa = (size_t)32 * g.lda, sb = (size_t)32 * g.ldb;
      ra0 = *reinterpret_cast<const float4*>(pa);
      ra1 = *reinterpret_cast<const float4*>(pa + sa);
      ra2 = *reinterpret_cast<const float4*>(pa + 2 * sa);
      ra3 = *reinterpret_cast<const float4*>(pa + 3 * sa);
      rb0 = *reinterpret_cast<const float4*>(pb);
      rb1 = *reinterpret_cast<const float4*>(pb + sb);
      if constexpr (NB > 2) {
        rb2 = *reinterpret_cast<const float4*>(pb + 2 * sb);
        rb3 = *reinterpret_cast<const float4*>(pb + 3 * sb);
      }
    } else {
      const float* pa = g.a + (size_t)(k0 + q_lo) * g.lda + m0 + 4 * q_hi;
      const float* pb = g.b + (size_t)(k0 + q_lo) * g.ldb + n0 + 4 * q_hi;
      const size_t sa = (size_t)8 * g.lda, sb = (size_t)8 * g.ldb;
      ra0 = *reinterpret_cast<const float4*>(pa);
      ra1 = *reinterpret_cast<const float4*>(pa + sa);
      ra2 = *reinterpret_cast<const float4*>(pa + 2 * sa);
      ra3 = *reinterpret_cast<const float4*>(pa + 3 * sa);
      rb0 = *reinterpret_cast<const float4*>(pb);
      rb1 = *reinterpret_cast<const float4*>(pb + sb);
      rb2 = *reinterpret_cast<const float4*>(pb + 2 * sb);
      rb3 = *reinterpret_cast<const float4*>(pb + 3 * sb);
    }
  };
  auto swrite = [&](float* s) {
    if constexpr (!TN) {
      float* d = s + q_hi * PITCH + 4 * q_lo;
      *reinterpret_cast<float4*>(d) = ra0;
      *reinterpret_cast<float4*>(d + 32 * PITCH) = ra1;
      *reinterpret_cast<float4*>(d + 64 * PITCH) = ra2;
      *reinterpret_cast<float4*>(d + 96 * PITCH) = ra3;
      d += OP_FLOATS;
      *reinterpret_cast<float4*>(d) = rb0;
      *reinterpret_cast<float4*>(d + 32 * PITCH) = rb1;
      if constexpr (NB > 2) {
        *reinterpret_cast<float4*>(d + 64 * PITCH) = rb2;
        *reinterpret_cast<float4*>(d + 96 * PITCH) = rb3;
      }
    } else {
      // element (k = q_lo + 8j, row = 4 q_hi + c) -> [row][k]; lanes of one write spread over 32
      // banks (2-way at most)
      float* d = s + 4 * q_hi * PITCH + q_lo;
      auto put = [&](float* base, const float4& v, int j) {
        base[0 * PITCH + 8 * j] = v.x;
        base[1 * PITCH + 8 * j] = v.y;
        base[2 * PITCH + 8 * j] = v.z;
        base[3 * PITCH + 8 * j] = v.w;
      };
      put(d, ra0, 0); put(d, ra1, 1); put(d, ra2, 2); put(d, ra3, 3);
      d += OP_FLOATS;
      put(d, rb0, 0); put(d, rb1, 1); put(d, rb2, 2); put(d, rb3, 3);
    }
  };

  f32x16 acc[2][NJ];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc[i][j] = f32x16{};

  if (nk > 0) {
    gload(0);
    swrite(sm[0]);
    __syncthreads();
  }
  for (int kt = 0; kt < nk; ++kt) {
    const float* s = sm[kt & 1];
    if (kt + 1 < nk) gload(kt + 1);   // lands under this K-step's MFMAs
    // two halves of 8 MFMA steps; fragments: rows (block * 32 + r), k = 16 hh + 8 half .. + 7
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      float4 fa[2][2], fb[NJ][2];
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int k = 16 * hh + 8 * half + 4 * c;
#pragma unroll
        for (int i = 0; i < 2; ++i)
          fa[i][c] = *reinterpret_cast<const float4*>(s + (wm * 64 + i * 32 + r) * PITCH + k);
#pragma unroll
        for (int j = 0; j < NJ; ++j)
          fb[j][c] = *reinterpret_cast<const float4*>(s + OP_FLOATS + (wn * 32 * NJ + j * 32 + r) * PITCH + k);
      }
#pragma unroll
      for (int st = 0; st < 8; ++st)
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < NJ; ++j)
            // transposed tile (B operand first): lane column = m, register rows = n
            acc[i][j] = mfma_f32(comp(fb[j][st >> 2], st & 3), comp(fa[i][st >> 2], st & 3), acc[i][j]);
    }
    if (kt + 1 < nk) {
      swrite(sm[(kt + 1) & 1]);
      __syncthreads();
    }
  }
  // lane holds C[m = m0 + wm*64 + i*32 + r][n = n0 + wn*32*NJ + j*32 + crow(reg, hh)]; registers
  // 4g .. 4g+3 are 4 consecutive n of one row: one float4 store each (the epilogue is a rounding
  // error next to the f32-MFMA main loop)
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int m = m0 + wm * 64 + i * 32 + r;
#pragma unroll
    for (int j = 0; j < NJ; ++j)
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        const int n = n0 + wn * 32 * NJ + j * 32 + 8 * gq + 4 * hh;
        float4 v = make_float4(acc[i][j][4 * gq], acc[i][j][4 * gq + 1], acc[i][j][4 * gq + 2], acc[i][j][4 * gq + 3]);
        if (!TN && g.bias) {
          const float4 bv = *reinterpret_cast<const float4*>(g.bias + n);
          v.x += bv.x; v.y += bv.y; v.z += bv.z; v.w += bv.w;
        }
        if (!TN && g.accumulate) {
          const float4 o = *reinterpret_cast<const float4*>(cbase + (size_t)m * g.ldc + n);
          v.x += o.x; v.y += o.y; v.z += o.z; v.w += o.w;
        }
        *reinterpret_cast<float4*>(cbase + (size_t)m * g.ldc + n) = v;
      }
  }
}

// ---------------------------------------------------------------------------------------------
// Register-direct form: one wave per workgroup, no LDS, no barrier.
//
// The LDS form above stalls on its per-K-step barrier: both co-resident workgroups of a CU start
// together and advance at the same rate, so they reach the barrier together and the MFMA pipe
// idles across both boundaries (profiles/r5_s49_f32_gemm.jsonl: 0.74-0.82 MFMA-busy vs the
// library's 0.83-0.92).  At the f32 MFMA rate (64 cycles per 32x32x2) a wave needs only
// ~16 KiB of operands per 8k MFMA cycles, so each wave can load its own fragments global->VGPR
// (L1/L2 absorb the re-reads) and run with no synchronisation at all: one wave per SIMD, a
// 128 x 32*NB wave tile (4 x NB blocks of 32x32, accumulators in AGPRs), 16-deep K-steps
// double-buffered in registers one step ahead.  MFMA step s (0..7) of a K-step takes k = 8 h + s
// in lane half h, for both operands.  Each operand is read in its own memory layout:
//   [row][k] ("blocked"): block b's lane r holds row 32 b + r; 2 float4 along k per block per step.
//   [k][row] ("interleaved"): the blocks are interleaved -- block b's lane r holds row NBLK r + b --
//     so ONE dwordx4 (dwordx3) of NBLK consecutive rows at one k feeds every block, and the 32
//     lanes of a half read 512 (384) contiguous bytes.
// Forms: NT (C = A B^T, Linear forward), NN (C = A B with B [K, N]: the input gradient dY W
// straight from the weight, no transposed copy), TN (C = A^T B, split-K weight-gradient partials).
// Output: lane (r, h), register q of block (i, j) is C[row_m(i, r)][row_n(j, crow(q, h))];
// `accumulate` adds C's old value (the residual-branch input gradient).
template <bool KMAJOR, int NBLK>
struct RegOp;
template <int NBLK>
struct RegOp<false, NBLK> {             // [row][k]
  float4 v[NBLK][2];
  __device__ __forceinline__ void load(const float* p, int ld, int row0, int k0, int r, int hh) {
#pragma unroll
    for (int b = 0; b < NBLK; ++b) {
      const float* q = p + (size_t)(row0 + 32 * b + r) * ld + k0 + 8 * hh;
      v[b][0] = *reinterpret_cast<const float4*>(q);
      v[b][1] = *reinterpret_cast<const float4*>(q + 4);
    }
  }
  __device__ __forceinline__ float get(int st, int b) const { return comp(v[b][st >> 2], st & 3); }
  __device__ __forceinline__ static int row(int b, int r) { return 32 * b + r; }
};
template <int NBLK>
struct RegOp<true, NBLK> {              // [k][row], blocks interleaved
  // one 4-float vector per step (3-block form: .xyz): the dwordx3 lands in an aligned register
  // quad that IS the operand storage -- with 3-float slots hipcc loaded into a temporary and
  // copied, waiting on the loads it had just issued (the prefetch collapsed)
  typedef float f32x4v __attribute__((ext_vector_type(4)));
  f32x4v v[8];
  __device__ __forceinline__ void load(const float* p, int ld, int row0, int k0, int r, int hh) {
#pragma unroll
    for (int st = 0; st < 8; ++st) {
      const float* q = p + (size_t)(k0 + 8 * hh + st) * ld + row0 + NBLK * r;
      if constexpr (NBLK == 4) {
        v[st] = *reinterpret_cast<const f32x4v*>(q);
      } else {
        static_assert(NBLK == 3, "block count");
        v[st].x = q[0]; v[st].y = q[1]; v[st].z = q[2];
      }
    }
  }
  __device__ __forceinline__ float get(int st, int b) const { return v[st][b]; }
  __device__ __forceinline__ static int row(int b, int r) { return NBLK * r + b; }
};

struct F32RegArgs {
  const float* a; const float* b; float* c; const float* bias;
  int M, N, K, lda, ldb, ldc;
  int ksplit;          // K-steps (16 deep, even) per split, grid.z = splits
  long long cstride;   // floats between split slices of C
  int accumulate;      // C += product
};

template <bool A_KM, bool B_KM, int NB>
__global__ void __launch_bounds__(64, 1) gemm_f32_reg_kernel(F32RegArgs g) {
  const int lane = threadIdx.x, r = lane & 31, hh = lane >> 5;
  constexpr int TNW = 32 * NB;          // wave tile width (n)
  const int ntn = g.N / TNW;
  int bm, bn;
  tile_xy(bm, bn, ntn);
  const int m0 = bm * 128, n0 = bn * TNW;
  const int nk_all = g.K / 16;
  const int kb = blockIdx.z * g.ksplit;
  const int nk = min(g.ksplit, nk_all - kb);
  float* cbase = g.c + (size_t)blockIdx.z * g.cstride;

  f32x16 acc[4][NB];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j) acc[i][j] = f32x16{};

  struct Frag { RegOp<A_KM, 4> a; RegOp<B_KM, NB> b; };
  auto load = [&](Frag& f, int kt) {
    const int k0 = (kb + kt) * 16;
    f.a.load(g.a, g.lda, m0, k0, r, hh);
    f.b.load(g.b, g.ldb, n0, k0, r, hh);
  };
  auto compute = [&](const Frag& f) {
#pragma unroll
    for (int st = 0; st < 8; ++st)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NB; ++j)
          // B operand first: lane column = m, register rows = n
          acc[i][j] = mfma_f32(f.b.get(st, j), f.a.get(st, i), acc[i][j]);
  };

  // nk is even (K % 32 == 0 and the host rounds split lengths up to even): steps run in pairs.
  // (straight-line body + sched_barrier: keeps the compiler from sinking the prefetch to its use)
  Frag f0, f1;
  if (nk > 0) load(f0, 0);
  for (int kt = 0; kt < nk; kt += 2) {
    load(f1, kt + 1);                       // one K-step ahead, lands under f0's MFMAs
    __builtin_amdgcn_sched_barrier(0);
    compute(f0);
    __builtin_amdgcn_sched_barrier(0);
    load(f0, min(kt + 2, nk - 1));          // unconditional (the last one re-reads): one basic block
    __builtin_amdgcn_sched_barrier(0);
    compute(f1);
    __builtin_amdgcn_sched_barrier(0);
  }

#pragma unroll
  for (int i = 0; i < 4; ++i) {
    float* cr = cbase + (size_t)(m0 + RegOp<A_KM, 4>::row(i, r)) * g.ldc;
    if constexpr (!B_KM) {
      // registers 4 gq .. 4 gq + 3 of block j: 4 consecutive n
#pragma unroll
      for (int j = 0; j < NB; ++j)
#pragma unroll
        for (int gq = 0; gq < 4; ++gq) {
          const int n = n0 + 32 * j + 8 * gq + 4 * hh;
          float4 v = make_float4(acc[i][j][4 * gq], acc[i][j][4 * gq + 1], acc[i][j][4 * gq + 2], acc[i][j][4 * gq + 3]);
          if (g.bias) {
            const float4 bv = *reinterpret_cast<const float4*>(g.bias + n);
            v.x += bv.x; v.y += bv.y; v.z += bv.z; v.w += bv.w;
          }
          if (g.accumulate) {
            const float4 o = *reinterpret_cast<const float4*>(cr + n);
            v.x += o.x; v.y += o.y; v.z += o.z; v.w += o.w;
          }
          *reinterpret_cast<float4*>(cr + n) = v;
        }
    } else {
      // register q of every block j is column NB * crow(q, h) + j: NB consecutive n per q
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int n = n0 + NB * crow(q, hh);
        float v[NB];
#pragma unroll
        for (int j = 0; j < NB; ++j) {
          v[j] = acc[i][j][q];
          if (g.bias) v[j] += g.bias[n + j];
          if (g.accumulate) v[j] += cr[n + j];
        }
        if constexpr (NB == 4) {
          *reinterpret_cast<float4*>(cr + n) = make_float4(v[0], v[1], v[2], v[3]);
        } else {
#pragma unroll
          for (int j = 0; j < NB; ++j) cr[n + j] = v[j];
        }
      }
    }
  }
}

// Many fp32 weights transposed in one launch (the NT input-gradient operands W^T of a whole fp32
// model at the start of its backward; ops/gemm.py::prepare_transposes): workgroup b takes 64 x 64
// tile b - tile0[e] of entry e, staged through LDS (pitch 65: the column reads are conflict-free).
constexpr int kMaxT32 = 64;
struct TransposeSet32 {
  const float* in[kMaxT32];
  float* out[kMaxT32];
  int rows[kMaxT32], cols[kMaxT32], tile0[kMaxT32 + 1];
  int n;
};
__global__ void __launch_bounds__(256) transpose_many_f32_kernel(TransposeSet32 s) {
  __shared__ float t[64][65];
  const int b = blockIdx.x;
  int e = 0;
  while (e + 1 < s.n && s.tile0[e + 1] <= b) ++e;
  const int rows = s.rows[e], cols = s.cols[e];
  const int ntc = (cols + 63) / 64, tt = b - s.tile0[e];
  const int r0 = (tt / ntc) * 64, c0 = (tt % ntc) * 64;
  const float* in = s.in[e];
  float* out = s.out[e];
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  // rows and cols are multiples of 4 (host check): float4 runs never straddle the edge
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = r0 + ty + 16 * i, c = c0 + 4 * tx;
    if (r < rows && c < cols) {
      const float4 v = *reinterpret_cast<const float4*>(in + (size_t)r * cols + c);
      t[ty + 16 * i][4 * tx] = v.x; t[ty + 16 * i][4 * tx + 1] = v.y;
      t[ty + 16 * i][4 * tx + 2] = v.z; t[ty + 16 * i][4 * tx + 3] = v.w;
    }
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int oc = c0 + ty + 16 * i, orr = r0 + 4 * tx;     // out [cols][rows]
    if (oc < cols && orr < rows) {
      const int j = ty + 16 * i;
      *reinterpret_cast<float4*>(out + (size_t)oc * rows + orr) =
          make_float4(t[4 * tx][j], t[4 * tx + 1][j], t[4 * tx + 2][j], t[4 * tx + 3][j]);
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

namespace {

// fraction of `slots` workgroup slots a grid of `wgs` workgroups keeps busy over its rounds
double slot_use(double wgs, double slots) { return wgs / (std::ceil(wgs / slots) * slots); }

// DTD_GEMM_F32_KERNEL = "reg" / "lds" forces one form (A/B runs); default: the register form
// where its grid fills >= 85 % of its last round, the LDS form otherwise (small grids)
int g_f32_pref = -1;
int f32_kernel_pref() {
  if (g_f32_pref < 0) {
    const char* e = getenv("DTD_GEMM_F32_KERNEL");
    g_f32_pref = (e && e[0] == 'l') ? 1 : (e && e[0] == 'r') ? 2 : 0;
  }
  return g_f32_pref;
}

}  // namespace

// 0: automatic, 1: LDS form, 2: register form (tests run both on every shape)
DTD_EXPORT int dtd_gemm_f32_set_kernel(int p) {
  g_f32_pref = p < 0 || p > 2 ? 0 : p;
  return 0;
}

namespace {
bool f32_tn_reg() { return f32_kernel_pref() != 1; }
}  // namespace

namespace {
// register-form launch over a 128 x 128 or 128 x 96 wave-tile grid (whichever fills the last round
// of one wave per SIMD better); false if the caller should take the LDS form instead
template <bool A_KM, bool B_KM>
bool launch_reg(const F32RegArgs& g, bool force, hipStream_t s) {
  const double slots = 4.0 * f32_num_cus();
  const int r128 = (g.M / 128) * (g.N / 128), r96 = g.N % 96 == 0 ? (g.M / 128) * (g.N / 96) : 0;
  const double u128 = slot_use(r128, slots), u96 = r96 ? slot_use(r96, slots) : 0.0;
  if (!force && std::max(u128, u96) < 0.85) return false;
  if (u96 > u128 + 0.02)
    hipLaunchKernelGGL((gemm_f32_reg_kernel<A_KM, B_KM, 3>), dim3(r96, 1, 1), dim3(64), 0, s, g);
  else
    hipLaunchKernelGGL((gemm_f32_reg_kernel<A_KM, B_KM, 4>), dim3(r128, 1, 1), dim3(64), 0, s, g);
  return true;
}
}  // namespace

// NT: a [M, K] (lda), b [N, K] (ldb) -> c [M, N] (ldc) (+ bias [N]) (+ c if accumulate)
DTD_EXPORT int dtd_gemm_f32_nt(const float* a, int lda, const float* b, int ldb, float* c, int ldc, const float* bias,
                               int M, int N, int K, int accumulate, hipStream_t s) {
  if (!dtd_gemm_f32_supported(M, N, K) || lda % 4 || ldb % 4 || ldc % 4 || lda < K || ldb < K || ldc < N)
    return (int)hipErrorInvalidValue;
  const double cus = f32_num_cus();
  const int pref = f32_kernel_pref();
  if (pref != 1 && launch_reg<false, false>(F32RegArgs{a, b, c, bias, M, N, K, lda, ldb, ldc, K / 16, 0, accumulate},
                                            pref == 2, s)) {
    DTD_LAUNCH_CHECK();
  }
  // LDS form: 128- or 64-wide tiles, 2 workgroups per CU, whichever fills the last round better
  F32GemmArgs g{a, b, c, bias, M, N, K, lda, ldb, ldc, K / BK, 0, accumulate};
  const int t128 = (M / BM) * (N / 128);
  if (slot_use(2.0 * t128, 2 * cus) > slot_use(t128, 2 * cus) + 0.02)
    hipLaunchKernelGGL((gemm_f32_kernel<false, 64>), dim3(2 * t128, 1, 1), dim3(256), 0, s, g);
  else
    hipLaunchKernelGGL((gemm_f32_kernel<false, 128>), dim3(t128, 1, 1), dim3(256), 0, s, g);
  DTD_LAUNCH_CHECK();
}

// split count for a TN product: minimises (rounds of resident workgroups) x (K-steps per split)
// plus the split-K reduce's extra HBM traffic (one M x N fp32 slice per split).  Register form:
// 128x128 wave tiles, 4 per CU, 16-deep K-steps of ~3.4 us; LDS form: 2 workgroups per CU,
// 32-deep K-steps of ~3.8 us.  The reduce streams at ~4 TB/s.

DTD_EXPORT int dtd_gemm_f32_tn_splits(int M, int N, int K) {
  const bool reg = f32_tn_reg();
  const int tiles = (M / BM) * (N / BN), nk = K / (reg ? 16 : BK);
  const double slots = (reg ? 4.0 : 2.0) * f32_num_cus();
  const double kstep_us = reg ? 3.4 : 3.8, slice_us = (double)M * N * 4 / 4e6;
  int best = 1;
  double best_t = 1e300;
  for (int sp = 1; sp <= nk && sp <= 64; ++sp) {
    int ks = (nk + sp - 1) / sp;
    if (reg) ks = (ks + 1) & ~1;
    const int sp_eff = (nk + ks - 1) / ks;
    const double t = std::ceil((double)tiles * sp_eff / slots) * ks * kstep_us + (sp_eff > 1 ? (sp_eff + 1) * slice_us : 0.0);
    if (t < best_t - 1e-9) { best_t = t; best = sp_eff; }
  }
  return best;
}

// TN: a [K, M] (lda), b [K, N] (ldb) -> part [splits][M][N] fp32 partial products over contiguous
// K ranges (splits == 1: the product itself)
DTD_EXPORT int dtd_gemm_f32_tn(const float* a, int lda, const float* b, int ldb, float* part, int M, int N, int K,
                               int splits, hipStream_t s) {
  if (!dtd_gemm_f32_supported(M, N, K) || lda % 4 || ldb % 4 || lda < M || ldb < N || splits < 1)
    return (int)hipErrorInvalidValue;
  if (f32_tn_reg()) {
    const int nk = K / 16, ks = ((nk + splits - 1) / splits + 1) & ~1;   // even split lengths
    F32RegArgs g{a, b, part, nullptr, M, N, K, lda, ldb, N, ks, (long long)M * N, 0};
    hipLaunchKernelGGL((gemm_f32_reg_kernel<true, true, 4>), dim3((M / 128) * (N / 128), 1, splits), dim3(64), 0, s, g);
    DTD_LAUNCH_CHECK();
  }
  const int nk = K / BK, ks = (nk + splits - 1) / splits;
  F32GemmArgs g{a, b, part, nullptr, M, N, K, lda, ldb, N, ks, (long long)M * N, 0};
  hipLaunchKernelGGL((gemm_f32_kernel<true, 128>), dim3((M / BM) * (N / BN), 1, splits), dim3(256), 0, s, g);
  DTD_LAUNCH_CHECK();
}

// NN: a [M, K] (lda), b [K, N] (ldb) -> c [M, N] (ldc) (+ c if accumulate): the input gradient dY W
// read straight from the weight [out, in] (register form only)
DTD_EXPORT int dtd_gemm_f32_nn(const float* a, int lda, const float* b, int ldb, float* c, int ldc, int M, int N, int K,
                               int accumulate, hipStream_t s) {
  if (!dtd_gemm_f32_supported(M, N, K) || lda % 4 || ldb % 4 || ldc % 4 || lda < K || ldb < N || ldc < N)
    return (int)hipErrorInvalidValue;
  launch_reg<false, true>(F32RegArgs{a, b, c, nullptr, M, N, K, lda, ldb, ldc, K / 16, 0, accumulate}, true, s);
  DTD_LAUNCH_CHECK();
}

// outs[i] = ins[i]^T for n <= 64 fp32 matrices [rows[i], cols[i]] (rows, cols multiples of 4)
DTD_EXPORT int dtd_transpose_many_f32(const float* const* ins, float* const* outs, const int* rows, const int* cols,
                                      int n, hipStream_t s) {
  if (n < 1 || n > kMaxT32) return (int)hipErrorInvalidValue;
  TransposeSet32 set{};
  int tiles = 0;
  for (int i = 0; i < n; ++i) {
    if (rows[i] <= 0 || cols[i] <= 0 || rows[i] % 4 || cols[i] % 4) return (int)hipErrorInvalidValue;
    set.in[i] = ins[i];
    set.out[i] = outs[i];
    set.rows[i] = rows[i];
    set.cols[i] = cols[i];
    set.tile0[i] = tiles;
    tiles += ((rows[i] + 63) / 64) * ((cols[i] + 63) / 64);
  }
  set.tile0[n] = tiles;
  set.n = n;
  hipLaunchKernelGGL(transpose_many_f32_kernel, dim3(tiles), dim3(256), 0, s, set);
  DTD_LAUNCH_CHECK();
}
