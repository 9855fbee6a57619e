// Weight-gradient GEMM (TN) for gfx950 (MI355X / CDNA4).
//
//   P[split][M][N] = A[k0:k1, :M]^T . B[k0:k1, :N]       bf16 in, fp32 partials out
//
// A Linear layer's weight gradient dW[o, i] = sum_t dY[t, o] X[t, i]: A = dY [T][o], B = X [T][i],
// both row-major over the token dimension, the reduction runs DOWN the rows.  Reference: the
// nn.Linear layers of /root/reference/model/transformer.py:37-40,50-51 and the HF BERT Linears
// trained by /root/reference/data_parallel_training.py:53-57 (backward at :55).
//
// Why this shape of kernel.  The output is small (768 x 768 .. 3072 x 768 = 9..36 tiles of 256 x 256)
// and K = tokens is huge (131072 at bench.py's b256), so the grid is split-K: every workgroup owns
// one 256 x 256 tile and one contiguous token range, and the number of ranges is chosen so that
// tiles x ranges fills the CUs once (one 512-thread workgroup per CU).  Each workgroup then runs
// one long K loop, and the kernel is a streaming kernel: every K-step brings 32 new token rows of
// both operands (32 KiB) that the workgroup has never seen.  The tiles of one range read the
// same rows, so the range's workgroups are placed on one XCD (T1 remap, tile index minor) and
// share those rows through its L2; the rows still come from HBM once per range, at the pace of
// the range's first reader.  What bounds the loop is therefore the HBM latency behind each
// K-step, not the MFMA work -- the round-2/3 TN kernel (ops/csrc/gemm.hip gemm_tn_kernel: two
// 64-deep K-step buffers, one K-step of lead) waited 16x longer on memory than hipBLASLt at the
// same MFMA count (profiles/r3b_wgrad_tn_pmc.json).  This kernel keeps NBUF-1 K-steps of LDS-DMA
// in flight (a ring of NBUF 32 KiB stages: 96-128 tokens of lead instead of 64) with ONE barrier
// per K-step, and software-pipelines the LDS fragment reads one K-step ahead in registers, so a
// wave's matrix work never waits on its own LDS reads.
//
// Layout.  A stage holds 32 token rows x 256 columns of A (16 KiB, 512-byte rows) then the same of
// B.  Each wave stages rows 4w .. 4w+3 of both panels by buffer_load_dwordx4 ... lds (two rows per
// instruction: lanes 0-31 one row, 32-63 the next), the 16-byte chunk index XOR-swizzled by
// swz(row) on the SOURCE address (the LDS destination of an LDS-DMA is lane-linear).  MFMA
// operands are read with the transposing ds_read_b64_tr_b16 (T10): a 16-lane group reads 4 token
// rows x 16 columns and lane i receives column i of the 4 rows, i.e. 4 consecutive k of one
// output row -- two reads make the 8-deep operand of v_mfma_f32_16x16x32_bf16.  The swizzle puts
// the 8 rows a 32-lane half reads ({8g + q, 8g + 8 + q}) on 8 distinct 32-byte bank slots.
//
// Waves: 8 as 2 (M) x 4 (N), each 128 x 64 of the tile = 8 x 4 MFMA tiles (128 fp32 accumulators).
// MFMAs take the B fragment first (the tile is computed transposed), so a lane's accumulator holds
// 4 consecutive columns of one row: the fp32 partial is stored as 16-byte vectors straight from
// the accumulators.  ops/csrc/reduce.hip (splitk_reduce) sums the ranges into the gradient.
//
// Measured alternatives (profiles/r5_s5_wgrad_unroll.jsonl, r5_s7_wgrad_4wave.jsonl): a 5-stage
// ring is no faster than 4; the K loop unrolled by the ring (variant 44, default) is 2-3 % faster
// than the rolled loop; a four-wave form (one wave per SIMD, 128 x 128 per wave: a third fewer LDS
// reads per MFMA; built with -mllvm -amdgpu-mfma-vgpr-form=1 to avoid scratch spills of its 256
// accumulators) ran 10 % slower -- with one wave per SIMD the DMA issue and waits sit in the MFMA
// stream.  Limiter probe (r5_s6_wgrad_limiter.jsonl, fc1 shape): no DMA -17 %, no barrier -7 %,
// no DMA / barrier / fragment reads -37 % (2.07 PF/s, the MFMA-only loop).
#include <type_traits>

#include "common.h"

using namespace dtd;

namespace {

typedef __attribute__((address_space(3))) void lds_void;
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

constexpr int BM = 256, BN = 256, BK = 32;
constexpr int ROWB = 512;              // bytes of one 256-column bf16 row
constexpr int PANEL = BK * ROWB;       // 16 KiB
constexpr int STAGE = 2 * PANEL;       // A and B panels of one K-step

struct WgArgs {
  const bf16* a; const bf16* b;        // A [K][M] (lda), B [K][N] (ldb)
  float* part;                         // [splits][M][N] fp32
  int M, N, K, lda, ldb;
  int splits, ksplit;                  // K-steps per range (the last range may be shorter)
};

// raw workgroup barrier (LDS-DMA stays in flight across it) that the compiler treats as a memory
// barrier: no LDS access is moved across it
__device__ __forceinline__ void bar() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ bf16x4 tr_read(const char* p) {
  const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p));
  return __builtin_bit_cast(bf16x4, v);
}

// 16-byte chunk XOR of LDS row t (bits 0, 1 and 3 of the row: rows t and t + 4 share it)
__device__ __forceinline__ int swz(int t) { return ((t & 3) | (((t >> 3) & 1) << 2)) << 1; }

// bijective XCD remap (cdna_hip_programming.md §5 "XCD swizzle must be bijective")
__device__ __forceinline__ int xcd_remap(int id, int n) {
  const int q = n / 8, r = n % 8, x = id % 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + id / 8;
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t uniform_rsrc(const void* p) {
  const uint64_t a = (uint64_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), (short)0, 0x7fffffff, 0x00020000);
}

template <int N> __device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" :: "n"(N) : "memory"); }

// LDS-DMA pieces go through dtd::dma16 (common.h): inline asm, counted only by this kernel's waits.

// NBUF: LDS ring depth (4 or 5 stages of 32 KiB).  The buffer of K-step j is read during
// K-steps j-1 (the B fragments and the first two A fragments, one K-step ahead) and j (the other
// A fragments, streamed two MFMA groups ahead), so it is free once barrier j+1 has passed: the DMA
// issued after barrier kt (spread over that K-step's MFMAs) fetches K-step kt + NBUF - 1 into the
// buffer of K-step kt - 1.  At barrier kt the wave needs K-step kt + 1 and keeps the NBUF - 3
// younger K-steps in flight.
// DIAG (timing-only builds, wrong results unless 0): 1 = no LDS-DMA in the K loop (stale stages),
// 2 = no barrier in the K loop, 4 = no fragment reads in the K loop (stale registers)
// SPREAD: the K-step's 4 DMA pieces go out with MFMA groups 0, 2, 4, 6 instead of 0-3 (one per 8
// MFMAs instead of one per 4 in the first half; the pieces' issue cost queued at the texture unit
// when bunched in gemm_w4.hip, profiles/r6_w4_pmc_bunched_dma.json)
template <int NBUF, bool UNROLL, int DIAG = 0, bool SPREAD = false>
__global__ void __launch_bounds__(512, 2) wgrad_tn_kernel(WgArgs g) {
  static_assert(NBUF >= 4 && NBUF <= 5 && (!UNROLL || NBUF == 4), "ring depth");
  constexpr int DMA = 4;                    // LDS-DMA instructions per wave per K-step
  constexpr int KEEP = (NBUF - 3) * DMA;    // vmcnt that retires K-step kt+1 at barrier kt
  __shared__ __attribute__((aligned(1024))) char smem[NBUF * STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 15, lq = lane >> 4;
  const int wm = w >> 2, wn = w & 3;
  const int ntn = g.N / BN, ntiles = (g.M / BM) * ntn;
  const int L = xcd_remap(blockIdx.x, gridDim.x);
  const int tile = L % ntiles, sp = L / ntiles;
  const int m0 = (tile / ntn) * BM, n0 = (tile % ntn) * BN;
  const int nk_all = g.K / BK;
  const int kb = sp * g.ksplit;
  const int nk = min(g.ksplit, nk_all - kb);
  float* out = g.part + (size_t)sp * g.M * g.N;
  if (nk <= 0) {   // empty range: a zero partial keeps the reduce a plain sum
    for (int i = tid; i < BM * BN / 4; i += 512) {
      const int r = i / (BN / 4), c = (i % (BN / 4)) * 4;
      *reinterpret_cast<f32x4*>(out + (size_t)(m0 + r) * g.N + n0 + c) = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    return;
  }

  // ---- LDS-DMA geometry: wave w stages token rows 4w + 2i + (lane >> 5) (i = 0, 1) of both panels
  int voa[2], vob[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r = 4 * w + 2 * i + (lane >> 5);
    const int gc = (lane & 31) ^ swz(r);
    voa[i] = (r * g.lda + gc * 8) * 2;
    vob[i] = (r * g.ldb + gc * 8) * 2;
  }
  const auto ra = uniform_rsrc(g.a + (size_t)kb * BK * g.lda + m0);
  const auto rb = uniform_rsrc(g.b + (size_t)kb * BK * g.ldb + n0);
  const int sa = BK * g.lda * 2, sb = BK * g.ldb * 2;   // bytes per K-step
  // DMA piece i (0..3: A pair 0, B pair 0, A pair 1, B pair 1) of K-step kt into buffer base `buf`
  const uint32_t lds0 = lds_addr(smem) + 4 * w * ROWB;   // this wave's first staged row
  auto dma = [&](int buf, int kt, int i) {                // buf: byte offset of the stage
    const uint32_t dst = lds0 + buf + (i >> 1 ? PANEL : 0) + 2 * (i & 1) * ROWB;
    if (i >> 1) dma16(rb, dst, vob[i & 1], kt * sb);
    else dma16(ra, dst, voa[i & 1], kt * sa);
  };

  // ---- transposing-read geometry: group lq reads rows 8 lq + (li >> 2) (+4), columns
  //      4 (li & 3) .. +3 of a 16-column block; one swizzle per lane (rows differ in bit 2 only).
  //      Column block c of the wave's A rows sits at chunk (wm*16 + 2c + (tcol>>3)) ^ tsw, and
  //      2c and tsw only touch chunk bits 1..3, so the per-block part is (2c ^ tsw) << 4.
  const int trow = 8 * lq + (li >> 2);
  const int tcol = 4 * (li & 3);
  const int tsw = swz(trow);
  //      The wave's B columns start at chunk 8 wn, which overlaps the swizzled bits: those four
  //      offsets are formed whole.
  const int tbase = trow * ROWB + (tcol & 7) * 2 + ((tcol >> 3) << 4);
  const int abase = tbase + wm * 256;
  auto aoff = [&](int c) { return abase + (((2 * c) ^ tsw) << 4); };
  int boffs[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) boffs[c] = PANEL + tbase + (((wn * 8 + 2 * c) ^ tsw) << 4);
  auto boff = [&](int c) { return boffs[c]; };
  auto frag = [&](const char* p) {
    return __builtin_shufflevector(tr_read(p), tr_read(p + 4 * ROWB), 0, 1, 2, 3, 4, 5, 6, 7);
  };

  // ---- prologue: K-steps 0 .. NBUF-2 in flight (indices past the range re-load its last K-step:
  //      every wave always issues DMA per K-step, so the counted waits are constants); wait
  //      for K-step 0; its B and first two A fragments
#pragma unroll
  for (int s = 0; s < NBUF - 1; ++s) {
#pragma unroll
    for (int i = 0; i < DMA; ++i) dma(s * STAGE, min(s, nk - 1), i);
  }
  wait_vm<(NBUF - 2) * DMA>();
  bar();
  bf16x8 b0[4], b1[4], a[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) b0[c] = frag(smem + boff(c));
  a[0] = frag(smem + aoff(0));
  a[1] = frag(smem + aoff(1));
  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // One K-step.  MFMA group mi (4 MFMAs on A fragment mi and the 4 B fragments of this K-step)
  // runs while the wave reads A fragment mi + 2 (of the next K-step for mi >= 6), half of a B
  // fragment of the next K-step (odd mi), and issues one DMA piece (mi < 4).  Nothing in the body
  // branches: past the range the DMA re-loads the range's last K-step into the free buffer and
  // the last K-step's reads of the "next" buffer are discarded.  cur / nxt / prv: byte offsets of
  // the buffers of K-steps kt, kt+1, kt-1 (compile-time constants in the unrolled form, so every
  // fragment read is a lane-offset register plus an immediate: no address VALU per K-step).
  auto kstep = [&](auto par_c, int kt, int cur, int nxt, int prv) {
    constexpr int PAR = decltype(par_c)::value;
    bf16x8 (&bc)[4] = PAR ? b1 : b0;
    bf16x8 (&bn)[4] = PAR ? b0 : b1;
    const int issue_k = min(kt + NBUF - 1, nk - 1);
    if constexpr (!(DIAG & 1)) wait_vm<KEEP>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if constexpr (!(DIAG & 2)) bar();
    const char* cb = smem + cur;
    const char* nb = smem + nxt;
#pragma unroll
    for (int mi = 0; mi < 8; ++mi) {
      if constexpr (!(DIAG & 4)) {
        if (mi < 6) a[(mi + 2) & 3] = frag(cb + aoff(mi + 2));
        else a[(mi + 2) & 3] = frag(nb + aoff(mi - 6));
        if (mi & 1) bn[mi >> 1] = frag(nb + boff(mi >> 1));
      } else {   // keep the registers live without reads
        asm volatile("" : "+v"(a[(mi + 2) & 3]));
        if (mi & 1) asm volatile("" : "+v"(bn[mi >> 1]));
      }
      if constexpr (SPREAD) {
        if (!(DIAG & 1) && (mi & 1) == 0) dma(prv, issue_k, mi >> 1);
      } else {
        if (!(DIAG & 1) && mi < DMA) dma(prv, issue_k, mi);
      }
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) acc[mi][ni] = mfma16(bc[ni], a[mi & 3], acc[mi][ni]);
      // keep each group's reads in their group: left alone the scheduler sinks a read down to the
      // MFMA group right before its consumer and exposes the LDS latency
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  if constexpr (UNROLL) {
    static_assert(NBUF % 2 == 0, "the B fragment parity follows the buffer index");
    using P0 = std::integral_constant<int, 0>;
    using P1 = std::integral_constant<int, 1>;
    for (int kt = 0; kt < nk; kt += NBUF) {
      kstep(P0{}, kt, 0, STAGE, (NBUF - 1) * STAGE);
      if (kt + 1 >= nk) break;
      kstep(P1{}, kt + 1, STAGE, 2 * STAGE, 0);
      if (kt + 2 >= nk) break;
      kstep(P0{}, kt + 2, 2 * STAGE, 3 * STAGE % (NBUF * STAGE), STAGE);
      if (kt + 3 >= nk) break;
      kstep(P1{}, kt + 3, 3 * STAGE, 4 * STAGE % (NBUF * STAGE), 2 * STAGE);
      if constexpr (NBUF == 6) {
        if (kt + 4 >= nk) break;
        kstep(P0{}, kt + 4, 4 * STAGE, 5 * STAGE, 3 * STAGE);
        if (kt + 5 >= nk) break;
        kstep(P1{}, kt + 5, 5 * STAGE, 0, 4 * STAGE);
      }
    }
  } else {
    int cur = 0;
    for (int kt = 0; kt < nk; kt += 2) {
      int nxt = cur + STAGE == NBUF * STAGE ? 0 : cur + STAGE;
      int prv = cur == 0 ? (NBUF - 1) * STAGE : cur - STAGE;
      kstep(std::integral_constant<int, 0>{}, kt, cur, nxt, prv);
      cur = nxt;
      if (kt + 1 >= nk) break;
      nxt = cur + STAGE == NBUF * STAGE ? 0 : cur + STAGE;
      prv = cur == 0 ? (NBUF - 1) * STAGE : cur - STAGE;
      kstep(std::integral_constant<int, 1>{}, kt + 1, cur, nxt, prv);
      cur = nxt;
    }
  }
  wait_vm<0>();   // no LDS-DMA may land after the workgroup has released its LDS

  // ---- fp32 partial tile straight from the accumulators: lane holds P[m][n .. n+3]
#pragma unroll
  for (int mi = 0; mi < 8; ++mi)
#pragma unroll
    for (int ni = 0; ni < 4; ++ni)
      *reinterpret_cast<f32x4*>(out + (size_t)(m0 + wm * 128 + mi * 16 + li) * g.N + n0 + wn * 64 + ni * 16 +
                                4 * lq) = acc[mi][ni];
}

int num_cus() {
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

DTD_EXPORT int dtd_wgrad_tn_supported(int M, int N, int K) {
  return M > 0 && N > 0 && K >= BK && M % BM == 0 && N % BN == 0 && K % BK == 0;
}

// ranges per tile: tiles x ranges <= CUs (one wave of workgroups), at least one
DTD_EXPORT int dtd_wgrad_tn_splits(int M, int N, int K) {
  const int tiles = (M / BM) * (N / BN);
  int s = num_cus() / (tiles > 0 ? tiles : 1);
  const int nk = K / BK;
  if (s > nk) s = nk;
  return s < 1 ? 1 : s;
}

// variant: LDS ring depth (4 or 5; 44 = depth 4, K loop unrolled by the ring); 0 = default
DTD_EXPORT int dtd_wgrad_tn(int variant, const void* a, int lda, const void* b, int ldb, void* part, int M, int N,
                            int K, int splits, hipStream_t s) {
  if (!dtd_wgrad_tn_supported(M, N, K) || splits < 1) return (int)hipErrorInvalidValue;
  if ((lda | ldb) % 8 || lda < M || ldb < N) return (int)hipErrorInvalidValue;
  const int nk = K / BK;
  const int ksplit = (nk + splits - 1) / splits;
  // buffer offsets are 32-bit; each workgroup's resource starts at its own K-range
  const size_t rows = (size_t)ksplit * BK;
  if (rows * lda * 2 >= 0x7fffffffull || rows * ldb * 2 >= 0x7fffffffull) return (int)hipErrorInvalidValue;
  WgArgs g{(const bf16*)a, (const bf16*)b, (float*)part, M, N, K, lda, ldb, splits, ksplit};
  const int nwg = (M / BM) * (N / BN) * splits;
  if (variant == 0) {   // 46: 128 KiB (leaves LDS for a co-resident side-stream kernel), spread DMA:
    // 5697 vs 5736 us per b1024 layer, +0.2 % step in both interleaved rounds
    // (profiles/r6_wgrad_spread.jsonl); DTD_WGRAD_VARIANT=44 restores the bunched pieces
    const char* e = getenv("DTD_WGRAD_VARIANT");
    variant = e ? atoi(e) : 46;
  }
  switch (variant) {
    case 4: hipLaunchKernelGGL((wgrad_tn_kernel<4, false>), dim3(nwg), dim3(512), 0, s, g); break;
    case 5: hipLaunchKernelGGL((wgrad_tn_kernel<5, false>), dim3(nwg), dim3(512), 0, s, g); break;
    case 44: hipLaunchKernelGGL((wgrad_tn_kernel<4, true>), dim3(nwg), dim3(512), 0, s, g); break;
    case 46: hipLaunchKernelGGL((wgrad_tn_kernel<4, true, 0, true>), dim3(nwg), dim3(512), 0, s, g); break;
    // diagnostic (timing-only) builds of variant 44: 440 + DIAG
    case 441: hipLaunchKernelGGL((wgrad_tn_kernel<4, true, 1>), dim3(nwg), dim3(512), 0, s, g); break;
    case 442: hipLaunchKernelGGL((wgrad_tn_kernel<4, true, 2>), dim3(nwg), dim3(512), 0, s, g); break;
    case 443: hipLaunchKernelGGL((wgrad_tn_kernel<4, true, 3>), dim3(nwg), dim3(512), 0, s, g); break;
    case 447: hipLaunchKernelGGL((wgrad_tn_kernel<4, true, 7>), dim3(nwg), dim3(512), 0, s, g); break;
    default: return (int)hipErrorInvalidValue;
  }
  DTD_LAUNCH_CHECK();
}
