// EXPERIMENT (round 5, not built): projection GEMM with B in MFMA-fragment order loaded straight
// into VGPRs.  Correct (tests were tests/test_proj_gpu.py, 9 passed) but 0.73-0.83x hipBLASLt
// (profiles/r5_s37_proj_fragB.jsonl): each B fragment is loaded by the two waves that share its
// columns, so L2 traffic per K-step is 1.5x the shared-LDS form's.  Kept as a record.
//
// Projection GEMM (NT) for gfx950 (MI355X / CDNA4): the Linear forward and input-gradient products.
//
//   C[M, N] (+)= A[M, K] . B[N, K]^T (+ bias[n])        bf16 in, fp32 accumulate, bf16 out
//
// A Linear forward is this product with A = the activations [tokens, in] and B = the weight
// [out, in]; its input gradient takes B = W^T.  Reference: the nn.Linear layers of
// /root/reference/model/transformer.py:37-40,50-51 and the HF BERT Linears trained by
// /root/reference/data_parallel_training.py:53-57.
//
// Operand delivery is what the round-3..5 forms of this product lost on (gemm.hip 0.89-0.92x of
// hipBLASLt, the LDS ring with both operands 0.81-0.87x: profiles/r5_s8_gemm_nt_ring.jsonl; the
// weight-gradient kernel's MFMA-only loop reaches 2.07 PF/s, its LDS-DMA + fragment reads cost a
// third, profiles/r5_s6_wgrad_limiter.jsonl).  So here:
//  * B (the weight, a few MiB, read by every row tile) never goes through LDS.  Once per step
//    it is packed into MFMA-fragment order (proj_pack_kernel: a 1 KiB block per 16 columns x 32 k,
//    lane-major), and each wave loads its fragments straight into VGPRs -- one coalesced 16-byte
//    buffer load per lane and fragment, from L2.
//  * A goes through a ring of 4 LDS stages, each the A panel of one 64-deep K-step (256 rows x
//    128 B = 32 KiB, full cache lines per LDS-DMA piece), filled by inline-asm LDS-DMA (dma16: no
//    compiler vmcnt drains); one barrier per K-step; A fragments read with ds_read_b128 two MFMA
//    groups ahead.  Chunk c of LDS row r sits at c ^ ((r >> 1) & 7): the 16 rows a 16-lane group
//    reads land on the 16 distinct 16-byte slots of the 64 banks.
//  * vmcnt counts returns in issue order, so each K-step issues the B loads of the next K-step
//    BEFORE the LDS-DMA of K-step + 3: the wait at the next barrier, vmcnt(4), retires those B loads
//    (and the A stage two ahead) and keeps the newest A stage in flight.
//  * Persistent: one 512-thread workgroup per CU walks a contiguous tile range of its XCD (the
//    tiles in flight on one XCD share A rows in its L2); the DMA and B cursors run across tile
//    boundaries, so the next tile's first K-steps land during this tile's epilogue.
// Waves: 8 as 2 (M) x 4 (N), each 128 x 64 of the 256 x 256 tile; MFMAs take the B fragment first
// (the tile is computed transposed) so a lane's accumulator holds 4 consecutive columns of one row.
#include <type_traits>

#include "common.h"

using namespace dtd;

namespace {

constexpr int BM = 256, BN = 256, BK = 64, NBUF = 4;
constexpr int ROWB = BK * 2;           // 128 bytes per LDS row (64 k)
constexpr int STAGE = BM * ROWB;       // 32 KiB: the A panel of one K-step
constexpr int DMA = 4;                 // LDS-DMA pieces (8 rows x 128 B) per wave per K-step
constexpr int KEEP = DMA;              // vmcnt at a barrier: the newest A stage stays in flight

enum ProjEpi : int { PJ_STORE = 0, PJ_ADD = 1 };

struct ProjArgs {
  const bf16* a;                       // A [M][K] (lda)
  const bf16* bp;                      // B packed: [N/16][K/32][64 lanes][8]
  bf16* c;                             // C [M][N] (ldc)
  const bf16* bias;                    // [N] or null (PJ_STORE)
  int M, N, K, lda, ldc;
};

__device__ __forceinline__ void bar() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ int fsw(int r) { return (r >> 1) & 7; }

__device__ __forceinline__ __amdgpu_buffer_rsrc_t uniform_rsrc(const void* p) {
  const uint64_t a = (uint64_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), (short)0, 0x7fffffff, 0x00020000);
}

template <int N> __device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" :: "n"(N) : "memory"); }

__device__ __forceinline__ bf16x4 cvt4(f32x4 v) {
  typedef float f32x2_t __attribute__((ext_vector_type(2)));
  const bf16x2 lo = __builtin_convertvector(f32x2_t{v[0], v[1]}, bf16x2);
  const bf16x2 hi = __builtin_convertvector(f32x2_t{v[2], v[3]}, bf16x2);
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3);
}

// one B fragment (16 columns x 32 k, 1 KiB) into this lane's 16 bytes
__device__ __forceinline__ bf16x8 bload(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
  typedef int i32x4 __attribute__((ext_vector_type(4)));
  const i32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, voff, __builtin_amdgcn_readfirstlane(soff), 0);
  return __builtin_bit_cast(bf16x8, v);
}

// vector-memory instructions one wave issues in an epilogue: 32 stores (+32 loads of C in place)
template <int EPI> constexpr int epi_vm() { return EPI == PJ_ADD ? 64 : 32; }

template <int EPI>
__global__ void __launch_bounds__(512, 1) proj_nt_kernel(ProjArgs g) {
  __shared__ __attribute__((aligned(1024))) char smem[NBUF * STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 15, lq = lane >> 4;
  const int wm = w >> 2, wn = w & 3;
  const int ntn = g.N / BN, ntiles = (g.M / BM) * ntn;
  const int nk = g.K / BK;   // a multiple of 12 (host check): every tile starts at ring position 0, slot phase 0
  const int KC = g.K / 32;
  // tile sequence: XCD group x owns tiles [beg, end), its member l takes beg + l + per * j
  const int nwg = gridDim.x, x = blockIdx.x % 8, l = blockIdx.x / 8, per = nwg / 8;
  const int q = ntiles / 8, r = ntiles % 8;
  const int beg = x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q;
  const int end = beg + q + (x < r ? 1 : 0);
  const int ntile = beg + l < end ? (end - beg - l + per - 1) / per : 0;
  if (ntile == 0) return;
  auto tile_m0 = [&](int j) __attribute__((always_inline)) { return ((beg + l + j * per) / ntn) * BM; };
  auto tile_n0 = [&](int j) __attribute__((always_inline)) { return ((beg + l + j * per) % ntn) * BN; };

  // ---- A: LDS-DMA piece i of wave w stages rows 32w + 8i + (lane >> 3), lane chunk (lane & 7)
  //      of the LDS row; the source chunk carries the swizzle
  int voa[DMA];
#pragma unroll
  for (int i = 0; i < DMA; ++i) {
    const int rr = 32 * w + 8 * i + (lane >> 3);
    voa[i] = rr * g.lda * 2 + (((lane & 7) ^ fsw(rr)) << 4);
  }
  const uint32_t lds0 = lds_addr(smem) + 32 * w * ROWB;
  int lj = 0, lk = 0;        // DMA cursor: tile lj, K-step lk
  auto ra = uniform_rsrc(g.a + (size_t)tile_m0(0) * g.lda);
  auto dma = [&](int buf, int i) __attribute__((always_inline)) { dma16(ra, lds0 + buf + 8 * i * ROWB, voa[i], lk * ROWB); };
  auto advance = [&]() __attribute__((always_inline)) {     // past the last tile it re-loads that tile's last K-step (harmless)
    if (lk + 1 < nk) {
      ++lk;
    } else if (lj + 1 < ntile) {
      ++lj;
      lk = 0;
      ra = uniform_rsrc(g.a + (size_t)tile_m0(lj) * g.lda);
    }
  };

  // ---- B: fragment (ni, c) of K-step k of the cursor's tile: column block (n0 + wn*64)/16 + ni,
  //      k chunk 2k + c; 1 KiB each, lane-major
  const auto rb = uniform_rsrc(g.bp);
  const int vob = lane * 16;
  int bj = 0, bk = 0;        // B cursor
  int bcol = (tile_n0(0) + wn * 64) / 16;
  auto bsoff = [&](int ni, int c) __attribute__((always_inline)) { return ((bcol + ni) * KC + 2 * bk + c) * 1024; };
  auto badvance = [&]() __attribute__((always_inline)) {
    if (bk + 1 < nk) {
      ++bk;
    } else if (bj + 1 < ntile) {
      ++bj;
      bk = 0;
      bcol = (tile_n0(bj) + wn * 64) / 16;
    }
  };

  // ---- A fragment reads: row wm*128 + mi*16 + li, chunk 4c + lq at (4c + lq) ^ fsw(li);
  //      stages 2 and 3 lie past the 64 KiB reach of the offset field: a second base register
  const int fl = fsw(li);
  // per-lane LDS byte addresses (VGPRs): k half c, stages 0/1 (lo) or 2/3 (hi); every read adds a
  // compile-time offset (stage parity, row block) that fits the instruction's 16-bit field
  const uint32_t lbase = lds_addr(smem) + wm * 128 * ROWB + li * ROWB;
  const uint32_t alo0 = lbase + ((lq ^ fl) << 4), alo1 = lbase + (((4 + lq) ^ fl) << 4);
  const uint32_t ahi0 = alo0 + 2 * STAGE, ahi1 = alo1 + 2 * STAGE;
  typedef __attribute__((address_space(3))) const bf16x8 lds_frag;
  auto fa = [&](auto pos_c, int mi, int c) __attribute__((always_inline)) {
    constexpr int POS = decltype(pos_c)::value;
    const uint32_t base = POS < 2 ? (c ? alo1 : alo0) : (c ? ahi1 : ahi0);
    return *(lds_frag*)(uintptr_t)(base + (POS & 1) * STAGE + mi * 16 * ROWB);
  };

  // ---- prologue: A K-steps 0, 1; B of K-step 0; A K-step 2 (the steady-state issue order)
#pragma unroll
  for (int s = 0; s < 2; ++s) {
#pragma unroll
    for (int i = 0; i < DMA; ++i) dma(s * STAGE, i);
    advance();
  }
  // B registers: 3 slots of one k half (4 column-block fragments).  K-step kt with slot phase SL
  // computes k half 0 from slot SL and half 1 from slot SL+1; it loads the next K-step's half 0
  // into slot SL+2 (free) and, once half 0 is done, its half 1 into slot SL.
  bf16x8 bs[3][4], a[3];
#pragma unroll
  for (int ni = 0; ni < 4; ++ni) bs[0][ni] = bload(rb, vob, bsoff(ni, 0));
#pragma unroll
  for (int ni = 0; ni < 4; ++ni) bs[1][ni] = bload(rb, vob, bsoff(ni, 1));
  badvance();
#pragma unroll
  for (int i = 0; i < DMA; ++i) dma(2 * STAGE, i);
  advance();
  wait_vm<KEEP>();
  bar();
  using P0 = std::integral_constant<int, 0>;
  a[0] = fa(P0{}, 0, 0);
  a[1] = fa(P0{}, 1, 0);
  f32x4 acc[8][4];

  // One K-step at ring position POS (stage POS), B slot phase SL.  16 MFMA groups g = (k half
  // c = g / 8, row block mi = g % 8): 4 MFMAs (the 4 column blocks) on A fragment (mi, c), which
  // was read two groups earlier (the next K-step's first two fragments come from its stage).
  // Groups 0-3 load the next K-step's B half 0, groups 8-11 its half 1, groups 12-15 issue the
  // LDS-DMA of the A cursor's K-step into the stage freed at this K-step's barrier -- the B loads
  // are older than the DMA the next barrier keeps in flight.  FIRST: the tile's first K-step (its
  // half-0 MFMAs take a zero C; after an epilogue its wait leaves the epilogue's stores in flight).
  auto kstep = [&](auto pos_c, auto sl_c, auto first_c, bool after_epi) __attribute__((always_inline)) {
    constexpr int POS = decltype(pos_c)::value;
    constexpr int SL = decltype(sl_c)::value;
    // A ring phase: 16 groups per K-step shift the 3-slot ring by one each K-step; the K-step index
    // mod 3 is (3 - SL) % 3 (SL runs 0, 2, 1, ...)
    constexpr int AP = (3 - SL) % 3;
    constexpr bool FIRST = decltype(first_c)::value;
    constexpr int prv = ((POS + NBUF - 1) % NBUF) * STAGE;
    constexpr int C0 = SL, C1 = (SL + 1) % 3, N0 = (SL + 2) % 3, N1 = SL;
    using PN = std::integral_constant<int, (POS + 1) % NBUF>;
    if (FIRST && after_epi) wait_vm<(KEEP + epi_vm<EPI>() > 63 ? 63 : KEEP + epi_vm<EPI>())>();
    else wait_vm<KEEP>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    bar();
#pragma clang loop unroll(full)
    for (int gi = 0; gi < 16; ++gi) {
      const int c = gi >> 3, mi = gi & 7;
      if (gi + 2 < 16) a[(gi + 2 + AP) % 3] = fa(pos_c, (gi + 2) & 7, (gi + 2) >> 3);
      else a[(gi + 2 + AP) % 3] = fa(PN{}, gi + 2 - 16, 0);
      if (gi < 4) {
        bs[N0][gi] = bload(rb, vob, bsoff(gi, 0));
      } else if (gi >= 8 && gi < 12) {
        bs[N1][gi - 8] = bload(rb, vob, bsoff(gi - 8, 1));
        if (gi == 11) badvance();
      } else if (gi >= 12) {
        dma(prv, gi - 12);
        if (gi == 15) advance();
      }
#pragma unroll
      for (int ni = 0; ni < 4; ++ni)
        acc[mi][ni] = mfma16(bs[c ? C1 : C0][ni], a[(gi + AP) % 3],
                             (FIRST && c == 0) ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[mi][ni]);
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  // 12 K-steps per pass: the ring position (period 4) and the B slot phase (period 3) repeat
  auto pass = [&](auto first_c, bool after_epi) __attribute__((always_inline)) {
    using F = std::false_type;
    kstep(std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{}, first_c, after_epi);
    kstep(std::integral_constant<int, 1>{}, std::integral_constant<int, 2>{}, F{}, false);
    kstep(std::integral_constant<int, 2>{}, std::integral_constant<int, 1>{}, F{}, false);
    kstep(std::integral_constant<int, 3>{}, std::integral_constant<int, 0>{}, F{}, false);
    kstep(std::integral_constant<int, 0>{}, std::integral_constant<int, 2>{}, F{}, false);
    kstep(std::integral_constant<int, 1>{}, std::integral_constant<int, 1>{}, F{}, false);
    kstep(std::integral_constant<int, 2>{}, std::integral_constant<int, 0>{}, F{}, false);
    kstep(std::integral_constant<int, 3>{}, std::integral_constant<int, 2>{}, F{}, false);
    kstep(std::integral_constant<int, 0>{}, std::integral_constant<int, 1>{}, F{}, false);
    kstep(std::integral_constant<int, 1>{}, std::integral_constant<int, 0>{}, F{}, false);
    kstep(std::integral_constant<int, 2>{}, std::integral_constant<int, 2>{}, F{}, false);
    kstep(std::integral_constant<int, 3>{}, std::integral_constant<int, 1>{}, F{}, false);
  };

  for (int j = 0; j < ntile; ++j) {
    pass(std::true_type{}, j > 0);
    for (int kt = 12; kt < nk; kt += 12) pass(std::false_type{}, false);
    // ---- epilogue: lane holds C[m][n .. n+3], m = m0 + wm*128 + mi*16 + li, n = n0 + wn*64 + ni*16 + 4 lq
    const int m0 = tile_m0(j), n0 = tile_n0(j);
    bf16* cb = g.c + (size_t)(m0 + wm * 128 + li) * g.ldc + n0 + wn * 64 + 4 * lq;
    if constexpr (EPI == PJ_ADD) {
      bf16x4 cin[8][4];
#pragma unroll
      for (int mi = 0; mi < 8; ++mi)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni)
          cin[mi][ni] = *reinterpret_cast<const bf16x4*>(cb + (size_t)mi * 16 * g.ldc + ni * 16);
#pragma unroll
      for (int mi = 0; mi < 8; ++mi)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni)
          *reinterpret_cast<bf16x4*>(cb + (size_t)mi * 16 * g.ldc + ni * 16) =
              cvt4(acc[mi][ni] + __builtin_convertvector(cin[mi][ni], f32x4));
    } else {
      f32x4 bv[4];
#pragma unroll
      for (int ni = 0; ni < 4; ++ni) {
        bv[ni] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (g.bias)
          bv[ni] = __builtin_convertvector(*reinterpret_cast<const bf16x4*>(g.bias + n0 + wn * 64 + ni * 16 + 4 * lq),
                                           f32x4);
      }
#pragma unroll
      for (int mi = 0; mi < 8; ++mi)
#pragma unroll
        for (int ni = 0; ni < 4; ++ni)
          *reinterpret_cast<bf16x4*>(cb + (size_t)mi * 16 * g.ldc + ni * 16) = cvt4(acc[mi][ni] + bv[ni]);
    }
  }
  wait_vm<0>();   // no LDS-DMA may land after the workgroup has released its LDS
}

// Bp[nj][kc][lane][e] = B[16 nj + (lane & 15)][32 kc + 8 (lane >> 4) + e]: B [N][K] from src [N][K]
// (trans = 0) or from src [K][N] (trans = 1: the input-gradient operand W^T of a weight W [K][N])
__global__ void __launch_bounds__(256) proj_pack_kernel(const bf16* __restrict__ src, int ld, int N, int K, int trans,
                                                        bf16x8* __restrict__ dst) {
  const int KC = K / 32;
  const size_t total = (size_t)(N / 16) * KC * 64;
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int lane = (int)(i & 63);
  const size_t rest = i >> 6;
  const int kc = (int)(rest % KC), nj = (int)(rest / KC);
  const int n = nj * 16 + (lane & 15), k0 = kc * 32 + (lane >> 4) * 8;
  bf16x8 v;
  if (!trans) {
    v = *reinterpret_cast<const bf16x8*>(src + (size_t)n * ld + k0);
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = src[(size_t)(k0 + e) * ld + n];
  }
  dst[i] = v;
}

int num_cus_proj() {
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

// K: whole passes of 12 K-steps (the ring period 4 times the B slot period 3): 768, 1536, 2304, 3072 ...
DTD_EXPORT int dtd_proj_supported(int M, int N, int K) {
  return M > 0 && N > 0 && M % BM == 0 && N % BN == 0 && K % (12 * BK) == 0 && K >= 12 * BK;
}

// pack B ([N][K], or [K][N] with trans) into dst (N * K bf16, 16-byte aligned)
DTD_EXPORT int dtd_proj_pack(const void* src, int ld, int N, int K, int trans, void* dst, hipStream_t s) {
  if (N % 16 || K % 32 || !src || !dst || ((uintptr_t)dst & 15)) return (int)hipErrorInvalidValue;
  if (!trans && (ld < K || ld % 8 || ((uintptr_t)src & 15))) return (int)hipErrorInvalidValue;
  if (trans && ld < N) return (int)hipErrorInvalidValue;
  const size_t total = (size_t)(N / 16) * (K / 32) * 64;
  hipLaunchKernelGGL(proj_pack_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, (const bf16*)src, ld, N,
                     K, trans, (bf16x8*)dst);
  DTD_LAUNCH_CHECK();
}

// epi: 0 = C = A B^T (+ bias), 1 = C += A B^T (in place); bp: B packed by dtd_proj_pack
DTD_EXPORT int dtd_proj_nt(int epi, const void* a, int lda, const void* bp, void* c, int ldc, const void* bias, int M,
                           int N, int K, hipStream_t s) {
  if (!dtd_proj_supported(M, N, K)) return (int)hipErrorInvalidValue;
  if ((lda | ldc) % 8 || lda < K || ldc < N || ((uintptr_t)bp & 15)) return (int)hipErrorInvalidValue;
  if ((size_t)M * lda * 2 >= 0x7fffffffull || (size_t)N * K * 2 >= 0x7fffffffull) return (int)hipErrorInvalidValue;
  ProjArgs g{(const bf16*)a, (const bf16*)bp, (bf16*)c, (const bf16*)bias, M, N, K, lda, ldc};
  const int ntiles = (M / BM) * (N / BN);
  const int cus = num_cus_proj() / 8 * 8;
  const int nwg = ntiles >= cus ? cus : (ntiles + 7) / 8 * 8;
  if (epi == PJ_ADD) hipLaunchKernelGGL(proj_nt_kernel<PJ_ADD>, dim3(nwg), dim3(512), 0, s, g);
  else if (epi == PJ_STORE) hipLaunchKernelGGL(proj_nt_kernel<PJ_STORE>, dim3(nwg), dim3(512), 0, s, g);
  else return (int)hipErrorInvalidValue;
  DTD_LAUNCH_CHECK();
}
