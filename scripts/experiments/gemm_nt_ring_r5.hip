// EXPERIMENT (round 5, not built): ring-pipelined projection GEMM (NT).  Measured 0.83-0.87x of
// hipBLASLt and 0.87-0.90x of ops/csrc/gemm.hip on the BERT-base products
// (profiles/r5_s8_gemm_nt_ring.jsonl): 32-deep K-steps make every LDS-DMA piece 16 rows x 64 B
// (half cache lines), twice the L2 requests of the 64-deep form.  Kept as a record.
//
// Plain projection GEMM (NT) for gfx950 (MI355X / CDNA4): the Linear forward and input-gradient
// products of the transformer layers.
//
//   C[M, N] (+)= A[M, K] . B[N, K]^T (+ bias[n])        bf16 in, fp32 accumulate, bf16 out
//
// A Linear forward is exactly this product (A = the activations [tokens, in], B = the [out, in]
// weight); its input gradient uses B = W^T (ops/gemm.py transposed()).  Reference: the nn.Linear
// layers of /root/reference/model/transformer.py:37-40,50-51 and the HF BERT Linears trained by
// /root/reference/data_parallel_training.py:53-57.
//
// The main loop is the weight-gradient kernel's (ops/csrc/wgrad.hip) with K-contiguous operands:
// a ring of 4 LDS stages of 32-deep K-steps (A and B panels of 256 rows x 64 bytes, 32 KiB), three
// K-steps of LDS-DMA in flight at every barrier, ONE barrier per K-step, fragments read with
// ds_read_b128 one K-step (B) / two MFMA groups (A) ahead of their MFMAs, and the K loop unrolled
// by the ring so every fragment read is a lane offset plus an immediate.  Eight waves as 2 (M) x 4
// (N), each 128 x 64 of the 256 x 256 tile (8 x 4 v_mfma_f32_16x16x32_bf16 tiles).
//
// Persistent: one workgroup per CU walks a sequence of tiles (the XCD group b % 8 owns a contiguous
// N-minor tile range, so the tiles in flight on one XCD share A panels in its L2).  The ring runs
// across tile boundaries -- the last K-steps of a tile prefetch the first K-steps of the next --
// and a tile's epilogue (bias / residual in fp32, one bf16 rounding, 8-byte stores straight from
// the accumulators) runs while those land.  The first K-step after an epilogue waits with the
// epilogue's stores left in flight (vmcnt counts them younger than the DMA it needs).
//
// LDS image: a 64-byte row holds 4 chunks of 16 bytes (8 k); chunk c of row r sits at slot
// c ^ f(r), f(r) = 3 * ((r >> 3) & 1): the 16 (row, chunk) pairs each ds_read_b128 lane group
// reads (rows 0-15, chunks lq) land on 16 distinct 16-byte bank slots.  LDS-DMA destinations stay
// lane-linear; the source address carries the (involutive) swizzle.
#include <type_traits>

#include "common.h"

using namespace dtd;

namespace {

constexpr int BM = 256, BN = 256, BK = 32, NBUF = 4;
constexpr int ROWB = BK * 2;           // 64 bytes per LDS row
constexpr int PANEL = BM * ROWB;       // 16 KiB
constexpr int STAGE = 2 * PANEL;       // 32 KiB
constexpr int DMA = 4;                 // LDS-DMA pieces per wave per K-step
constexpr int KEEP = (NBUF - 3) * DMA;

enum NtEpi : int { NT_STORE = 0, NT_ADD = 1 };

struct NtArgs {
  const bf16* a; const bf16* b;        // A [M][K] (lda), B [N][K] (ldb)
  bf16* c;                             // [M][N] (ldc)
  const bf16* bias;                    // [N] or null (NT_STORE)
  int M, N, K, lda, ldb, ldc;
};

__device__ __forceinline__ void bar() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ int fsw(int r) { return 3 * ((r >> 3) & 1); }

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

// vector-memory instructions one wave issues in an epilogue (what the next tile's first wait
// leaves in flight): 32 stores, plus 32 loads of C for the in-place form
template <int EPI> constexpr int epi_vm() { return EPI == NT_ADD ? 64 : 32; }

template <int EPI>
__global__ void __launch_bounds__(512, 2) gemm_nt_kernel(NtArgs g) {
  __shared__ __attribute__((aligned(1024))) char smem[NBUF * STAGE];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 15, lq = lane >> 4;
  const int wm = w >> 2, wn = w & 3;
  const int ntn = g.N / BN, ntiles = (g.M / BM) * ntn;
  const int nk = g.K / BK;   // a multiple of 4 (host check): tiles start at a ring position 0
  // tile sequence: XCD group x owns tiles [beg, end), its member l takes beg + l + per * j
  const int nwg = gridDim.x, x = blockIdx.x % 8, l = blockIdx.x / 8, per = nwg / 8;
  const int q = ntiles / 8, r = ntiles % 8;
  const int beg = x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q;
  const int end = beg + q + (x < r ? 1 : 0);
  const int ntile = beg + l < end ? (end - beg - l + per - 1) / per : 0;
  if (ntile == 0) return;
  auto tile_m0 = [&](int j) { return ((beg + l + j * per) / ntn) * BM; };
  auto tile_n0 = [&](int j) { return ((beg + l + j * per) % ntn) * BN; };

  // ---- LDS-DMA: wave w stages rows 32w + 16(i & 1) + (lane >> 2) of panel i >> 1, 16 rows x
  //      64 bytes per piece; the source chunk carries the swizzle
  int voa[2], vob[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int rr = 32 * w + 16 * i + (lane >> 2);
    const int gc = (lane & 3) ^ fsw(rr);
    voa[i] = rr * g.lda * 2 + gc * 16;
    vob[i] = rr * g.ldb * 2 + gc * 16;
  }
  const uint32_t lds0 = lds_addr(smem) + 32 * w * ROWB;
  // load cursor: the K-step the next DMA fetches (tile lj of this workgroup, K-step lk)
  int lj = 0, lk = 0;
  auto ra = uniform_rsrc(g.a + (size_t)tile_m0(0) * g.lda);
  auto rb = uniform_rsrc(g.b + (size_t)tile_n0(0) * g.ldb);
  // DMA piece i of the cursor's K-step into stage byte offset `buf`
  auto dma = [&](int buf, int i) {
    const uint32_t dst = lds0 + buf + (i >> 1 ? PANEL : 0) + 16 * (i & 1) * ROWB;
    if (i >> 1) dma16(rb, dst, vob[i & 1], lk * ROWB);
    else dma16(ra, dst, voa[i & 1], lk * ROWB);
  };
  // advance the cursor (past the last tile it re-loads that tile's last K-step: harmless, keeps
  // the per-K-step DMA count -- and so every counted wait -- constant)
  auto advance = [&]() {
    if (lk + 1 < nk) {
      ++lk;
    } else if (lj + 1 < ntile) {
      ++lj;
      lk = 0;
      ra = uniform_rsrc(g.a + (size_t)tile_m0(lj) * g.lda);
      rb = uniform_rsrc(g.b + (size_t)tile_n0(lj) * g.ldb);
    }
  };

  // ---- fragment reads (ds_read_b128): A fragment mi = rows wm*128 + mi*16 + li, chunk lq;
  //      B fragment ni = rows wn*64 + ni*16 + li.  Stages 2 and 3 sit past the 64 KiB reach of the
  //      instruction's offset field: a second base register 64 KiB up.
  const int loff = li * ROWB + ((lq ^ fsw(li)) << 4);
  const char* abase = smem + loff + wm * 128 * ROWB;
  const char* bbase = smem + PANEL + loff + wn * 64 * ROWB;
  auto fa = [&](int buf, int mi) { return *reinterpret_cast<const bf16x8*>(abase + buf + mi * 16 * ROWB); };
  auto fb = [&](int buf, int ni) { return *reinterpret_cast<const bf16x8*>(bbase + buf + ni * 16 * ROWB); };

  // ---- prologue: stream K-steps 0..2 (nk >= 4: all in tile 0); fragments of K-step 0
#pragma unroll
  for (int s = 0; s < NBUF - 1; ++s) {
#pragma unroll
    for (int i = 0; i < DMA; ++i) dma(s * STAGE, i);
    advance();
  }
  wait_vm<(NBUF - 2) * DMA>();
  bar();
  bf16x8 b0[4], b1[4], a[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) b0[c] = fb(0, c);
  a[0] = fa(0, 0);
  a[1] = fa(0, 1);
  f32x4 acc[8][4];

  // One K-step (ring position POS, stage POS): MFMA group mi runs while the wave reads A fragment
  // mi + 2 (of the next K-step for mi >= 6), B fragment (mi - 1) / 2 of the next K-step (odd mi)
  // and issues one DMA piece of the cursor's K-step (mi < 4) into the stage freed at the previous
  // barrier.  FIRST: the tile's first K-step -- its MFMAs take a zero C operand, and its wait (when
  // an epilogue ran just before) leaves that epilogue's stores in flight.
  auto kstep = [&](auto pos_c, auto first_c, bool after_epi) {
    constexpr int POS = decltype(pos_c)::value;
    constexpr bool FIRST = decltype(first_c)::value;
    constexpr int cur = POS * STAGE, nxt = ((POS + 1) % NBUF) * STAGE, prv = ((POS + NBUF - 1) % NBUF) * STAGE;
    bf16x8 (&bc)[4] = (POS & 1) ? b1 : b0;
    bf16x8 (&bn)[4] = (POS & 1) ? b0 : b1;
    if (FIRST && after_epi) wait_vm<(KEEP + epi_vm<EPI>() > 63 ? 63 : KEEP + epi_vm<EPI>())>();
    else wait_vm<KEEP>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    bar();
#pragma unroll
    for (int mi = 0; mi < 8; ++mi) {
      if (mi < 6) a[(mi + 2) & 3] = fa(cur, mi + 2);
      else a[(mi + 2) & 3] = fa(nxt, mi - 6);
      if (mi & 1) bn[mi >> 1] = fb(nxt, mi >> 1);
      if (mi < DMA) dma(prv, mi);
      if (mi == DMA - 1) advance();
#pragma unroll
      for (int ni = 0; ni < 4; ++ni)
        acc[mi][ni] = mfma16(bc[ni], a[mi & 3], FIRST ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[mi][ni]);
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  using P0 = std::integral_constant<int, 0>;
  using P1 = std::integral_constant<int, 1>;
  using P2 = std::integral_constant<int, 2>;
  using P3 = std::integral_constant<int, 3>;

  for (int j = 0; j < ntile; ++j) {
    kstep(P0{}, std::true_type{}, j > 0);
    kstep(P1{}, std::false_type{}, false);
    kstep(P2{}, std::false_type{}, false);
    kstep(P3{}, std::false_type{}, false);
    for (int kt = 4; kt < nk; kt += 4) {
      kstep(P0{}, std::false_type{}, false);
      kstep(P1{}, std::false_type{}, false);
      kstep(P2{}, std::false_type{}, false);
      kstep(P3{}, std::false_type{}, false);
    }
    // ---- epilogue: lane holds C[m][n .. n+3], m = m0 + wm*128 + mi*16 + li,
    //      n = n0 + wn*64 + ni*16 + 4 lq
    const int m0 = tile_m0(j), n0 = tile_n0(j);
    bf16* cb = g.c + (size_t)(m0 + wm * 128 + li) * g.ldc + n0 + wn * 64 + 4 * lq;
    if constexpr (EPI == NT_ADD) {
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

int num_cus_nt() {
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

DTD_EXPORT int dtd_gemm_nt_supported(int M, int N, int K) {
  return M > 0 && N > 0 && M % BM == 0 && N % BN == 0 && K % (NBUF * BK) == 0 && K >= NBUF * BK;
}

// epi: 0 = C = A B^T (+ bias), 1 = C += A B^T (in place)
DTD_EXPORT int dtd_gemm_nt(int epi, const void* a, int lda, const void* b, int ldb, void* c, int ldc,
                           const void* bias, int M, int N, int K, hipStream_t s) {
  if (!dtd_gemm_nt_supported(M, N, K)) return (int)hipErrorInvalidValue;
  if ((lda | ldb | ldc) % 8 || lda < K || ldb < K || ldc < N) return (int)hipErrorInvalidValue;
  if ((size_t)M * lda * 2 >= 0x7fffffffull || (size_t)N * ldb * 2 >= 0x7fffffffull) return (int)hipErrorInvalidValue;
  NtArgs g{(const bf16*)a, (const bf16*)b, (bf16*)c, (const bf16*)bias, M, N, K, lda, ldb, ldc};
  const int ntiles = (M / BM) * (N / BN);
  const int cus = num_cus_nt() / 8 * 8;
  const int nwg = ntiles >= cus ? cus : (ntiles + 7) / 8 * 8;
  if (epi == NT_ADD) hipLaunchKernelGGL(gemm_nt_kernel<NT_ADD>, dim3(nwg), dim3(512), 0, s, g);
  else if (epi == NT_STORE) hipLaunchKernelGGL(gemm_nt_kernel<NT_STORE>, dim3(nwg), dim3(512), 0, s, g);
  else return (int)hipErrorInvalidValue;
  DTD_LAUNCH_CHECK();
}
