// Four-wave MFMA GEMM for gfx950 (MI355X / CDNA4): one wave per SIMD, 128 x 128 per wave.
//
//   C[M, N] = A[M, K] . B[N, K]^T (+ bias[n])     bf16 in, fp32 accumulate, both operands K-contiguous
//
// Why a second main loop next to gemm.hip's 8-wave one: at 8 waves of 128 x 64 each wave reads
// (128 + 64) rows of LDS per 128 x 64 outputs; at 4 waves of 128 x 128 it reads 256 rows per
// 128 x 128 -- a third fewer LDS bytes (and LDS instructions) per MFMA, which is both less issue
// pressure and less energy per FLOP (the MFMA loops run clock-limited, MI355X_MICROARCH.md "DVFS
// give-back").  The accumulators are 256 AGPRs (8 x 8 tiles of v_mfma_f32_16x16x32_bf16), the
// fragments and the staging ring live in the 256 arch VGPRs: one workgroup of 4 waves per CU.
//
// With one wave per SIMD nothing else hides a stall, so the loop is software-pipelined inside the
// wave: each 64-deep K-step is two 32-deep phases; while the 64 MFMAs of phase 0 run on fragment
// set F0, the wave reads fragment set F1 (the K-step's second half) from LDS, writes the staged
// registers of K-step kt+1 into the other LDS buffer and issues the global loads of K-step kt+2
// into the (now free) staging registers.  ONE barrier per K-step, in the middle: after it, phase
// 1's MFMAs run on F1 while the wave reads F0 of K-step kt+1 from the buffer just completed.  LDS
// latency and global latency both hide under MFMAs; only the barrier skew between the four waves
// is exposed.  Register staging (global_load_dwordx4 -> ds_write_b128), not LDS-DMA: a DMA issue
// costs ~60 cycles of the issuing wave among bare MFMAs (MI355X_MICROARCH.md cycle table), which
// at one wave per SIMD would idle the matrix pipe.
//
// LDS: two 64 KiB K-step buffers (A panel 256 rows x 128 B, then B panel); the 16-byte chunk c
// of row r sits at chunk c ^ (r & 7), which makes both the ds_write_b128 staging stores (8-lane
// groups = one row) and the ds_read_b128 fragment reads (16-lane groups = 16 rows at one chunk)
// bank-conflict free.  MFMAs take the B fragment first (the tile is computed transposed) so a
// lane's accumulator holds 4 consecutive columns of one row.
//
// Persistent: 8 XCD groups of workgroups each walk a contiguous tile range (N-minor, so the tiles
// in flight on one XCD share A panels in its L2).  The last K-step of a tile issues the global
// loads of the NEXT tile's K-step 0; the epilogue (two rounds of 128 rows through LDS buffer 1,
// stored as full 512-byte row segments) writes them into buffer 0 meanwhile, so the next tile
// starts with its first K-step resident.
#include <stdlib.h>
#include <type_traits>

#include "common.h"

using namespace dtd;

namespace {

constexpr int BM = 256, BN = 256, BK = 64;
constexpr int PANEL = 256 * BK * 2;   // 32 KiB: 256 rows x 128 B
constexpr int BUF = 2 * PANEL;        // A and B panels of one K-step
constexpr int LDS_BYTES = 2 * BUF;    // 128 KiB

enum Epi4 : int { E4_STORE = 0, E4_LAST = E4_STORE };

struct G4Args {
  const bf16* a; const bf16* b;   // A [M, K] (lda), B [N, K] (ldb)
  bf16* c;                        // C [M, N] (ldc)
  const bf16* bias;               // [N] or null
  int M, N, K, lda, ldb, ldc;
};

// raw workgroup barrier (no vmcnt drain: the staging loads stay in flight across it) that the
// compiler also treats as a memory barrier
__device__ __forceinline__ void bar() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t uniform_rsrc(const void* p) {
  const uint64_t a = (uint64_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), (short)0, 0x7fffffff, 0x00020000);
}

__device__ __forceinline__ bf16x4 cvt4(f32x4 v) {
  typedef float f32x2_t __attribute__((ext_vector_type(2)));
  const bf16x2 lo = __builtin_convertvector(f32x2_t{v[0], v[1]}, bf16x2);
  const bf16x2 hi = __builtin_convertvector(f32x2_t{v[2], v[3]}, bf16x2);
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3);
}

// DIAG (timing-only builds, wrong results unless 0): 1 = no barrier in the K loop, 2 = every
// K-step loads K-step 0 of its tile (L2-hot source), 4 = no staging stores, 8 = no loads in the loop
template <int EPI, int DIAG = 0>
__global__ void __launch_bounds__(256, 1) gemm4_kernel(G4Args g) {
  __shared__ __attribute__((aligned(1024))) char smem[LDS_BYTES];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 15, lq = lane >> 4;
  const int wm = w >> 1, wn = w & 1;
  const int ntn = g.N / BN, ntiles = (g.M / BM) * ntn, nk = g.K / BK;
  // tile sequence: XCD group x owns tiles [beg, end), its member l takes beg + l + per * i
  const int nwg = gridDim.x, x = blockIdx.x % 8, l = blockIdx.x / 8, per = nwg / 8;
  const int q = ntiles / 8, r = ntiles % 8;
  const int beg = x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q;
  const int end = beg + q + (x < r ? 1 : 0);
  int t = beg + l;
  if (t >= end) return;
  int m0 = (t / ntn) * BM, n0 = (t % ntn) * BN;

  // staging: thread = chunk sc of rows srow + 32 i (i = 0..7) of both panels
  const int srow = tid >> 3, sc = tid & 7;
  const int lst = srow * 128 + ((sc ^ (srow & 7)) << 4);
  const int voa = (srow * g.lda + sc * 8) * 2, vob = (srow * g.ldb + sc * 8) * 2;
  const int sta = 32 * g.lda * 2, stb = 32 * g.ldb * 2;
  // fragment reads: row li of each 16-row block, chunk (ks * 4 + lq) swizzled by li & 7
  const int fa = (wm * 128 + li) * 128, fb = PANEL + (wn * 128 + li) * 128;
  const int ch0 = (lq ^ (li & 7)) << 4, ch1 = ((4 + lq) ^ (li & 7)) << 4;

  bf16x8 R[16];
  auto gload = [&](__amdgpu_buffer_rsrc_t ra, __amdgpu_buffer_rsrc_t rb, int kt) {
    const int ko = (DIAG & 2) ? 0 : kt * BK * 2;
#pragma unroll
    for (int i = 0; i < 8; ++i)
      R[i] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(ra, voa, i * sta + ko, 0));
#pragma unroll
    for (int i = 0; i < 8; ++i)
      R[8 + i] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rb, vob, i * stb + ko, 0));
  };
  auto swrite = [&](char* buf) {
    if constexpr ((DIAG & 4) != 0) return;
#pragma unroll
    for (int i = 0; i < 8; ++i) *reinterpret_cast<bf16x8*>(buf + lst + i * 4096) = R[i];
#pragma unroll
    for (int i = 0; i < 8; ++i) *reinterpret_cast<bf16x8*>(buf + PANEL + lst + i * 4096) = R[8 + i];
  };
  bf16x8 A0[8], B0[8], A1[8], B1[8];
  auto fread = [&](const char* buf, int ch, bf16x8 (&A)[8], bf16x8 (&B)[8]) {
#pragma unroll
    for (int i = 0; i < 8; ++i) A[i] = *reinterpret_cast<const bf16x8*>(buf + fa + i * 2048 + ch);
#pragma unroll
    for (int i = 0; i < 8; ++i) B[i] = *reinterpret_cast<const bf16x8*>(buf + fb + i * 2048 + ch);
  };
  f32x4 acc[8][8];
  // MFMAs of accumulator rows [MLO, MHI) over one 32-deep fragment set
  auto mma = [&](auto zero_c, auto mlo_c, auto mhi_c, const bf16x8 (&A)[8], const bf16x8 (&B)[8]) {
    constexpr bool zero = decltype(zero_c)::value;
    constexpr int MLO = decltype(mlo_c)::value, MHI = decltype(mhi_c)::value;
#pragma unroll
    for (int mi = MLO; mi < MHI; ++mi)
#pragma unroll
      for (int ni = 0; ni < 8; ++ni)
        acc[mi][ni] = mfma16(B[ni], A[mi], zero ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[mi][ni]);
  };
  using I0 = std::integral_constant<int, 0>;
  using I2 = std::integral_constant<int, 2>;
  using I4 = std::integral_constant<int, 4>;
  using I8 = std::integral_constant<int, 8>;

  // The K-steps of all of this workgroup's tiles form one stream (global K-step gk, LDS buffer
  // gk & 1): K-step gk's phase 0 stages K-step gk + 1 (loaded during gk - 1) and loads gk + 2,
  // which past the end of a tile are the first K-steps of the next one -- so a tile boundary
  // costs only the epilogue.  Requires nk >= 2.
  auto rsa = uniform_rsrc(g.a + (size_t)m0 * g.lda), rsb = uniform_rsrc(g.b + (size_t)n0 * g.ldb);
  gload(rsa, rsb, 0);
  swrite(smem);
  gload(rsa, rsb, 1);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  bar();
  fread(smem, ch0, A0, B0);
  int gk = 0;

  while (true) {
    const int tn = t + per;
    const bool has_next = tn < end;
    const int m1 = has_next ? (tn / ntn) * BM : m0, n1 = has_next ? (tn % ntn) * BN : n0;
    const auto rsa1 = uniform_rsrc(g.a + (size_t)m1 * g.lda), rsb1 = uniform_rsrc(g.b + (size_t)n1 * g.ldb);
    auto kstep = [&](auto first_c, int kt) {
      char* cur = smem + (gk & 1) * BUF;
      char* nxt = smem + ((gk & 1) ^ 1) * BUF;
      ++gk;
      // K-step to load: kt + 2 of this tile, else of the next tile (the last tile re-loads its
      // own last K-step: a harmless unconsumed load keeps the issue unconditional)
      const bool here = kt + 2 < nk;
      const auto la = here ? rsa : rsa1, lb = here ? rsb : rsb1;
      const int lk = here ? kt + 2 : (has_next ? kt + 2 - nk : nk - 1);
      // ---- phase 0: MFMAs on F0 with the F1 reads, the staging stores of K-step gk + 1 and the
      //      loads of K-step gk + 2 interleaved
      fread(cur, ch1, A1, B1);
      mma(first_c, I0{}, I2{}, A0, B0);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // MFMA
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);   // DS read
      }
      __builtin_amdgcn_sched_barrier(0);
      swrite(nxt);
      mma(first_c, I2{}, I4{}, A0, B0);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // MFMA
        __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);   // DS write
      }
      __builtin_amdgcn_sched_barrier(0);
      if constexpr ((DIAG & 8) == 0) gload(la, lb, lk);
      mma(first_c, I4{}, I8{}, A0, B0);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);   // MFMA
        __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);   // VMEM read
      }
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if constexpr ((DIAG & 1) == 0) bar();
      // ---- phase 1: MFMAs on F1 with the F0 reads of K-step gk + 1
      fread(nxt, ch0, A0, B0);
      mma(std::false_type{}, I0{}, I8{}, A1, B1);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // MFMA
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);   // DS read
      }
      __builtin_amdgcn_sched_barrier(0);
    };
    kstep(std::true_type{}, 0);
    for (int kt = 1; kt < nk; ++kt) kstep(std::false_type{}, kt);

    // ---- epilogue through the buffer of the last K-step (free: the next tile's K-step 0 sits in
    //      the other one): fp32 bias, one bf16 rounding; two rounds of 128 rows (round rr carries
    //      accumulator rows mi = 4rr..4rr+3 of every wave: image row wm * 64 + (mi & 3) * 16 + li
    //      <-> tile row wm * 128 + mi * 16 + li), 8-byte slots XOR-swizzled by image row & 15,
    //      read back as 512-byte row segments of 16-byte vectors.
    f32x4 bv[8];
#pragma unroll
    for (int ni = 0; ni < 8; ++ni) {
      bv[ni] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (g.bias) {
        const bf16x4 b4 = *reinterpret_cast<const bf16x4*>(g.bias + n0 + wn * 128 + ni * 16 + 4 * lq);
        bv[ni] = __builtin_convertvector(b4, f32x4);
      }
    }
    char* img = smem + ((gk - 1) & 1) * BUF;
    const int c = lane & 31;
#pragma unroll
    for (int rr = 0; rr < 2; ++rr) {
#pragma unroll
      for (int m4 = 0; m4 < 4; ++m4) {
        const int mi = rr * 4 + m4;
        const int ir = wm * 64 + m4 * 16 + li;
#pragma unroll
        for (int ni = 0; ni < 8; ++ni) {
          const int n = wn * 128 + ni * 16 + 4 * lq;
          *reinterpret_cast<bf16x4*>(img + ir * 512 + (((n >> 2) ^ ((ir & 15) << 1)) << 3)) =
              cvt4(acc[mi][ni] + bv[ni]);
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      bar();
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int ir = w * 32 + 2 * i + (lane >> 5);
        const bf16x8 v = *reinterpret_cast<const bf16x8*>(img + ir * 512 + ((c ^ (ir & 15)) << 4));
        const int tr = (ir >> 6) * 128 + rr * 64 + (ir & 63);
        *reinterpret_cast<bf16x8*>(g.c + (size_t)(m0 + tr) * g.ldc + n0 + c * 8) = v;
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      bar();
    }
    if (!has_next) break;   // (the clamped, never-consumed loads of the last K-step drain below)
    t = tn;
    m0 = m1;
    n0 = n1;
    rsa = rsa1;
    rsb = rsb1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// ---------------------------------------------------------------------------------------------
// Ring form (default when K % 128 == 0, K >= 256): the staging registers form a TWO-deep ring, so
// a K-step's global loads are issued two K-steps (~4k cycles) before their LDS stores -- one
// K-step of lead (the form above) left the single wave per SIMD waiting on L2 / HBM latency.
// The registers for the second staging set come from the fragments: B fragments are double
// buffered per 32-deep slice (2 x 32 VGPRs) and A fragments are streamed one 16-row block ahead
// (2 x 4 VGPRs) instead of a whole K-step of both (128 VGPRs).  Streaming A means a buffer is read
// until the end of its K-step, so there are two barriers per K-step: B_j at its start (every wave
// finished reading K-step j-1's buffer -> K-step j+1 may be stored there) and B'_j in the middle
// (K-step j+1 stored -> its fragments may be read during slice 1).
//   K-step j, slice 0: MFMAs on (B0, A streamed) | read A of slice 0, B of slice 1 (buffer j) |
//                      store ring set (j+1)&1 = K-step j+1, reload it with K-step j+3
//   B'_j
//   K-step j, slice 1: MFMAs on (B1, A streamed) | read A of slice 1, then A / B of K-step j+1's
//                      slice 0 (buffer j+1)
template <int EPI, int DIAG = 0>
__global__ void __launch_bounds__(256, 1) gemm4r_kernel(G4Args g) {
  __shared__ __attribute__((aligned(1024))) char smem[LDS_BYTES];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 15, lq = lane >> 4;
  const int wm = w >> 1, wn = w & 1;
  const int ntn = g.N / BN, ntiles = (g.M / BM) * ntn, nk = g.K / BK;
  const int nwg = gridDim.x, x = blockIdx.x % 8, l = blockIdx.x / 8, per = nwg / 8;
  const int q = ntiles / 8, r = ntiles % 8;
  const int beg = x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q;
  const int end = beg + q + (x < r ? 1 : 0);
  int t = beg + l;
  if (t >= end) return;
  int m0 = (t / ntn) * BM, n0 = (t % ntn) * BN;

  const int srow = tid >> 3, sc = tid & 7;
  const int lst = srow * 128 + ((sc ^ (srow & 7)) << 4);
  const int voa = (srow * g.lda + sc * 8) * 2, vob = (srow * g.ldb + sc * 8) * 2;
  const int sta = 32 * g.lda * 2, stb = 32 * g.ldb * 2;
  const int fa = (wm * 128 + li) * 128, fb = PANEL + (wn * 128 + li) * 128;
  const int ch0 = (lq ^ (li & 7)) << 4, ch1 = ((4 + lq) ^ (li & 7)) << 4;

  bf16x8 R0[16], R1[16];
  // staging piece i of a K-step: i < 8 -> A rows srow + 32 i, else B rows srow + 32 (i - 8)
  auto gload1 = [&](bf16x8 (&R)[16], int i, __amdgpu_buffer_rsrc_t ra, __amdgpu_buffer_rsrc_t rb, int kt) {
    const int ko = (DIAG & 2) ? 0 : kt * BK * 2;
    if (i < 8) R[i] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(ra, voa, i * sta + ko, 0));
    else R[i] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rb, vob, (i - 8) * stb + ko, 0));
  };
  auto swrite1 = [&](const bf16x8 (&R)[16], char* buf, int i) {
    if constexpr ((DIAG & 4) != 0) return;
    *reinterpret_cast<bf16x8*>(buf + (i < 8 ? 0 : PANEL) + lst + (i & 7) * 4096) = R[i];
  };
  auto rdA = [&](const char* buf, int ch, int mi) { return *reinterpret_cast<const bf16x8*>(buf + fa + mi * 2048 + ch); };
  auto rdB = [&](const char* buf, int ch, int ni) { return *reinterpret_cast<const bf16x8*>(buf + fb + ni * 2048 + ch); };
  bf16x8 B0[8], B1[8], A0, A1;
  f32x4 acc[8][8];

  auto rsa = uniform_rsrc(g.a + (size_t)m0 * g.lda), rsb = uniform_rsrc(g.b + (size_t)n0 * g.ldb);
  // prologue: K-step 0 in buffer 0, K-steps 1 and 2 in flight in R1 / R0, fragments of K-step 0
#pragma unroll
  for (int i = 0; i < 16; ++i) gload1(R0, i, rsa, rsb, 0);
#pragma unroll
  for (int i = 0; i < 16; ++i) swrite1(R0, smem, i);
#pragma unroll
  for (int i = 0; i < 16; ++i) gload1(R1, i, rsa, rsb, 1);
#pragma unroll
  for (int i = 0; i < 16; ++i) gload1(R0, i, rsa, rsb, 2);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  bar();
#pragma unroll
  for (int ni = 0; ni < 8; ++ni) B0[ni] = rdB(smem, ch0, ni);
  A0 = rdA(smem, ch0, 0);

  while (true) {
    const int tn = t + per;
    const bool has_next = tn < end;
    const int m1 = has_next ? (tn / ntn) * BM : m0, n1 = has_next ? (tn % ntn) * BN : n0;
    const auto rsa1 = uniform_rsrc(g.a + (size_t)m1 * g.lda), rsb1 = uniform_rsrc(g.b + (size_t)n1 * g.ldb);
    // K-step j (parity PAR = j & 1, buffers fixed by it since nk is even)
    auto kstep = [&](auto par_c, auto first_c, int j) {
      constexpr int PAR = decltype(par_c)::value;
      constexpr bool FIRST = decltype(first_c)::value;
      bf16x8 (&Rw)[16] = PAR ? R0 : R1;   // holds K-step j+1 (loaded during j-2)
      char* cur = smem + PAR * BUF;
      char* nxt = smem + (PAR ^ 1) * BUF;
      const bool here = j + 3 < nk;
      const auto la = here ? rsa : rsa1, lb = here ? rsb : rsb1;
      const int lk = here ? j + 3 : (has_next ? j + 3 - nk : nk - 1);
      if constexpr ((DIAG & 1) == 0) bar();                  // B_j
      // ---- slice 0
#pragma unroll
      for (int mi = 0; mi < 8; ++mi) {
        bf16x8& Ac = (mi & 1) ? A1 : A0;
        bf16x8& An = (mi & 1) ? A0 : A1;
        An = mi < 7 ? rdA(cur, ch0, mi + 1) : rdA(cur, ch1, 0);
        if (mi >= 4) {
          B1[2 * (mi - 4)] = rdB(cur, ch1, 2 * (mi - 4));
          B1[2 * (mi - 4) + 1] = rdB(cur, ch1, 2 * (mi - 4) + 1);
        }
        swrite1(Rw, nxt, 2 * mi);
        swrite1(Rw, nxt, 2 * mi + 1);
        if constexpr ((DIAG & 8) == 0) {
          gload1(Rw, 2 * mi, la, lb, lk);
          gload1(Rw, 2 * mi + 1, la, lb, lk);
        }
#pragma unroll
        for (int ni = 0; ni < 8; ++ni)
          acc[mi][ni] = mfma16(B0[ni], Ac, FIRST ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[mi][ni]);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // MFMA
        __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);   // DS read
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
        __builtin_amdgcn_sched_group_barrier(0x200, 2, 0);   // DS write
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
        __builtin_amdgcn_sched_group_barrier(0x020, 2, 0);   // VMEM read
        __builtin_amdgcn_sched_group_barrier(0x008, 3, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if constexpr ((DIAG & 1) == 0) bar();                  // B'_j
      // ---- slice 1
#pragma unroll
      for (int mi = 0; mi < 8; ++mi) {
        bf16x8& Ac = (mi & 1) ? A1 : A0;
        bf16x8& An = (mi & 1) ? A0 : A1;
        An = mi < 7 ? rdA(cur, ch1, mi + 1) : rdA(nxt, ch0, 0);
        if (mi >= 4) {
          B0[2 * (mi - 4)] = rdB(nxt, ch0, 2 * (mi - 4));
          B0[2 * (mi - 4) + 1] = rdB(nxt, ch0, 2 * (mi - 4) + 1);
        }
#pragma unroll
        for (int ni = 0; ni < 8; ++ni) acc[mi][ni] = mfma16(B1[ni], Ac, acc[mi][ni]);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 3, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 7, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
    };
    kstep(std::integral_constant<int, 0>{}, std::true_type{}, 0);
    kstep(std::integral_constant<int, 1>{}, std::false_type{}, 1);
    for (int j = 2; j < nk; j += 2) {
      kstep(std::integral_constant<int, 0>{}, std::false_type{}, j);
      kstep(std::integral_constant<int, 1>{}, std::false_type{}, j + 1);
    }

    // ---- epilogue through buffer 1 (the last K-step's; buffer 0 holds the next tile's K-step 0)
    f32x4 bv[8];
#pragma unroll
    for (int ni = 0; ni < 8; ++ni) {
      bv[ni] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (g.bias) {
        const bf16x4 b4 = *reinterpret_cast<const bf16x4*>(g.bias + n0 + wn * 128 + ni * 16 + 4 * lq);
        bv[ni] = __builtin_convertvector(b4, f32x4);
      }
    }
    bar();   // every wave is done reading buffer 1
    char* img = smem + BUF;
    const int c = lane & 31;
#pragma unroll
    for (int rr = 0; rr < 2; ++rr) {
#pragma unroll
      for (int m4 = 0; m4 < 4; ++m4) {
        const int mi = rr * 4 + m4;
        const int ir = wm * 64 + m4 * 16 + li;
#pragma unroll
        for (int ni = 0; ni < 8; ++ni) {
          const int n = wn * 128 + ni * 16 + 4 * lq;
          *reinterpret_cast<bf16x4*>(img + ir * 512 + (((n >> 2) ^ ((ir & 15) << 1)) << 3)) =
              cvt4(acc[mi][ni] + bv[ni]);
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      bar();
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int ir = w * 32 + 2 * i + (lane >> 5);
        const bf16x8 v = *reinterpret_cast<const bf16x8*>(img + ir * 512 + ((c ^ (ir & 15)) << 4));
        const int tr = (ir >> 6) * 128 + rr * 64 + (ir & 63);
        *reinterpret_cast<bf16x8*>(g.c + (size_t)(m0 + tr) * g.ldc + n0 + c * 8) = v;
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      bar();
    }
    if (!has_next) break;
    t = tn;
    m0 = m1;
    n0 = n1;
    rsa = rsa1;
    rsb = rsb1;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

int num_cus4() {
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

DTD_EXPORT int dtd_gemm4_supported(int M, int N, int K) {
  return M > 0 && N > 0 && K >= 2 * BK && M % BM == 0 && N % BN == 0 && K % BK == 0;
}

DTD_EXPORT int dtd_gemm4_bt(int epi, const void* a, int lda, const void* b, int ldb, void* c, int ldc,
                            const void* bias, int M, int N, int K, hipStream_t s) {
  if (!dtd_gemm4_supported(M, N, K)) return (int)hipErrorInvalidValue;
  if ((lda | ldb | ldc) % 8 || lda < K || ldb < K || ldc < N) return (int)hipErrorInvalidValue;
  if (epi < E4_STORE || epi > E4_LAST) return (int)hipErrorInvalidValue;
  G4Args g{(const bf16*)a, (const bf16*)b, (bf16*)c, (const bf16*)bias, M, N, K, lda, ldb, ldc};
  const int ntiles = (M / BM) * (N / BN);
  const int cus = num_cus4() / 8 * 8;
  const int nwg = ntiles >= cus ? cus : (ntiles + 7) / 8 * 8;
  static const int diag = getenv("DTD_GEMM4_DIAG") ? atoi(getenv("DTD_GEMM4_DIAG")) : 0;
  static const int form = getenv("DTD_GEMM4_FORM") ? atoi(getenv("DTD_GEMM4_FORM")) : 1;
  if (form == 1 && K % (2 * BK) == 0 && K >= 4 * BK) {
    switch (diag) {
      case 1: hipLaunchKernelGGL((gemm4r_kernel<E4_STORE, 1>), dim3(nwg), dim3(256), 0, s, g); break;
      case 2: hipLaunchKernelGGL((gemm4r_kernel<E4_STORE, 2>), dim3(nwg), dim3(256), 0, s, g); break;
      case 4: hipLaunchKernelGGL((gemm4r_kernel<E4_STORE, 4>), dim3(nwg), dim3(256), 0, s, g); break;
      case 8: hipLaunchKernelGGL((gemm4r_kernel<E4_STORE, 8>), dim3(nwg), dim3(256), 0, s, g); break;
      case 15: hipLaunchKernelGGL((gemm4r_kernel<E4_STORE, 15>), dim3(nwg), dim3(256), 0, s, g); break;
      default: hipLaunchKernelGGL((gemm4r_kernel<E4_STORE, 0>), dim3(nwg), dim3(256), 0, s, g);
    }
    DTD_LAUNCH_CHECK();
  }
  switch (diag) {
    case 1: hipLaunchKernelGGL((gemm4_kernel<E4_STORE, 1>), dim3(nwg), dim3(256), 0, s, g); break;
    case 2: hipLaunchKernelGGL((gemm4_kernel<E4_STORE, 2>), dim3(nwg), dim3(256), 0, s, g); break;
    case 4: hipLaunchKernelGGL((gemm4_kernel<E4_STORE, 4>), dim3(nwg), dim3(256), 0, s, g); break;
    case 8: hipLaunchKernelGGL((gemm4_kernel<E4_STORE, 8>), dim3(nwg), dim3(256), 0, s, g); break;
    case 15: hipLaunchKernelGGL((gemm4_kernel<E4_STORE, 15>), dim3(nwg), dim3(256), 0, s, g); break;
    default: hipLaunchKernelGGL((gemm4_kernel<E4_STORE, 0>), dim3(nwg), dim3(256), 0, s, g);
  }
  DTD_LAUNCH_CHECK();
}
