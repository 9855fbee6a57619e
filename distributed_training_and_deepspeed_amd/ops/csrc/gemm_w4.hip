// Plain projection GEMM for gfx950 (MI355X / CDNA4): one wave per SIMD, 128 x 128 per wave.
//
//   C[M, N] = A[M, K] . B[N, K]^T (+ bias[n])      EPI_STORE   (Linear forward, NT input gradient)
//   C[M, N] += A[M, K] . B[N, K]^T                  EPI_ADD     (residual-branch input gradient)
//
// bf16 operands, fp32 accumulation, one bf16 rounding.  This is the delivery schedule of the
// library kernel that ran these products before (hipBLASLt's stream-K MT256x256x64 kernel; its main
// loop, disassembled from the shipped code object for study, is in profiles/r6_hipblaslt_sk3_mainloop.s),
// re-derived for this framework's LDS image, tile order and epilogues:
//
// * 256-thread workgroup, one per CU (128 KiB of LDS), waves 2 (M) x 2 (N), each wave owns a
//   128 x 128 output block = 8 x 8 tiles of v_mfma_f32_16x16x32_bf16 with its 256 fp32 accumulators in
//   AGPRs (inline-asm MFMAs with "+a" operands: hipcc never moves them).  Per 64-deep K-step a wave
//   issues 128 MFMAs against 32 ds_read_b128 and 16 LDS-DMA pieces -- a quarter of a fragment read per
//   MFMA, where the 8-wave kernel of gemm.hip needs 3/8 and 8 barriers.
// * A K-step's whole fragment set lives in VGPRs: R0 = the first 32 k (8 A + 8 B fragments), R1 = the
//   second 32.  Phase 0 (MFMAs on R0) reads R1 from the current LDS buffer; once every wave has
//   its R1 (barrier 1) the buffer is free and the 16 pieces of K-step s + 2 land in it by LDS-DMA
//   (buffer_load_dwordx4 ... lds) while phase 0 continues.  Phase 1 (MFMAs on R1) waits for K-step
//   s + 1's pieces (issued one K-step earlier; counted vmcnt), barrier 2, and reads the next R0.
//   Two buffers therefore carry three K-steps in flight: registers, landed, landing.  Two barriers
//   per K-step, and no MFMA ever waits on an LDS read issued less than ~10 MFMAs earlier.
// * Persistent: one workgroup per CU walks its tiles in the XCD-aware order of gemm.hip (the 32
//   workgroups of an XCD take consecutive tiles, so tiles in flight on an XCD share A panels).  The
//   K-step stream runs straight across tiles: the last two K-steps of a tile prefetch the next
//   tile's first two, so its epilogue runs while they land and nothing drains between tiles.
// * LDS image: [row][64 k] rows of 128 B, 16-byte chunk index XOR (row & 7) (conflict-free
//   ds_read_b128 and DMA writes; the DMA source address carries the swizzle).  The B rows are stored
//   permuted (sigma below) so that after the MFMAs a lane holds 8 consecutive output columns per
//   pair of tiles: the epilogue stores 16-byte vectors straight from the accumulators (a wave
//   instruction covers 16 rows x 64 contiguous bytes), no LDS round trip.
// * Bias: each wave DMAs the tile's bias row into its own 1 KiB LDS slot with the first K-step of
//   the tile (older than every counted wait that follows, so it has landed by the epilogue).
//
// Shape contract (host-checked): M % 256 == 0, N % 256 == 0, K % 64 == 0, K >= 128, leading
// dimensions % 8 == 0, 16-byte aligned bases.
#include <type_traits>

#include "common.h"

using namespace dtd;

namespace {

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

constexpr int BM = 256, BN = 256, BK = 64;
constexpr int BUF = 65536;            // one K-step: A [256][128 B] then B [256][128 B]
constexpr int B_OFF = 32768;
constexpr int BIAS_OFF = 2 * BUF;     // 4 x 1 KiB bias slots (one per wave)
constexpr int LDS_BYTES = 2 * BUF + 4096;

enum : int { EPI_STORE = 0, EPI_ADD = 3 };

// Schedule of one K-step (128 MFMA slots; side operations follow the MFMA of their slot):
//   slots 0..15       R1 fragment reads (cur), one per MFMA
//   slot  19          lgkmcnt(0) + barrier 1: cur is free
//   slots 20 + 7k     the 16 LDS-DMA pieces of K-step s + 2 into cur, k = 0..15 (..125): spread
//                     over the K-step so the 4 waves' pieces never queue at the texture unit
//                     (a piece is 1 KiB; bunched 1 per 2 MFMAs they stalled the MFMA issue)
//   slot  64 + B2I    vmcnt(pieces of this step issued so far) + barrier 2: K-step s + 1 landed
//   slots 64+B2I+1+2k R0 fragment reads of K-step s + 1 (nxt), k = 0..15
// (DMA0, DSTEP, B2I) is a template parameter set: SCHEDS lists the measured forms, SCHED_DEFAULT the
// one that runs (dtd_gemm_w4_set_sched picks another for A/B runs, scripts/bench_gemm_w4.py).
template <int DMA0, int DSTEP, int B2I>
struct Sched {
  static constexpr int dma0 = DMA0, dstep = DSTEP, b2i = B2I;
  static constexpr int dma_slot(int k) { return DMA0 + DSTEP * k; }
  static constexpr int pieces_before(int slot) {
    int n = 0;
    for (int k = 0; k < 16; ++k) n += dma_slot(k) < slot ? 1 : 0;
    return n;
  }
  static constexpr int nb2 = pieces_before(64 + B2I);
  static_assert(DMA0 > 19 && dma_slot(15) < 128 && nb2 < 16 && B2I + 31 < 64, "K-step schedule");
};
// (the round-6 sweep over DMA0 20-21, DSTEP 6-7, B2I 16-30 measured all forms within 1 %,
// profiles/r6_w4_sched.jsonl; two are kept.  Non-temporal epilogue stores lost 1 %: the next kernel
// reads these outputs, profiles/r6_w4nt.jsonl)
#define DTD_W4_SCHEDS(X) X(0, 20, 7, 24) X(1, 20, 6, 24)
constexpr int SCHED_COUNT = 2, SCHED_DEFAULT = 0;

struct W4Args {
  const bf16* a; const bf16* b; bf16* c; const bf16* bias;
  int M, N, K, lda, ldb, ldc;
};

// ---- inline-asm building blocks (issue order = source order: every statement is volatile) ----
__device__ __forceinline__ void mfma_acc(f32x4& c, const i32x4& b, const i32x4& a) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c) : "v"(b), "v"(a));
}
__device__ __forceinline__ void mfma_zero(f32x4& c, const i32x4& b, const i32x4& a) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0" : "=a"(c) : "v"(b), "v"(a));
}
// LDS fragment read; the result is valid only after the matching s_waitcnt lgkmcnt
template <int OFF>
__device__ __forceinline__ void lds_rd(i32x4& d, uint32_t addr) {
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(d) : "v"(addr), "i"(OFF));
}
__device__ __forceinline__ void wait_lgkm0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
template <int N>
__device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" :: "n"(N) : "memory"); }
__device__ __forceinline__ void barrier() { asm volatile("s_barrier" ::: "memory"); }
// 16-byte store with two wait states behind it.  Issued through the builtin, hipcc let a VALU write
// (the next accumulator read) land on the store's data VGPRs in the very next instruction, and on
// gfx950 the stored bytes then came out corrupted -- rows of zeros where the data registers were
// reused (scripts/diag/w4_debug.py; any instruction between store and rewrite hid it).  In asm the
// wait is part of the statement, so no schedule can put a write closer.
__device__ __forceinline__ void store16(const i32x4& v, __amdgpu_buffer_rsrc_t r, int voff, int soff) {
  asm volatile("buffer_store_dwordx4 %0, %1, %2, %3 offen\n\ts_nop 1" :: "v"(v), "v"(voff), "s"(r), "s"(soff) : "memory");
}

// One LDS-DMA piece: 16 bytes per lane from rsrc + voff + soff to LDS address lds + 16 * lane.  M0 is
// written here and not restored: no instruction hipcc emits in this kernel reads M0 (checked on the
// ISA by tests/test_gemm_w4_asm_cpu.py), so the save / restore pair of common.h's dma16 is dropped
// (2 SALU issues per piece, 32 per K-step).  The s_nop covers the M0-write -> LDS-DMA hazard.
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ void dma_lds(__amdgpu_buffer_rsrc_t r, uint32_t lds, int voff, int soff) {
  asm volatile("s_mov_b32 m0, %0\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds"
               :: "s"(__builtin_amdgcn_readfirstlane(lds)), "v"(voff), "s"(r), "s"(__builtin_amdgcn_readfirstlane(soff))
               : "memory", "m0");
}
#pragma clang diagnostic pop

// 16-byte global load issued as asm (invisible to hipcc's wait-count pass, which would otherwise
// wait vmcnt(0) -- for every DMA piece in flight -- at its first use); the result may be read only
// after a counted wait that names it (wait_vm_pin) or one that provably retired it (pin_v4)
__device__ __forceinline__ void load16(i32x4& d, __amdgpu_buffer_rsrc_t r, int voff, int soff) {
  asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen" : "=v"(d) : "v"(voff), "s"(r), "s"(soff) : "memory");
}
__device__ __forceinline__ void pin_v4(i32x4 (&v)[4]) {
  asm volatile("" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]));
}
// The EPI_ADD prefetch of rows 0..2 (12 loads) as ONE asm statement executed at every K-step, whose
// loads are skipped by a scalar branch inside the statement unless `go` (the tile's last K-step):
// to hipcc the registers are written unconditionally every K-step, so their value never merges
// across a branch or the loop edge -- where hipcc copied the conditionally loaded registers,
// reading them before the data had landed (scripts/diag/audit_w4_asm.py).
__device__ __forceinline__ void prefetch3(i32x4 (&c)[3][4], int go, __amdgpu_buffer_rsrc_t r, int voff, int s0,
                                          int s1, int s2) {
  asm volatile(
      "s_cmp_eq_u32 %12, 0\n\ts_cbranch_scc1 .Lw4pf%=\n\t"
      "buffer_load_dwordx4 %0, %13, %14, %15 offen\n\tbuffer_load_dwordx4 %1, %13, %14, %15 offen offset:64\n\t"
      "buffer_load_dwordx4 %2, %13, %14, %15 offen offset:128\n\tbuffer_load_dwordx4 %3, %13, %14, %15 offen offset:192\n\t"
      "buffer_load_dwordx4 %4, %13, %14, %16 offen\n\tbuffer_load_dwordx4 %5, %13, %14, %16 offen offset:64\n\t"
      "buffer_load_dwordx4 %6, %13, %14, %16 offen offset:128\n\tbuffer_load_dwordx4 %7, %13, %14, %16 offen offset:192\n\t"
      "buffer_load_dwordx4 %8, %13, %14, %17 offen\n\tbuffer_load_dwordx4 %9, %13, %14, %17 offen offset:64\n\t"
      "buffer_load_dwordx4 %10, %13, %14, %17 offen offset:128\n\tbuffer_load_dwordx4 %11, %13, %14, %17 offen offset:192\n"
      ".Lw4pf%=:"
      : "=&v"(c[0][0]), "=&v"(c[0][1]), "=&v"(c[0][2]), "=&v"(c[0][3]), "=&v"(c[1][0]), "=&v"(c[1][1]),
        "=&v"(c[1][2]), "=&v"(c[1][3]), "=&v"(c[2][0]), "=&v"(c[2][1]), "=&v"(c[2][2]), "=&v"(c[2][3])
      : "s"(__builtin_amdgcn_readfirstlane(go)), "v"(voff), "s"(r), "s"(__builtin_amdgcn_readfirstlane(s0)),
        "s"(__builtin_amdgcn_readfirstlane(s1)), "s"(__builtin_amdgcn_readfirstlane(s2))
      : "memory", "scc");
}
template <int N>
__device__ __forceinline__ void wait_vm_pin(i32x4 (&v)[4]) {
  asm volatile("s_waitcnt vmcnt(%4)" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]) : "n"(N) : "memory");
}

// compile-time loop: f(std::integral_constant<int, I>) for I = B .. E-1, in order
template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, int bytes) {
  const uint64_t a = (uint64_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), (short)0, bytes, 0x00020000);
}

__device__ __forceinline__ int xcd_beg(int x, int ntiles) {
  const int q = ntiles / 8, r = ntiles % 8;
  return x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q;
}

// LDS row l (0..255) of the B image holds weight row sigma(l): within each 128-row half (a wave
// column), tile ni = (l >> 4) & 7, lane row i = l & 15 ->
//   32 (ni >> 1) + 8 (i >> 2) + 4 (ni & 1) + (i & 3)
// so the MFMA output of tiles 2j, 2j + 1 gives lane quad lq the columns 32 j + 8 lq + 0..7.
// For a DMA piece p (rows 8p .. 8p + 7, lane row d = lane >> 3) this is piece_row(p) + 8 (d >> 2) + (d & 3).
__host__ __device__ constexpr int b_piece_row(int p) {
  return (p >> 4) * 128 + 32 * ((p >> 2) & 3) + 16 * (p & 1) + 4 * ((p >> 1) & 1);
}

template <int EPI, typename SC>
__global__ void __launch_bounds__(256, 1) gemm_w4_kernel(W4Args g) {
  constexpr int B2I = SC::b2i, NB2 = SC::nb2;
  __shared__ __attribute__((aligned(1024))) char smem[LDS_BYTES];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = w >> 1, wn = w & 1;
  const int li = lane & 15, lq = lane >> 4;
  const int ntn = g.N / BN, ntiles = (g.M / BM) * ntn, nk = g.K / BK;
  const int nwg = gridDim.x, x = blockIdx.x % 8, l = blockIdx.x / 8, per = nwg / 8;
  const int beg = xcd_beg(x, ntiles), end = xcd_beg(x + 1, ntiles);
  int t = beg + l;
  if (t >= end) return;

  const uint32_t lds0 = lds_addr(smem);
  // ---- per-lane constants
  const int d = lane >> 3, sc = ((lane & 7) ^ d) * 8;                 // DMA: lane row, swizzled chunk
  const int vA = (d * g.lda + sc) * 2;
  const int vB = ((8 * (d >> 2) + (d & 3)) * g.ldb + sc) * 2;
  const uint32_t sw0 = ((lq ^ (li & 7)) * 16), sw1 = (((4 + lq) ^ (li & 7)) * 16);
  const uint32_t rA0 = lds0 + (wm * 128 + li) * 128 + sw0, rA1 = lds0 + (wm * 128 + li) * 128 + sw1;
  const uint32_t rB0 = lds0 + B_OFF + (wn * 128 + li) * 128 + sw0, rB1 = lds0 + B_OFF + (wn * 128 + li) * 128 + sw1;

  // ---- DMA cursor: the K-step two ahead of the compute side
  int dt = t, dkt = 0;
  auto rsA_of = [&](int tt) { return rsrc(g.a + (size_t)(tt / ntn) * BM * g.lda, 0x7fffffff); };
  auto rsB_of = [&](int tt) { return rsrc(g.b + (size_t)(tt % ntn) * BN * g.ldb, 0x7fffffff); };
  auto dsA = rsA_of(dt), dsB = rsB_of(dt);
  // one K-step's 16 pieces of the cursor into LDS buffer `buf`; then advance the cursor (past the
  // last tile it keeps re-issuing a valid step: those pieces land in a buffer nothing reads again)
  auto dma_piece = [&](int k, uint32_t buf) {
    if (k < 8) {
      const int p = w * 8 + k;
      dma_lds(dsA, buf + p * 1024, vA, p * 8 * g.lda * 2 + dkt * 128);
    } else {
      const int p = w * 8 + (k - 8);
      dma_lds(dsB, buf + B_OFF + p * 1024, vB, b_piece_row(p) * g.ldb * 2 + dkt * 128);
    }
  };
  auto dma_advance = [&]() {
    if (++dkt == nk) {
      dkt = 0;
      if (dt + per < end) {
        dt += per;
        dsA = rsA_of(dt);
        dsB = rsB_of(dt);
      }
    }
  };
  const bool has_bias = EPI == EPI_STORE && g.bias != nullptr;
  const auto rsBias = rsrc(g.bias, g.N * 2);   // out-of-range lanes read 0
  auto dma_bias = [&](int tt) {
    if (has_bias) dma_lds(rsBias, lds0 + BIAS_OFF + w * 1024, lane * 16, (tt % ntn) * BN * 2);
  };

  // ---- prologue: K-steps 0 and 1 (buffers 0, 1); R0 of K-step 0 (the first K-step DMAs the bias)
#pragma unroll
  for (int k = 0; k < 16; ++k) dma_piece(k, lds0);
  dma_advance();
#pragma unroll
  for (int k = 0; k < 16; ++k) dma_piece(k, lds0 + BUF);
  dma_advance();
  wait_vm<16>();
  barrier();

  i32x4 fa0[8], fb0[8], fa1[8], fb1[8];
  f32x4 acc[8][8];
  static_for<0, 8>([&](auto ic) {
    constexpr int i = decltype(ic)::value;
    lds_rd<i * 2048>(fb0[i], rB0);
  });
  static_for<0, 8>([&](auto ic) {
    constexpr int i = decltype(ic)::value;
    lds_rd<i * 2048>(fa0[i], rA0);
  });
  wait_lgkm0();

  // EPI_ADD reads the residual C tile in the epilogue (a row = this wave's 16 output rows x 128
  // columns, 4 loads per lane).  Rows 0..2 are loaded during the tile's last K-step, before its DMA
  // pieces, so that step's barrier-2 wait retires them; each row's registers are refilled with row
  // + 3 as the epilogue consumes it, and rows 3..7 are waited for by count -- two rows of epilogue
  // work cover each load.  The loads are asm (load16): issued through the builtin, hipcc waited
  // vmcnt(0) at their first use, i.e. for every DMA piece of the next tile in flight.
  i32x4 cpre[3][4];
  const int vc = ((wm * 128 + li) * g.ldc + wn * 128 + 8 * lq) * 2;
  auto c_load = [&](__amdgpu_buffer_rsrc_t rc, int r, i32x4 (&dst)[4]) {
#pragma unroll
    for (int j = 0; j < 4; ++j) load16(dst[j], rc, vc, (r * 16 * g.ldc + 32 * j) * 2);
  };

  int kt = 0;
  uint32_t cur = 0;          // byte offset of the current K-step's buffer (0 / BUF)
  bool after_epi = false;    // the previous step ran an epilogue (its stores sit in the vm queue)
  int m0 = (t / ntn) * BM, n0 = (t % ntn) * BN;

  while (true) {
    const uint32_t nxt = cur ^ BUF;
    // ---------------- phase 0: MFMAs on R0; read R1 (cur); barrier; DMA K-step s + 2 into cur
    auto phase0 = [&](auto first_c) {
      constexpr bool first = decltype(first_c)::value;
      const uint32_t b1 = rB1 + cur, a1 = rA1 + cur;
      static_for<0, 64>([&](auto ic) {
        constexpr int i = decltype(ic)::value, mi = i >> 3, ni = i & 7;
        if constexpr (first) mfma_zero(acc[mi][ni], fb0[ni], fa0[mi]);
        else mfma_acc(acc[mi][ni], fb0[ni], fa0[mi]);
        if constexpr (i < 8) lds_rd<i * 2048>(fb1[i], b1);
        else if constexpr (i < 16) lds_rd<(i - 8) * 2048>(fa1[i - 8], a1);
        else if constexpr (i == 19) {
          wait_lgkm0();
          barrier();
          if (kt == 0) dma_bias(t);   // the tile's bias, older than every later counted wait
          if constexpr (EPI == EPI_ADD) {
            const auto rc = rsrc(g.c + (size_t)m0 * g.ldc + n0, 0x7fffffff);
            prefetch3(cpre, kt == nk - 1, rc, vc, 0, 16 * g.ldc * 2, 2 * 16 * g.ldc * 2);
          }
        }
        static_for<0, 16>([&](auto kc) {
          constexpr int k = decltype(kc)::value;
          if constexpr (SC::dma_slot(k) == i) dma_piece(k, lds0 + cur);
        });
      });
    };
    if (kt == 0) phase0(std::true_type{});
    else phase0(std::false_type{});
    // ---------------- phase 1: MFMAs on R1; K-step s + 1 landed (barrier 2); read R0 from nxt
    const uint32_t b0n = rB0 + nxt, a0n = rA0 + nxt;
    static_for<0, 64>([&](auto ic) {
      constexpr int i = decltype(ic)::value, mi = i >> 3, ni = i & 7;
      mfma_acc(acc[mi][ni], fb1[ni], fa1[mi]);
      if constexpr (i == B2I) {
        // K-step s + 1 was issued one K-step ago; younger: the pieces of this step issued so far
        // (+ the epilogue's stores / loads and the bias piece when the previous step ended a tile)
        constexpr int after = NB2 + 1 + (EPI == EPI_ADD ? 52 : 32);   // ADD: 20 loads + 32 stores after the step
        if (after_epi) wait_vm<(after > 63 ? 63 : after)>();
        else wait_vm<NB2>();
        barrier();
      } else if constexpr (i > B2I && i <= B2I + 31 && ((i - B2I) & 1) == 1) {
        constexpr int k = (i - B2I - 1) >> 1;
        if constexpr (k < 8) lds_rd<k * 2048>(fb0[k], b0n);
        else lds_rd<(k - 8) * 2048>(fa0[k - 8], a0n);
      }
      static_for<0, 16>([&](auto kc) {
        constexpr int k = decltype(kc)::value;
        if constexpr (SC::dma_slot(k) == 64 + i) dma_piece(k, lds0 + cur);
      });
    });
    wait_lgkm0();
    dma_advance();
    after_epi = false;
    cur = nxt;
    if (++kt < nk) continue;

    // ---------------- epilogue of tile t (the next tile's K-steps 0 and 1 are landing meanwhile)
    // the asm MFMAs' results: wait out the last ones' passes before any accumulator read (hipcc
    // does not know the asm statements are MFMAs); then one row of tiles at a time, each behind a
    // fence that also orders it after the previous row's stores (live copies stay at 32 VGPRs)
    asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory");
    if constexpr (EPI == EPI_ADD) {
      // rows 0..2 landed (retired by the last K-step's barrier-2 wait): no use may move above it
#pragma unroll
      for (int r = 0; r < 3; ++r) pin_v4(cpre[r]);
    }
    {
      const auto rc = rsrc(g.c + (size_t)m0 * g.ldc + n0, 0x7fffffff);
      bf16x8 b8[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        b8[j] = bf16x8{};
        if (has_bias)
          b8[j] = *reinterpret_cast<const bf16x8*>(smem + BIAS_OFF + w * 1024 + (wn * 128 + 32 * j + 8 * lq) * 2);
      }
      static_for<0, 8>([&](auto mic) {
        constexpr int mi = decltype(mic)::value;
        asm volatile("" : "+a"(acc[mi][0]), "+a"(acc[mi][1]), "+a"(acc[mi][2]), "+a"(acc[mi][3]),
                     "+a"(acc[mi][4]), "+a"(acc[mi][5]), "+a"(acc[mi][6]), "+a"(acc[mi][7]) :: "memory");
        if constexpr (EPI == EPI_ADD && mi >= 3) {
          // row mi was loaded after row mi - 3's stores; younger since: the stores of rows mi-2,
          // mi-1 and the loads of rows mi+1, mi+2 (those that exist)
          wait_vm_pin<8 + 4 * ((mi + 1 <= 7) + (mi + 2 <= 7))>(cpre[mi % 3]);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const f32x4 lo = acc[mi][2 * j], hi = acc[mi][2 * j + 1];
          const float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
          const bf16x8 add8 = EPI == EPI_ADD ? __builtin_bit_cast(bf16x8, cpre[mi % 3][j]) : b8[j];
          i32x4 o;
#pragma unroll
          for (int e = 0; e < 4; ++e)   // fp32 sum, one v_cvt_pk_bf16_f32 per pair
            o[e] = __builtin_bit_cast(int, __builtin_convertvector(
                       f32x2{v[2 * e] + (float)add8[2 * e], v[2 * e + 1] + (float)add8[2 * e + 1]}, bf16x2));
          store16(o, rc, vc, (mi * 16 * g.ldc + 32 * j) * 2);
        }
        if constexpr (EPI == EPI_ADD && mi + 3 <= 7) c_load(rc, mi + 3, cpre[mi % 3]);
      });
    }
    t += per;
    if (t >= end) break;
    kt = 0;
    after_epi = true;
    m0 = (t / ntn) * BM;
    n0 = (t % ntn) * BN;
  }
  // nothing may still write this workgroup's LDS when it ends (the cursor's trailing pieces)
  wait_vm<0>();
}

int num_cus() {
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

}  // namespace

// DTD_GEMM_W4_SCHED: the schedule variant at load (A/B runs); dtd_gemm_w4_set_sched at run time
static int g_sched = [] {
  const char* e = getenv("DTD_GEMM_W4_SCHED");
  const int i = e ? atoi(e) : SCHED_DEFAULT;
  return i >= 0 && i < SCHED_COUNT ? i : SCHED_DEFAULT;
}();
DTD_EXPORT int dtd_gemm_w4_set_sched(int i) {
  if (i < 0 || i >= SCHED_COUNT) return (int)hipErrorInvalidValue;
  g_sched = i;
  return 0;
}

DTD_EXPORT int dtd_gemm_w4_supported(int M, int N, int K) {
  return M > 0 && N > 0 && K >= 2 * BK && M % BM == 0 && N % BN == 0 && K % BK == 0;
}

// epi: 0 = store (+ bias), 3 = add into c (no bias)
DTD_EXPORT int dtd_gemm_w4(int epi, const void* a, int lda, const void* b, int ldb, void* c, int ldc, const void* bias,
                           int M, int N, int K, hipStream_t s) {
  if (!dtd_gemm_w4_supported(M, N, K)) return (int)hipErrorInvalidValue;
  if ((lda | ldb | ldc) % 8 || lda < K || ldb < K || ldc < N) return (int)hipErrorInvalidValue;
  if (((uintptr_t)a | (uintptr_t)b | (uintptr_t)c | (uintptr_t)bias) % 16) return (int)hipErrorInvalidValue;
  // every byte offset the kernel forms inside one A / B panel or C tile must fit 31 bits
  if ((long long)BM * lda * 2 >= 0x7fffffffLL || (long long)BN * ldb * 2 >= 0x7fffffffLL ||
      (long long)BM * ldc * 2 >= 0x7fffffffLL)
    return (int)hipErrorInvalidValue;
  if (epi != EPI_STORE && epi != EPI_ADD) return (int)hipErrorInvalidValue;
  if (epi == EPI_ADD && bias) return (int)hipErrorInvalidValue;
  W4Args g{(const bf16*)a, (const bf16*)b, (bf16*)c, (const bf16*)bias, M, N, K, lda, ldb, ldc};
  const int ntiles = (M / BM) * (N / BN);
  const int cus = num_cus() / 8 * 8;
  const int nwg = ntiles >= cus ? cus : (ntiles + 7) / 8 * 8;
#define DTD_W4_LAUNCH(i, a0, st, b2)                                                                         \
  case i:                                                                                                     \
    if (epi == EPI_STORE)                                                                                     \
      hipLaunchKernelGGL((gemm_w4_kernel<EPI_STORE, Sched<a0, st, b2>>), dim3(nwg), dim3(256), 0, s, g);     \
    else                                                                                                      \
      hipLaunchKernelGGL((gemm_w4_kernel<EPI_ADD, Sched<a0, st, b2>>), dim3(nwg), dim3(256), 0, s, g);       \
    break;
  switch (g_sched) {
    DTD_W4_SCHEDS(DTD_W4_LAUNCH)
    default: return (int)hipErrorInvalidValue;
  }
#undef DTD_W4_LAUNCH
  DTD_LAUNCH_CHECK();
}
