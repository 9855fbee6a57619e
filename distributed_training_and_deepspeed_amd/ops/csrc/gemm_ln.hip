// Projection GEMM + bias + hidden dropout + residual + LayerNorm in ONE kernel for gfx950: the
// output sublayer of a post-LN transformer block (BERT's attention-output and FFN-output
// projections; HF BertSelfOutput / BertOutput, SURVEY.md K1/K4, reference
// data_parallel_training.py:30-31 via transformers, model/transformer.py:95-104):
//
//   y    = bf16(X[M, K] . W[NH, K]^T + b)        the Linear's output, rounded once (as stored by
//                                                hipBLASLt on the unfused path)
//   z    = r + dropout(y)                         hidden dropout, the counter-RNG law of norm.hip
//   out  = (z - mean) * rstd * gamma + beta       LayerNorm over the NH = 768 features of a row
//
// The unfused path writes y to HBM and the LayerNorm kernel reads it back with the residual
// (ln_fwd_wave: 113 us per call at 131k x 768, 24 calls per BERT-base step).  Here a workgroup owns
// WHOLE rows -- 128 tokens x all 768 features -- so the row statistics close inside the kernel and
// y never leaves the chip.
//
// Main loop: 4 waves, one per SIMD (512 registers each); wave w owns features [192w, 192w + 192)
// of the workgroup's 128 tokens: 4 x 6 tiles of v_mfma_f32_32x32x16_bf16, 384 fp32 accumulators.
// The tile is computed transposed (C^T = W . X^T: the weight rows are the MFMA A operand), so a
// lane holds ONE token and 16 of its features per tile (crow layout) -- a row's statistics are
// in-lane adds, one lane^32 exchange and a 4-wave combine through LDS.
// K-steps of 32: the 768 x 32 weight panel (48 KiB, each wave DMAs and reads only its own 192
// rows) double-buffered, the 128 x 32 activation panel (8 KiB, all waves read all rows) in a
// 3-deep ring so its HBM latency has two K-steps to land.  Both arrive by 16-byte LDS-DMA
// (buffer_load_dwordx4 ... lds) into 64-byte rows whose 16-byte chunks are XOR-swizzled by
// (row >> 2) & 3 (the source address carries the swizzle; every ds_read_b128 fragment read of 32
// rows at one chunk is bank-conflict free).  One barrier per K-step; the next K-step's first
// fragments are read right after it, under the current K-step's second half of MFMAs.
#include <stdlib.h>
#include <type_traits>

// Experimental (DTD_BUILD_EXPERIMENTAL=1, ops/build.py): slower than the hipBLASLt GEMM + LayerNorm
// kernel pair it replaces (profiles/r4_s9_results.jsonl, r5 session 9 with the asm LDS-DMA), so the
// default library omits it and ops/gemm.py linear_ln_supported() reports it unavailable.
#if DTD_GEMM_LN_BUILD
#include "common.h"

using namespace dtd;

typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace {

typedef __attribute__((address_space(3))) void lds_void;

constexpr int NH = 768, BM = 128, BK = 32, NWAVE = 4;
constexpr int FPW = NH / NWAVE;             // 192 features per wave
constexpr int FB = FPW / 32, TB = BM / 32;  // 6 feature tiles x 4 token tiles per wave
constexpr int ROWB = BK * 2;                // 64-byte LDS rows
constexpr int W_STAGE = NH * ROWB;          // 48 KiB
constexpr int X_STAGE = BM * ROWB;          // 8 KiB
constexpr int X_OFF = 2 * W_STAGE;
constexpr int LDS_BYTES = X_OFF + 3 * X_STAGE;   // 120 KiB
constexpr int W_DMA = FPW / 16, X_DMA = 32 / 16;   // 16-row DMA wave-instructions per K-step per wave

struct GemmLnArgs {
  const bf16* x; const bf16* w; const bf16* bias; const bf16* r; const bf16* gamma; const bf16* beta;
  bf16* out; bf16* z; float* mean; float* rstd;
  int M, K, ldx, ldw, ldr, ldo;
  float eps, p; const uint64_t* rng; uint32_t sid;
};

// 384 accumulators exceed the 256-entry accumulator file: the builtin MFMA made hipcc cycle tiles
// through a few AGPRs with spills.  The MFMAs are issued as asm with each tile pinned to a register
// file -- feature tiles 0-3 in AGPRs ("+a", 256), tiles 4-5 in arch VGPRs ("+v", 128).  The A / B
// operands are LDS reads (no VALU-write hazard).  hipcc takes an asm statement as complete at its
// end: acc_settle() waits the last results out before anything but an MFMA chain reads them.
template <int F>
__device__ __forceinline__ void mfma_acc(f32x16& acc, bf16x8 a, bf16x8 b) {
  if constexpr (F < 4) asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
  else asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b));
}
template <int I, int N, class Fn>
__device__ __forceinline__ void static_for(Fn&& fn) {
  if constexpr (I < N) {
    fn(std::integral_constant<int, I>{});
    static_for<I + 1, N>(fn);
  }
}

// keep a tile's values in its register file (the epilogue rewrites the accumulators in place)
template <int F>
__device__ __forceinline__ void pin(f32x16& acc) {
  if constexpr (F < 4) asm volatile("" : "+a"(acc));
  else asm volatile("" : "+v"(acc));
}
__device__ __forceinline__ int crow(int i, int h) { return (i & 3) + 8 * (i >> 2) + 4 * h; }

// raw workgroup barrier that the compiler also treats as a memory barrier (LDS-DMA may stay in
// flight across it; the counted vmcnt waits retire it)
__device__ __forceinline__ void bar() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t uniform_rsrc(const void* p) {
  const uint64_t a = (uint64_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), (short)0, 0x7fffffff, 0x00020000);
}

__device__ __forceinline__ float xhalf_sum(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

__device__ __forceinline__ float bf16_round(float v) { return (float)(bf16)v; }

__device__ __forceinline__ bf16x4 cvt4(float a, float b, float c, float d) {
  typedef float f32x2_t __attribute__((ext_vector_type(2)));
  const bf16x2 lo = __builtin_convertvector(f32x2_t{a, b}, bf16x2);
  const bf16x2 hi = __builtin_convertvector(f32x2_t{c, d}, bf16x2);
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3);
}

// PIPE = 0: per K-step, DMA issue and fragment reads up front, MFMAs, barrier (simple form).
// PIPE = 1: the memory instructions ride in the MFMA gaps (sched_barrier-pinned): the second
// half-step's fragments are read under the first half's MFMAs, and the barrier sits after the
// first 12 MFMAs of the second half, so the next K-step's first fragments and the DMA of the
// panels two steps ahead issue under its last 12 -- the matrix pipe never drains at the barrier.
template <bool DROP, bool BIAS, bool STORE_Z, int PIPE>
__global__ void __launch_bounds__(256, 1) gemm_ln_kernel(GemmLnArgs g) {
  __shared__ __attribute__((aligned(1024))) char smem[LDS_BYTES];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int m0 = blockIdx.x * BM;
  const int nk = g.K / BK;

  // ---- LDS-DMA map: a wave-instruction fills 16 rows; lane L -> row r0 + L/4, slot L%4 <- global
  //      chunk (L%4) ^ swz(row), swz(row) = (row >> 2) & 3 = (L >> 4) & 3 (r0 is a multiple of 16)
  const int drow = lane >> 2, dch = (lane & 3) ^ ((lane >> 4) & 3);
  const int vw = (drow * g.ldw + dch * 8) * 2, vx = (drow * g.ldx + dch * 8) * 2;
  const auto rw = uniform_rsrc(g.w + (size_t)w * FPW * g.ldw);
  const auto rx = uniform_rsrc(g.x + (size_t)(m0 + w * 32) * g.ldx);
  const int sw16 = 16 * g.ldw * 2, sx16 = 16 * g.ldx * 2;
  char* const wl = smem + w * FPW * ROWB;              // this wave's weight rows (+ stage * W_STAGE)
  char* const xl = smem + X_OFF + w * 32 * ROWB;       // the activation rows this wave stages
  auto dma_w = [&](int kt, int s) {
#pragma unroll
    for (int j = 0; j < W_DMA; ++j)
      dma16(rw, wl + s * W_STAGE + j * 16 * ROWB, vw, j * sw16 + kt * ROWB);
  };
  auto dma_x = [&](int kt, int s) {
#pragma unroll
    for (int j = 0; j < X_DMA; ++j)
      dma16(rx, xl + s * X_STAGE + j * 16 * ROWB, vx, j * sx16 + kt * ROWB);
  };

  // ---- fragment reads: lane reads row (lane & 31) of a 32-row tile, 16-byte chunk 2 ks + (lane >> 5)
  const int fr = lane & 31, hh = lane >> 5, sz = (fr >> 2) & 3;
  const int c0 = ((0 + hh) ^ sz) * 16, c1 = ((2 + hh) ^ sz) * 16;
  const char* const wfr = smem + (w * FPW + fr) * ROWB;
  const char* const xfr = smem + X_OFF + fr * ROWB;
  bf16x8 wa[FB], xa[TB], wb[FB], xb[TB];
  auto read_frags = [&](int kt, int c, bf16x8 (&wf)[FB], bf16x8 (&xf)[TB]) {
    const char* wp = wfr + (kt & 1) * W_STAGE + c;
    const char* xp = xfr + (kt % 3) * X_STAGE + c;
#pragma unroll
    for (int t = 0; t < TB; ++t) xf[t] = *reinterpret_cast<const bf16x8*>(xp + t * 32 * ROWB);
#pragma unroll
    for (int f = 0; f < FB; ++f) wf[f] = *reinterpret_cast<const bf16x8*>(wp + f * 32 * ROWB);
  };

  f32x16 acc[TB][FB];
#pragma unroll
  for (int t = 0; t < TB; ++t)
#pragma unroll
    for (int f = 0; f < FB; ++f) acc[t][f] = f32x16{};

  auto mfma_step = [&](const bf16x8 (&wf)[FB], const bf16x8 (&xf)[TB]) {
#pragma unroll
    for (int t = 0; t < TB; ++t) {
      mfma_acc<0>(acc[t][0], wf[0], xf[t]);
      mfma_acc<1>(acc[t][1], wf[1], xf[t]);
      mfma_acc<2>(acc[t][2], wf[2], xf[t]);
      mfma_acc<3>(acc[t][3], wf[3], xf[t]);
      mfma_acc<4>(acc[t][4], wf[4], xf[t]);
      mfma_acc<5>(acc[t][5], wf[5], xf[t]);
    }
  };
  if constexpr (PIPE == 2) {
    // The weight rows are private to the wave: their MFMA A fragments come straight from global
    // memory (L2) into registers -- lane l reads row 32 f + (l & 31), 8 k-values at 8 (l >> 5) --
    // with no LDS round trip and no LDS-DMA (whose issue cost, 60-185 cycles per 1 KiB piece inside
    // an MFMA stream, bounded the PIPE 0/1 forms at ~3.7k cycles per K-step).  Only the shared
    // activation panel goes through LDS (3-deep ring, 2 DMA pieces per wave per K-step).  The half
    // K-step's weight fragments load one half-step ahead: wb under the ks0 MFMAs, wa (next K-step)
    // under the first ks1 MFMAs.
    const int vwf = ((lane & 31) * g.ldw + (lane >> 5) * 8) * 2;
    const int swf = 32 * g.ldw * 2;   // bytes per 32 weight rows
    auto load_w = [&](int j, int kt2, int ks, bf16x8 (&wf)[FB]) {
      wf[j] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rw, vwf, j * swf + kt2 * ROWB + ks * 32, 0));
    };
    auto read_x = [&](int j, int kt2, int c, bf16x8 (&xf)[TB]) {
      xf[j] = *reinterpret_cast<const bf16x8*>(xfr + (kt2 % 3) * X_STAGE + c + j * 32 * ROWB);
    };
    auto dma_x_one = [&](int j, int kx, int sx) {
      dma16(rx, xl + sx * X_STAGE + j * 16 * ROWB, vx, j * sx16 + kx * ROWB);
    };
    // prologue: X(0), X(1), X(2) and the first half-step's weight fragments in flight
    dma_x(0, 0);
    dma_x(min(1, nk - 1), 1);
    dma_x(min(2, nk - 1), 2);
#pragma unroll
    for (int j = 0; j < FB; ++j) load_w(j, 0, 0, wa);
    asm volatile("s_waitcnt vmcnt(10)" ::: "memory");   // X(0) landed (own rows)
    bar();
#pragma unroll
    for (int j = 0; j < TB; ++j) read_x(j, 0, c0, xa);
    for (int kt = 0; kt < nk; ++kt) {
      const int kn = min(kt + 1, nk - 1), kx = min(kt + 3, nk - 1), sx = kt % 3;
      static_for<0, TB * FB>([&](auto jc) {
        constexpr int j = decltype(jc)::value, t = j / FB, f = j % FB;
        mfma_acc<f>(acc[t][f], wa[f], xa[t]);
        if constexpr (j < FB) load_w(j, kt, 1, wb);
        else if constexpr (j < FB + TB) read_x(j - FB, kt, c1, xb);
        __builtin_amdgcn_sched_barrier(0);
      });
      static_for<0, TB * FB>([&](auto jc) {
        constexpr int j = decltype(jc)::value, t = j / FB, f = j % FB;
        if constexpr (j == TB * FB / 2) {
          // B(kt): X(kt+1) landed for every wave -- at most the 20 youngest vector-memory ops may
          // still fly (steady state: wa(kt+1) 6, wb(kt) 6, X(kt+2) 2, wa(kt) 6; X(kt+1) is older)
          // -- and every wave has read stage kt out
          asm volatile("s_waitcnt vmcnt(20) lgkmcnt(0)" ::: "memory");
          bar();
        }
        mfma_acc<f>(acc[t][f], wb[f], xb[t]);
        // gaps 0-5: the next K-step's first-half weight fragments (a half-step of flight before
        // their MFMAs); after the barrier: its first activation fragments, then the DMA of X(kt+3)
        if constexpr (j < FB) load_w(j, kn, 0, wa);
        else if constexpr (j >= TB * FB / 2 && j < TB * FB / 2 + TB) read_x(j - TB * FB / 2, kt + 1, c0, xa);
        else if constexpr (j >= TB * FB / 2 + TB && j < TB * FB / 2 + TB + X_DMA)
          dma_x_one(j - TB * FB / 2 - TB, kx, sx);
        __builtin_amdgcn_sched_barrier(0);
      });
    }
  } else {
  // prologue: W(0), X(0), X(1) issued; W(0) and X(0) landed
  dma_w(0, 0);
  dma_x(0, 0);
  dma_x(nk > 1 ? 1 : 0, 1);
  asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  bar();
  read_frags(0, c0, wa, xa);

  if constexpr (PIPE == 1) {
    // one 16-row DMA instruction / one fragment read, by index
    auto dma_one = [&](int j, int kw, int sw, int kx, int sx) {
      if (j < W_DMA)
        dma16(rw, wl + sw * W_STAGE + j * 16 * ROWB, vw, j * sw16 + kw * ROWB);
      else
        dma16(rx, xl + sx * X_STAGE + (j - W_DMA) * 16 * ROWB, vx, (j - W_DMA) * sx16 + kx * ROWB);
    };
    auto read_one = [&](int j, int kt2, int c, bf16x8 (&wf)[FB], bf16x8 (&xf)[TB]) {
      if (j < TB) xf[j] = *reinterpret_cast<const bf16x8*>(xfr + (kt2 % 3) * X_STAGE + c + j * 32 * ROWB);
      else wf[j - TB] = *reinterpret_cast<const bf16x8*>(wfr + (kt2 & 1) * W_STAGE + c + (j - TB) * 32 * ROWB);
    };
    // the panels "issued after barrier B(-1)": W(1), X(2)
    dma_w(min(1, nk - 1), 1);
    dma_x(min(2, nk - 1), 2);
    for (int kt = 0; kt < nk; ++kt) {
      const int kw = min(kt + 2, nk - 1), kx = min(kt + 3, nk - 1), sw = kt & 1, sx = kt % 3;
      // first half-step: MFMAs on (wa, xa); the second half's 10 fragment reads in gaps 0-9
      static_for<0, TB * FB>([&](auto jc) {
        constexpr int j = decltype(jc)::value, t = j / FB, f = j % FB;
        mfma_acc<f>(acc[t][f], wa[f], xa[t]);
        if constexpr (j < TB + FB) read_one(j, kt, c1, wb, xb);
        __builtin_amdgcn_sched_barrier(0);
      });
      // second half-step: 12 MFMAs, barrier B(kt) (W(kt+1), X(kt+1) landed; stage kt read out),
      // 12 MFMAs with the next K-step's first fragments and the DMA of W(kt+2), X(kt+3) in the gaps
      static_for<0, TB * FB>([&](auto jc) {
        constexpr int j = decltype(jc)::value, t = j / FB, f = j % FB;
        if constexpr (j == TB * FB / 2) {
          asm volatile("s_waitcnt vmcnt(2) lgkmcnt(0)" ::: "memory");
          bar();
        }
        mfma_acc<f>(acc[t][f], wb[f], xb[t]);
        if constexpr (j >= TB * FB / 2) {
          constexpr int g0 = 2 * (j - TB * FB / 2);   // memory ops g0, g0 + 1 of 24
#pragma unroll
          for (int u = g0; u < g0 + 2; ++u) {
            if (u < TB + FB) read_one(u, kt + 1, c0, wa, xa);
            else dma_one(u - (TB + FB), kw, sw, kx, sx);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      });
    }
  } else
  for (int kt = 0; kt < nk; ++kt) {
    // the next weight panel and the activation panel two K-steps ahead (clamped re-loads of the
    // last panel keep the issue and the counted waits unconditional; their stages are not read)
    dma_w(min(kt + 1, nk - 1), (kt + 1) & 1);
    dma_x(min(kt + 2, nk - 1), (kt + 2) % 3);
    read_frags(kt, c1, wb, xb);
    mfma_step(wa, xa);
    mfma_step(wb, xb);
    // W(kt+1) and X(kt+1) landed (only X(kt+2) may still fly); every wave done reading stage kt
    asm volatile("s_waitcnt vmcnt(2) lgkmcnt(0)" ::: "memory");
    bar();
    if (kt + 1 < nk) read_frags(kt + 1, c0, wa, xa);
  }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  // acc_settle: 16 wait states for the last MFMAs' results (8-pass XDL needs 12 before a VALU or
  // v_accvgpr_read touches them), then pin every tile in its file so no read is hoisted above
  // (scheduling barriers on both sides: the machine scheduler otherwise hoists the epilogue's
  // v_accvgpr_read of the last tiles above the wait)
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_nop 15" ::: "memory");
#pragma unroll
  for (int t = 0; t < TB; ++t) {
    asm volatile("" : "+a"(acc[t][0]), "+a"(acc[t][1]), "+a"(acc[t][2]), "+a"(acc[t][3]));
    asm volatile("" : "+v"(acc[t][4]), "+v"(acc[t][5]));
  }
  __builtin_amdgcn_sched_barrier(0);
  bar();

  // ---- epilogue, 64 tokens at a time: y = bf16(acc + b) as a row-major [64][768] image in LDS
  //      (row pitch 1552 B: the 32 token rows of one 8-byte accumulator store land 4 banks apart),
  //      then the LayerNorm of norm.hip's ln_fwd_wave with y read from LDS instead of HBM: two rows
  //      per wave-instruction, lane sub of a row holding features 8 (32 c + sub) .. +7 (c < 3), so
  //      the residual loads and output stores are whole 512-byte row segments and the dropout
  //      element index, the keep law and the two-pass statistics are ln_fwd_wave's.
  constexpr int YP = NH * 2 + 16;
  const DropoutRng rg(g.rng, g.sid);
  const uint32_t thr = keep_threshold(g.p);
  const float dscale = DROP ? 1.f / (1.f - g.p) : 1.f;
  const int sub = lane & 31, rsel = lane >> 5;
  bf16x8 gm8[3], bt8[3];
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    gm8[c] = *reinterpret_cast<const bf16x8*>(g.gamma + (c * 32 + sub) * 8);
    bt8[c] = *reinterpret_cast<const bf16x8*>(g.beta + (c * 32 + sub) * 8);
  }
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    // accumulators of token tiles 2 half, 2 half + 1 -> LDS (bias added in fp32, one rounding)
#pragma unroll
    for (int tt = 0; tt < 2; ++tt) {
      const int t = 2 * half + tt;
      char* yrow = smem + (tt * 32 + fr) * YP;
#pragma unroll
      for (int f = 0; f < FB; ++f)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int i = 4 * q, col = w * FPW + f * 32 + 4 * hh + 8 * q;
          const bf16x4 b4 = BIAS ? *reinterpret_cast<const bf16x4*>(g.bias + col) : bf16x4{};
          *reinterpret_cast<bf16x4*>(yrow + col * 2) =
              cvt4(acc[t][f][i] + (float)b4[0], acc[t][f][i + 1] + (float)b4[1], acc[t][f][i + 2] + (float)b4[2],
                   acc[t][f][i + 3] + (float)b4[3]);
        }
    }
    bar();
    // LayerNorm of the 64 rows: wave w takes rows 16 w .. 16 w + 15, two per step.  One wave per
    // SIMD hides no memory latency by itself: the residual rows of the next step are loaded while
    // this step computes.
    auto load_r = [&](int rp, bf16x8 (&rv)[3]) {
      const int row = m0 + half * 64 + w * 16 + 2 * rp + rsel;
#pragma unroll
      for (int c = 0; c < 3; ++c)
        rv[c] = *reinterpret_cast<const bf16x8*>(g.r + (size_t)row * g.ldr + (c * 32 + sub) * 8);
    };
    bf16x8 rnext[3];
    load_r(0, rnext);
#pragma unroll 1
    for (int rp = 0; rp < 8; ++rp) {
      const int lr = w * 16 + 2 * rp + rsel;          // row within the half
      const int row = m0 + half * 64 + lr;
      const size_t base = (size_t)row * NH;
      bf16x8 rcur[3];
#pragma unroll
      for (int c = 0; c < 3; ++c) rcur[c] = rnext[c];
      if (rp + 1 < 8) load_r(rp + 1, rnext);
      float z[24];
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const int col = (c * 32 + sub) * 8;
        const bf16x8 y8 = *reinterpret_cast<const bf16x8*>(smem + lr * YP + col * 2);
        float rr[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) rr[j] = (float)rcur[c][j];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float y = (float)y8[j];
          if constexpr (DROP) {
            const uint32_t e = (uint32_t)(base + col + j);
            const uint32_t bits = rg.bits(e >> 1);
            const uint32_t h16 = (e & 1) ? (bits >> 16) : (bits & 0xffffu);
            y *= h16 >= thr ? dscale : 0.f;
          }
          z[8 * c + j] = y + rr[j];
        }
        if constexpr (STORE_Z) vstore<bf16, 8>(g.z + (size_t)row * g.ldo + col, z + 8 * c);
      }
      float s = 0.f;
#pragma unroll
      for (int i = 0; i < 24; ++i) s += z[i];
#pragma unroll
      for (int o = 16; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
      const float mu = s / NH;
      float v = 0.f;
#pragma unroll
      for (int i = 0; i < 24; ++i) { const float d = z[i] - mu; v += d * d; }
#pragma unroll
      for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
      const float rs = rsqrtf(v / NH + g.eps);
      if (sub == 0) { g.mean[row] = mu; g.rstd[row] = rs; }
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const int col = (c * 32 + sub) * 8;
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = (z[8 * c + j] - mu) * rs * (float)gm8[c][j] + (float)bt8[c][j];
        vstore<bf16, 8>(g.out + (size_t)row * g.ldo + col, o);
      }
    }
    bar();
  }
}

}  // namespace

// out = LN(r + dropout(bf16(x . w^T + bias))) over rows of 768 features; mean / rstd per row
// (fp32), z (bf16, optional).  x [M, K] (ldx), w [768, K] (ldw), r / out / z [M, 768] (ldr / ldo).
// Returns hipErrorInvalidValue for shapes the kernel does not take (callers fall back).
DTD_EXPORT int dtd_gemm_ln_supported(int M, int N, int K, int ldx, int ldw, int ldr, int ldo) {
  return N == NH && M > 0 && M % BM == 0 && K >= BK && K % BK == 0 && ldx % 8 == 0 && ldw % 8 == 0 &&
         ldr % 4 == 0 && ldo % 4 == 0 && (long long)M * NH / 2 < (1LL << 32) &&
         (long long)M * ldx * 2 < 0x7fffffffLL && (long long)NH * ldw * 2 < 0x7fffffffLL;
}

DTD_EXPORT int dtd_gemm_ln(const void* x, const void* w, const void* bias, const void* r, const void* gamma,
                           const void* beta, void* out, void* z, float* mean, float* rstd, int M, int N, int K,
                           int ldx, int ldw, int ldr, int ldo, float eps, float p, const uint64_t* rng,
                           uint32_t sid, hipStream_t s) {
  if (!dtd_gemm_ln_supported(M, N, K, ldx, ldw, ldr, ldo)) return (int)hipErrorInvalidValue;
  if (((uintptr_t)x | (uintptr_t)w) & 15) return (int)hipErrorInvalidValue;
  if ((p > 0.f && !rng) || !r || !gamma || !beta || !out || !mean || !rstd) return (int)hipErrorInvalidValue;
  GemmLnArgs a{(const bf16*)x, (const bf16*)w, (const bf16*)bias, (const bf16*)r, (const bf16*)gamma,
               (const bf16*)beta, (bf16*)out, (bf16*)z, mean, rstd, M, K, ldx, ldw, ldr, ldo, eps, p, rng, sid};
  const dim3 grid(M / BM), block(256);
  const bool d = p > 0.f, b = bias != nullptr, zz = z != nullptr;
  static const int pipe = [] { const char* e = getenv("DTD_GEMM_LN_PIPE"); return e ? atoi(e) : 1; }();
#define DTD_GLN(D, B, Z)                                                                              \
  do {                                                                                                \
    if (pipe == 2) hipLaunchKernelGGL((gemm_ln_kernel<D, B, Z, 2>), grid, block, 0, s, a);           \
    else if (pipe) hipLaunchKernelGGL((gemm_ln_kernel<D, B, Z, 1>), grid, block, 0, s, a);           \
    else hipLaunchKernelGGL((gemm_ln_kernel<D, B, Z, 0>), grid, block, 0, s, a);                     \
  } while (0)
  if (d && b && !zz) DTD_GLN(true, true, false);
  else if (d && b) DTD_GLN(true, true, true);
  else if (!d && b && !zz) DTD_GLN(false, true, false);
  else if (!d && b) DTD_GLN(false, true, true);
  else if (d && !zz) DTD_GLN(true, false, false);
  else if (d) DTD_GLN(true, false, true);
  else if (!zz) DTD_GLN(false, false, false);
  else DTD_GLN(false, false, true);
#undef DTD_GLN
  DTD_LAUNCH_CHECK();
}
#endif  // DTD_GEMM_LN_BUILD
