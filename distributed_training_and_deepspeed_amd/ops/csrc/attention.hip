// Flash-style fused attention (forward + backward) on gfx950 MFMA matrix cores.
//
// Replaces the reference's eager attention (HF BertSelfAttention / OPT / BLOOM: QK^T matmul,
// softmax, dropout, PV matmul, materialising B*H*S*S scores -- SURVEY.md K2/K3/K6/K11,
// reference model/transformer.py:80-86).  Scores never leave registers/LDS.
//
// Instruction: v_mfma_f32_32x32x16_bf16 (wave64).  Fragment maps (cdna_hip_programming.md §3):
//   A: lane l holds A[l&31][8*(l>>5)+j],  B: B[8*(l>>5)+j][l&31],  j = 0..7
//   C/D reg i: col = l&31, row = (i&3) + 8*(i>>2) + 4*(l>>5)
// Forward computes the transposed score tile S^T = K.Q^T so each lane owns ONE query column
// and 32 of its keys in registers: the online-softmax row max/sum is an in-lane reduction plus
// one cross-half exchange (lane ^ 32), and the score accumulator feeds the P.V product
// directly as the MFMA B operand (no LDS round trip for P).  Using an accumulator as an
// operand permutes its k order (element j of half h <-> row 16s + 8(j>>2) + 4h + (j&3)); V is
// staged row-major (16-byte writes) and read in that permuted order with the gfx950 transposing
// LDS read ds_read_b64_tr_b16.  K/V tiles are double-buffered: the next tile's global loads are
// issued before the current tile's MFMAs, one barrier per tile.
//
// Backward = two kernels, neither uses atomics:
//  * dK/dV ("key on the lane"): one workgroup = 4 waves = 128 keys of one (batch, head); each
//    wave keeps its 32 keys' K/V fragments in registers and dK^T/dV^T accumulators for the whole
//    sweep over 64-row query tiles; P is recomputed from the forward LSE; the S and dP
//    accumulators are the B operands of dV^T += dO^T.P and dK^T += Q^T.dS, whose A operands are
//    transposed LDS reads (ds_read_b64_tr_b16) of the row-major Q / dO tiles.
//  * dQ ("query on the lane", mirror of the forward): recomputes S^T and dP^T per key tile and
//    accumulates dQ^T = K^T.dS^T in registers.  Seven MFMA products per tile pair instead of
//    five, but no [B,H,S,D] fp32 atomic traffic (which bounded the first version at ~1.3 TB/s).
//
// Features: causal mask, ALiBi (bias = slope_h * key), attention-probability dropout with the
// counter RNG (mask index ((b*H+h)*S + q)*S + key, regenerated in backward), arbitrary S
// (bounds-masked), head_dim 64 or 128.  q/k/v/o are strided views (row stride `ld`) into the
// fused [B*S, 3*H*D] projection output, so no transpose/copy kernels are needed.
#include <stdio.h>
#include <type_traits>
#include <stdlib.h>
#include <string.h>

#include "common.h"

#ifndef DTD_ATTN_FUSED_BWD
#define DTD_ATTN_FUSED_BWD 0
#endif

using namespace dtd;

typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace {

constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

__device__ __forceinline__ f32x16 mfma32(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ int crow(int i, int h) { return (i & 3) + 8 * (i >> 2) + 4 * h; }

// ds_read_b64_tr_b16: lane 4q+p of each 16-lane group passes the address of row q, columns
// 4p..4p+3 of a 4x16 block; lane i of the group receives column i (rows 0..3).
__device__ __forceinline__ bf16x4 tr_read(const bf16* p) {
  const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p));
  return __builtin_bit_cast(bf16x4, v);
}
__device__ __forceinline__ bf16x8 cat(bf16x4 lo, bf16x4 hi) {
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}
// A operand for (acc-as-B) products: rows = 32 columns of a row-major LDS tile (`col0` + lane),
// k = rows row0 + {0..3, 8..11} (+4 for the upper half-wave) -- the permuted k order of an
// accumulator used as operand (cdna_hip_programming.md §3).
__device__ __forceinline__ bf16x8 tr_operand(const bf16* tile, int stride, int row0, int col0, int lane) {
  const int hh = lane >> 5, g = (lane >> 4) & 1, li = lane & 15;
  const bf16* p = tile + (row0 + 4 * hh + (li >> 2)) * stride + col0 + 16 * g + 4 * (li & 3);
  return cat(tr_read(p), tr_read(p + 8 * stride));
}

// 64-column (D = 64) Q / dO / K tiles of the backward kernels: unpadded 128-byte rows whose
// 16-byte chunk index is XOR-swizzled by swz64(row) (bits 1, 2 and 1^3 of the row).  Both reads of
// such a tile are then bank-conflict free: the row-operand ds_read_b128 (16-lane groups of 16 rows
// at one chunk: distinct (row parity, chunk ^ swz) slots) and the transposed operand read
// ds_read_b64_tr_b16 (4 rows x 2 column blocks per 32-lane half; rows 4k and 4k+2 land in
// different 4-chunk groups).  The padded D + 8 pitch left the transposed reads 2-way conflicted
// (rows r and r + 2 are 72 dwords = 8 banks apart, the second column block's offset) -- 1.6 M
// (dQ) and 3.2 M (dK/dV) conflict cycles per dispatch (profiles/r2_attention_pmc.json).
// swz64 depends on row bits 1..3 only, so blocks starting at a multiple of 16 rows share it.
__device__ __forceinline__ int swz64(int row) {
  return ((row >> 1) & 1) | (((row >> 2) & 1) << 1) | ((((row >> 1) ^ (row >> 3)) & 1) << 2);
}
// element offset of 16-byte chunk `ch` (0..7) of row `row`
__device__ __forceinline__ int swz64_off(int row, int ch) { return row * 64 + 8 * (ch ^ swz64(row)); }
// row operand (ds_read_b128) of the swizzled tile: row row0 + r (row0 % 16 == 0), chunk ch
__device__ __forceinline__ bf16x8 swz_row_read(const bf16* tile, int row0, int r, int ch) {
  return *reinterpret_cast<const bf16x8*>(tile + row0 * 64 + swz64_off(r, ch));
}
// tr_operand on the swizzled tile (row0 % 16 == 0, col0 % 32 == 0)
__device__ __forceinline__ bf16x8 tr_operand_swz(const bf16* tile, int row0, int col0, int lane) {
  const int hh = lane >> 5, g = (lane >> 4) & 1, li = lane & 15;
  const int rl = 4 * hh + (li >> 2);                  // rows rl and rl + 8 of the 16-row block
  const int ch = (col0 >> 3) + 2 * g + ((li >> 1) & 1);
  const int e = 4 * (li & 1);
  const bf16* base = tile + row0 * 64 + e;
  return cat(tr_read(base + swz64_off(rl, ch)), tr_read(base + swz64_off(rl + 8, ch)));
}

// Raw v_exp_f32 (2^x): the softmax arguments are <= 0, so the libm wrapper's denormal
// range handling (extra VALU per element) is not needed -- tiny results flush to 0.
__device__ __forceinline__ float fexp2(float x) { return __builtin_amdgcn_exp2f(x); }
// Dropout as a bit select: all-ones / zero lane mask from bit `b` of `w` (one v_bfe_i32), AND-ed
// into the float's bits -- 2 VALU per element instead of shift/compare/select/multiply; the
// 1/(1-p) rescale is folded into the per-row epilogue.
// The empty asm hides that the mask is 0 / -1: otherwise the compiler rewrites the AND into
// v_and (bit test) + v_cmp + v_cndmask, with an s_nop for the VCC hazard -- 3-4 issues a score.
__device__ __forceinline__ int bit_mask(uint32_t w, int b) {
  int m = __builtin_amdgcn_sbfe((int)w, b, 1);
  asm("" : "+v"(m));
  return m;
}
__device__ __forceinline__ float keep_bits(float v, uint32_t w, int b) {
  return __int_as_float(__float_as_int(v) & bit_mask(w, b));
}

// Lane l <-> lane l^32 combine with v_permlane32_swap (a VALU op; __shfl_xor(x, 32) would be a
// ds_bpermute round trip through the LDS pipe on the softmax critical path).
__device__ __forceinline__ float xhalf_max(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float xhalf_sum(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
// Keep word pre-shifted by 4*hh so the bit of accumulator register i is the compile-time
// constant crow(i, 0): one v_bfe_i32 with inline offsets, no per-register bit-index VGPRs.
__device__ __forceinline__ uint32_t half_word(uint32_t w, int hh) { return w >> (4 * hh); }
// Defer-max threshold (log2 units, FwdArgs::thr): the running max is raised -- and O, l
// rescaled -- only when some row's tile max exceeds it by more than this, so P = 2^(s - m)
// stays <= 2^thr.  Default 8; DTD_ATTN_RESCALE_THR overrides it (0 = textbook online softmax,
// used by the tests to check that deferral does not change the result beyond rounding).
constexpr float kRescaleThr = 8.f;

typedef float f32x2 __attribute__((ext_vector_type(2)));
// Packed fp32 (v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32: two lanes' worth of work per VALU
// issue) for the per-score softmax / dropout math of the backward kernels, which is VALU-bound.
__device__ __forceinline__ f32x2 pk_fma(f32x2 a, f32x2 b, f32x2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ f32x2 pk2(float x, float y) { return f32x2{x, y}; }
__device__ __forceinline__ float mask_bits(float v, int m) { return __int_as_float(__float_as_int(v) & m); }

// Keep-word layout.  Both mask layouts hold [B*H][W][Sp] words (Sp = 32 W) with the words of each
// 32-position group permuted: the word of position 32g + c sits at 32g + lm_pos(c), c = 8a + 4b + j
// -> 8a + 2j + b.  The words of positions c and c + 4 (b = 0) -- the two rows one accumulator
// register of a 32x32 MFMA tile holds in its lower / upper 32 lanes (crow(i, 0), crow(i, 1)) -- are
// then adjacent: register i's 64-lane keep mask is the aligned 64-bit word i of the group, one
// scalar load away, and a keep is ONE v_cndmask_b32 with that SGPR pair (attn_fwd_kernel).
__device__ __forceinline__ int lm_pos(int x) {
  const int c = x & 31;
  return (x & ~31) | (c & 24) | ((c & 3) << 1) | ((c >> 2) & 1);
}
// v ? keep : 0 for the lane's bit of a wave-uniform 64-bit mask held in an SGPR pair
__device__ __forceinline__ float sel_keep(float v, uint64_t m) {
  float r;
  asm("v_cndmask_b32_e64 %0, 0, %1, %2" : "=v"(r) : "v"(v), "s"(m));
  return r;
}
typedef __attribute__((address_space(4))) const uint64_t cu64;
// Word offset of a 32-position block's keep words inside its [Sp] row, clamped so the 32 words a
// scalar load group reads never leave the row (blocks past S -- whose scores are masked, so the
// words are discarded -- re-read the row's last block instead of running past the buffer).
__device__ __forceinline__ int keep_off(int off, int Sp) { return min(off, Sp - 32); }

struct FwdArgs {
  const bf16* q; const bf16* k; const bf16* v; bf16* o; float* lse; const float* slopes;
  const uint32_t* maskA;  // dropout keep bits [B*H][W][Sp]: bit j of word (w, q) = key 32w+j  (nullptr: no dropout)
  const uint32_t* maskB;  // [B*H][W][Sp]: bit j of word (w, key) = query 32w+j
  int B, S, H, ld, ldo, causal, W;
  float scale, p, thr;
};

// Dropout keep-masks for one attention call, generated once in a VALU-only pass at full
// occupancy (instead of re-hashing inside the MFMA-bound forward, dK/dV and dQ kernels) and
// stored as bits in two layouts so every consumer reads ONE 32-bit word per 32x32 tile:
//   A [bh][w][q]  : bit j = key 32w+j   (forward / dQ: query on the lane)
//   B [bh][w][key]: bit j = q   32w+j   (dK/dV: key on the lane) -- the transpose of A.
// Word-major ([w] outside the position) so that the 64 lanes of a consumer wave, which own 64
// consecutive queries (keys), load one contiguous 256 B line per tile -- and the generator's
// stores are contiguous too.
//
// Random stream (ops/rng.py attn_keep_mask, bit-identical), one per (bh, query) lane:
//  * seed: one counter hash of (bh * S + q), expanded by xorshift32 into a 16-word state s[0..15];
//  * per 32-key word: one additive lagged-Fibonacci round with rotation,
//      s[i] += rotl(s[(i + 11) & 15], 13)   for i = 0..15 in order (in place: lag 16 and 5),
//    2 VALU per 32 random bits (an xorshift32 step is 6);
//  * the 16 words are BIT PLANES: key j's 16-bit draw has bit i = bit j of s[i].  keep <=> draw
//    >= thr is evaluated for all 32 keys at once by the LSB-first comparator
//      acc = ~0;  acc = thr_i ? (s[i] & acc) : (s[i] | acc)     (i = 0..15)
//    -- one v_bitop3 (majority of s[i], acc and the wave-uniform ~thr_i) per plane: 0.5 VALU per
//    decision instead of 2-3 for extracting, comparing and inserting each 16-bit half.
// The generator is VALU-bound (B*H*S*S decisions per layer): ~80 VALU per 32-key word against
// ~230 for the round-2..4 form (hash-seeded xorshift per word, alignbit sign insertion).
// B words: the 32x32 bit matrix held by each 32-lane half (row = query lane, column = key) is
// transposed in registers by five block-swap stages (ds_swizzle lane ^ s, v_alignbit rotate,
// v_bfi merge): 15 issues per word.
// grid: (ceil(S / 256), B*H); block 256 = 4 waves of 64 consecutive queries, each walking all W
// key words of its queries (the stream is sequential in the word index).
template <int S_>
__device__ __forceinline__ uint32_t swap_stage(uint32_t t, uint32_t sh, uint32_t mk) {
  const uint32_t y = (uint32_t)__builtin_amdgcn_ds_swizzle((int)t, (S_ << 10) | 0x1f);   // lane ^ S_ (32-lane groups)
  const uint32_t rot = __builtin_amdgcn_alignbit(y, y, sh);
  return (rot & mk) | (t & ~mk);
}
constexpr int kMaskRot = 13;     // rotl amount of the lagged-Fibonacci round
__global__ void __launch_bounds__(256) attn_mask_kernel(uint32_t* __restrict__ maskA, uint32_t* __restrict__ maskB,
                                                        int S, int W, const uint64_t* rng, uint32_t sid, uint32_t thr) {
  const int lane = threadIdx.x & 63, bh = blockIdx.y;
  const int q0 = blockIdx.x * 256 + (threadIdx.x & ~63);     // first query of this wave
  if (q0 >= 32 * W) return;                                   // wave-uniform: nothing to store
  DropoutRng g(rng, sid);
  const int q = q0 + lane;
  const bool qv = q < S;
  uint32_t st[16];
  {
    uint32_t x = g.bits((uint64_t)bh * S + (uint64_t)(qv ? q : 0));
    x = x ? x : 0x6d2b79f5u;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      if (i) { x ^= x << 13; x ^= x >> 17; x ^= x << 5; }
      st[i] = x;
    }
  }
  // comparator constants: nt[i] = ~0 where thr's bit i is 0 (OR), 0 where it is 1 (AND); p = 1
  // (thr = 65536) and lanes past S keep nothing
  uint32_t nt[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) nt[i] = ((thr >> i) & 1u) ? 0u : 0xffffffffu;
  const uint32_t live = (qv && thr < 65536u) ? 0xffffffffu : 0u;
  // per-stage lane constants of the transpose: rotate amount and merge mask
  uint32_t sh[5], mk[5];
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    const int s = 16 >> i;
    const uint32_t Hs = i == 0 ? 0xffff0000u : i == 1 ? 0xff00ff00u : i == 2 ? 0xf0f0f0f0u : i == 3 ? 0xccccccccu : 0xaaaaaaaau;
    const bool up = lane & s;
    sh[i] = up ? s : 32 - s;
    mk[i] = up ? ~Hs : Hs;
  }
  const int qw = q0 / 32 + (lane >> 5);          // query word of the B entry this lane stores
  uint32_t* pa = maskA + (size_t)bh * W * (32 * W) + lm_pos(q);
  for (int kw = 0; kw < W; ++kw) {
    uint32_t acc = 0xffffffffu;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      st[i] += __builtin_amdgcn_alignbit(st[(i + 11) & 15], st[(i + 11) & 15], 32 - kMaskRot);
      acc = __builtin_amdgcn_bitop3_b32(st[i], acc, nt[i], 0xe8);   // majority(s, acc, nt)
    }
    uint32_t word = acc & live;
    const int nk = S - kw * 32;                  // valid keys in this word
    if (nk < 32) word &= (0xffffffffu >> (32 - nk));
    if (qv) pa[(size_t)kw * (32 * W)] = word;
    uint32_t t = word;
    t = swap_stage<16>(t, sh[0], mk[0]);
    t = swap_stage<8>(t, sh[1], mk[1]);
    t = swap_stage<4>(t, sh[2], mk[2]);
    t = swap_stage<2>(t, sh[3], mk[3]);
    t = swap_stage<1>(t, sh[4], mk[4]);
    const int key = kw * 32 + (lane & 31);
    if (key < S && qw < W) maskB[((size_t)bh * W + qw) * (32 * W) + lm_pos(key)] = t;
  }
}

// XCD-aware tile order.  Workgroups are dealt round-robin to the 8 XCDs, each with its own
// L2; in HW order the gridDim.x tiles of one (batch, head) -- which all stream the same K/V
// (dK/dV: Q/dO) -- would land on gridDim.x different XCDs and fetch those operands once per XCD.
// Renumber so each XCD runs a contiguous range of tiles: the tiles of a head share one L2.
__device__ __forceinline__ void xcd_tile(int& tx, int& ty) {
  const int nx = gridDim.x, n = nx * gridDim.y;
  const int L = blockIdx.x + nx * blockIdx.y;
  if (n % 8) { tx = blockIdx.x; ty = blockIdx.y; return; }
  const int T = (L % 8) * (n / 8) + L / 8;
  tx = T % nx;
  ty = T / nx;
}

// Bounded buffer resource (base readfirstlane'd into SGPRs): loads at byte offsets >= `bytes`
// return 0 without touching memory, which is how the tile loads below handle rows past S and
// absent dropout masks (bytes = 0) with no per-lane clamp or select.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t bounded_rsrc(const void* p, uint32_t bytes) {
  const uint64_t a = (uint64_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), (short)0, (int)bytes, 0x00020000);
}

// The [nrows x D] bf16 rows (row stride ld elements) of one (batch, head): a bounded resource,
// this thread's byte offset inside a tile, and the row pitch.  A tile load is then one
// buffer_load_dwordx4 per chunk with the row offset in an SGPR -- no per-tile VALU address math
// (64-bit multiply-adds, clamps and zeroing selects cost ~40 VALU a tile in the VALU-bound loops).
struct RowSrc {
  __amdgpu_buffer_rsrc_t rs;
  int voff, ld2;
};
template <int D>
__device__ __forceinline__ RowSrc row_src(const bf16* base, int ld, int nrows) {
  RowSrc r;
  r.rs = bounded_rsrc(base, nrows > 0 ? (uint32_t)(((nrows - 1) * ld + D) * 2) : 0u);
  r.voff = ((threadIdx.x / (D / 8)) * ld + (threadIdx.x % (D / 8)) * 8) * 2;
  r.ld2 = ld * 2;
  return r;
}
// One dropout keep word per lane (its query / key `pos`) per 32-wide word index: [W][S] uint32
// words of one (batch, head); indices past W (and every index when there is no mask) read 0.
struct WordSrc {
  __amdgpu_buffer_rsrc_t rs;
  int voff, stride;
  __device__ __forceinline__ uint32_t load(int wi) const {
    return __builtin_amdgcn_raw_buffer_load_b32(rs, voff, wi * stride, 0);
  }
};
__device__ __forceinline__ WordSrc word_src(const uint32_t* words, const void* dummy, int W, int pos) {
  WordSrc w;
  const int Sp = 32 * W;
  w.rs = bounded_rsrc(words ? (const void*)words : dummy, words ? (uint32_t)W * Sp * 4u : 0u);
  w.voff = lm_pos(pos) * 4;
  w.stride = Sp * 4;
  return w;
}

// Stage a [rows x D] bf16 tile into registers, then LDS.
template <int D, int ROWS>
struct TileLoader {
  static constexpr int CH = ROWS * D / 8;  // 16-byte chunks
  static constexpr int PER = (CH + 255) / 256;
  static constexpr int RPI = 256 / (D / 8);  // rows per 256-chunk round
  bf16x8 reg[PER];
  static_assert(CH % 256 == 0, "tile must split evenly over 256 threads");
  // straight-line loads (rows past the end read 0 through the bounded resource), so the
  // compiler can count them (partial vmcnt waits) while a second tile's loads are in flight
  // (the register ring of the kernels below)
  __device__ __forceinline__ void load(const RowSrc& src, int row0) {
#pragma unroll
    for (int i = 0; i < PER; ++i)
      reg[i] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(src.rs, src.voff, (row0 + RPI * i) * src.ld2, 0));
  }
  __device__ __forceinline__ void store(bf16* lds, int stride) const {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = threadIdx.x + 256 * i;
      *reinterpret_cast<bf16x8*>(lds + (c / (D / 8)) * stride + (c % (D / 8)) * 8) = reg[i];
    }
  }
  // D = 64: the swizzled 128-byte-row image (swz64_off); 8 contiguous lanes fill one row
  __device__ __forceinline__ void store_swz(bf16* lds) const {
    static_assert(D == 64, "swizzled tile image is for 64-column tiles");
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = threadIdx.x + 256 * i;
      *reinterpret_cast<bf16x8*>(lds + swz64_off(c >> 3, c & 7)) = reg[i];
    }
  }
  // the image the backward kernels use: swizzled for D = 64, padded rows of `stride` otherwise
  __device__ __forceinline__ void store_bwd(bf16* lds, int stride) const {
    if constexpr (D == 64) store_swz(lds);
    else store(lds, stride);
  }
};

// grid: (ceil(S/128), B*H); block 256 = 4 waves x 32 queries.  KV tiles of BN keys,
// double-buffered in LDS, fed by a 2-deep register ring of global loads: one barrier per tile.
// PK: the exp-argument FMAs and the row-sum adds as packed fp32 (v_pk_fma_f32 / v_pk_add_f32, two
// scores per issue) -- 32 fewer VALU issues per 64-key tile; the row sum's add order differs.
template <int D, int OCC, int BN, int RING, bool PK = false>
__global__ void __launch_bounds__(256, OCC) attn_fwd_kernel(FwdArgs a) {
  // K rows (ds_read_b128, 4x16-lane groups): pitch D+8 puts the 16 rows of a group on 16
  // distinct 4-bank windows.  V (ds_read_b64_tr_b16, rows rr = 0..3 x column halves g = 0,1 per
  // 32-lane group): pitch D+32 (48 / 80 dwords = 16 mod 64) places the eight 8-dword windows
  // at distinct multiples of 8 mod 64 -- D+8 aliased rows 0/2 and 1/3 (2-way conflicts).
  constexpr int KP = D + 8, VP = D + 32, NC = D / 16, NDB = D / 32, NKB = BN / 32;
  __shared__ __attribute__((aligned(16))) bf16 Ks[2][BN * KP];
  __shared__ __attribute__((aligned(16))) bf16 Vs[2][BN * VP];

  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), hh = lane >> 5,
            r = lane & 31;
  int tx, ty;
  xcd_tile(tx, ty);
  const int bh = ty, b = bh / a.H, h = bh % a.H;
  const int S = a.S;
  const int qblk = tx * 128, q0 = qblk + w * 32;
  const int q = q0 + r;
  const bool qvalid = q < S;
  const float sl2 = a.slopes ? a.slopes[h] * kLog2e : 0.f;
  const float sc2 = a.scale * kLog2e;
  const bool drop = a.maskA != nullptr;
  const float inv_keep = drop ? 1.f / (1.f - a.p) : 1.f;
  const RowSrc ksrc = row_src<D>(a.k + (size_t)b * S * a.ld + h * D, a.ld, S);
  const RowSrc vsrc = row_src<D>(a.v + (size_t)b * S * a.ld + h * D, a.ld, S);
  // dropout: this wave's 32 queries are one query word of the key-major layout, so the keep masks
  // of a 32-key block are 16 aligned 64-bit words (lm_pos) -- scalar loads, one v_cndmask per
  // score.  A one-dword-per-lane vector load of the same 64 words a tile ahead pulls them into L2.
  const int Sp = 32 * a.W;
  // keep-word addresses stay inside the real mask buffer: the row is clamped to the plane (a wave
  // whose queries lie past S still forms it) and each block's offset to the row (keep_off)
  const uint32_t* mrow = drop ? a.maskB + ((size_t)bh * a.W + min(q0 >> 5, a.W - 1)) * Sp : nullptr;
  const __amdgpu_buffer_rsrc_t mrs = bounded_rsrc(drop ? (const void*)mrow : (const void*)a.lse, drop ? (uint32_t)Sp * 4u : 0u);

  bf16x8 qf[NC];
  {
    const bf16* qp = a.q + ((size_t)(b * S + (qvalid ? q : 0)) * a.ld + h * D);
#pragma unroll
    for (int c = 0; c < NC; ++c) qf[c] = qvalid ? *reinterpret_cast<const bf16x8*>(qp + 16 * c + 8 * hh) : bf16x8{};
  }
  f32x16 oacc[NDB];
#pragma unroll
  for (int d = 0; d < NDB; ++d) oacc[d] = f32x16{};
  float m = -INFINITY, l = 0.f;

  const int kend = a.causal ? min(S, qblk + 128) : S;
  const int nt = (kend + BN - 1) / BN;
  // K/V tiles stream through a 2-deep register ring: tile t+2's global loads are issued while
  // tile t is computed and written to LDS only at the end of tile t+1, so each load has two
  // tiles of compute to arrive (one tile of MFMA/softmax work is shorter than an HBM round trip).
  // The dropout keep words (one per 32 keys) ride along in the same ring.
  // RING = 1: one register set (tile t+1 in flight during tile t) -- 16 fewer VGPRs at BN = 64,
  // which is what 3 waves per SIMD needs.
  TileLoader<D, BN> kl0, vl0, kl1r, vl1r;
  TileLoader<D, BN>& kl1 = RING == 2 ? kl1r : kl0;
  TileLoader<D, BN>& vl1 = RING == 2 ? vl1r : vl0;
  uint32_t pf0 = 0, pf1r = 0;   // L2 prefetch of keep words (value unused)
  uint32_t& pf1 = RING == 2 ? pf1r : pf0;
  auto prefetch_words = [&](int k0, uint32_t& out) {
    asm volatile("" :: "v"(out));   // retire the previous prefetch held in this register
    out = __builtin_amdgcn_raw_buffer_load_b32(mrs, lane * 4, k0 * 4, 0);
  };
  kl0.load(ksrc, 0);
  vl0.load(vsrc, 0);
  kl0.store(Ks[0], KP);
  vl0.store(Vs[0], VP);
  {
    const int k1 = min(1, nt - 1) * BN, k2 = min(2, nt - 1) * BN;
    kl1.load(ksrc, k1); vl1.load(vsrc, k1); prefetch_words(k1, pf1);
    if constexpr (RING == 2) { kl0.load(ksrc, k2); vl0.load(vsrc, k2); prefetch_words(k2, pf0); }
  }
  __syncthreads();
  // SET = register set holding tile t+1 (t even -> 1, t odd -> 0)
  auto tile = [&](auto set_c, int t) {
    constexpr int SET = decltype(set_c)::value;
    TileLoader<D, BN>& kn = SET ? kl1 : kl0;
    TileLoader<D, BN>& vn = SET ? vl1 : vl0;
    uint32_t& pfn = SET ? pf1 : pf0;
    const int buf = t & 1, k0 = t * BN;
    const bf16* K = Ks[buf];
    const bf16* V = Vs[buf];
    // keep masks of the tile's first 32-key block: issued ahead of the score MFMAs (their L2
    // round trip hides under the QK^T / softmax work); the next block's after this one's selects
    uint64_t mk[16];
    auto load_masks = [&](int kb) {
      const cu64* mp = (const cu64*)(uintptr_t)(mrow + keep_off(k0 + kb * 32, Sp));
#pragma unroll
      for (int i = 0; i < 16; ++i) mk[i] = mp[i];
    };
    f32x16 sacc[NKB];
#pragma unroll
    for (int kb = 0; kb < NKB; ++kb) {
      f32x16 acc = f32x16{};
#pragma unroll
      for (int c = 0; c < NC; ++c)
        acc = mfma32(*reinterpret_cast<const bf16x8*>(&K[(kb * 32 + r) * KP + 16 * c + 8 * hh]), qf[c], acc);
      sacc[kb] = acc;
    }
    // the first block's keep masks: issued once the score MFMAs' LDS operands are consumed (an
    // outstanding scalar load makes every later LDS wait a full lgkmcnt(0)), landing under the
    // max / exp work
    if (drop) load_masks(0);
    // log2-domain scores.  Fast path (no ALiBi, interior tile): the row max is taken on the raw
    // accumulator (scale > 0) and the scale is folded into the exponent's FMA -- 4 VALU per score
    // incl. the running sum, vs 10+ with a per-element scale/bias/mask pass.
    const bool needmask = (k0 + BN > S) || (a.causal && k0 + BN - 1 > q0);
    const bool slow = needmask || sl2 != 0.f;
    float tmax = -INFINITY;
    if (slow) {
#pragma unroll
      for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int key = k0 + kb * 32 + crow(i, hh);
          float s = fmaf(sacc[kb][i], sc2, sl2 * (float)key);
          if (needmask && (key >= S || (a.causal && key > q))) s = -INFINITY;
          sacc[kb][i] = s;
          tmax = fmaxf(tmax, s);
        }
    } else {
#pragma unroll
      for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
        for (int i = 0; i < 16; ++i) tmax = fmaxf(tmax, sacc[kb][i]);
      tmax *= sc2;
    }
    tmax = xhalf_max(tmax);
    // defer-max (wave-uniform decision): keep the running max unless some row's tile max
    // exceeds it by > kRescaleThr; the previous tile's P.V is complete, so O and l are the
    // only terms at the old scale.  m = -inf (first tile / fully masked so far) -> alpha 0.
    if (!__all(tmax - m <= a.thr)) {
      const float mnew = fmaxf(m, tmax);
      const float alpha = m == -INFINITY ? 0.f : fexp2(m - mnew);
      m = mnew;
      l *= alpha;
#pragma unroll
      for (int d = 0; d < NDB; ++d) oacc[d] *= alpha;
    }
    const float mexp = m == -INFINITY ? 0.f : m;
    const float msc = slow ? 1.f : sc2;
    // l stays a per-half partial (both halves share m, hence every rescale); the two halves
    // are combined once in the epilogue.  Four independent partial sums shorten the add chain.
    if constexpr (PK) {
      const f32x2 msc2 = pk2(msc, msc), nm2 = pk2(-mexp, -mexp);
      f32x2 ps2[2];
#pragma unroll
      for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
        for (int i = 0; i < 16; i += 2) {
          const f32x2 x = pk_fma(pk2(sacc[kb][i], sacc[kb][i + 1]), msc2, nm2);
          const f32x2 pv = pk2(fexp2(x.x), fexp2(x.y));
          const int j = (i >> 1) & 1;
          ps2[j] = (kb == 0 && i < 4) ? pv : ps2[j] + pv;
          sacc[kb][i] = pv.x;
          sacc[kb][i + 1] = pv.y;
        }
      l += (ps2[0].x + ps2[0].y) + (ps2[1].x + ps2[1].y);
    } else {
      float ps[4];
#pragma unroll
      for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const float pv = fexp2(fmaf(sacc[kb][i], msc, -mexp));
          ps[i & 3] = (kb == 0 && i < 4) ? pv : ps[i & 3] + pv;   // no "+ 0" adds (-0 semantics keep them)
          sacc[kb][i] = pv;
        }
      l += (ps[0] + ps[1]) + (ps[2] + ps[3]);
    }
    if (drop) {
#pragma unroll
      for (int kb = 0; kb < NKB; ++kb) {
        if (kb > 0) load_masks(kb);
#pragma unroll
        for (int i = 0; i < 16; ++i) sacc[kb][i] = sel_keep(sacc[kb][i], mk[i]);
      }
    }
    // O^T += V^T . P^T: the score accumulator is the B operand; V^T comes from transposed reads
#pragma unroll
    for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bf16x8 pf;
#pragma unroll
        for (int j = 0; j < 8; ++j) pf[j] = (bf16)sacc[kb][8 * s + j];
#pragma unroll
        for (int d = 0; d < NDB; ++d) oacc[d] = mfma32(tr_operand(V, VP, kb * 32 + 16 * s, d * 32, lane), pf, oacc[d]);
      }
    if (t + 1 < nt) {
      kn.store(Ks[buf ^ 1], KP);
      vn.store(Vs[buf ^ 1], VP);
      // tile t+1+RING (clamped to the last tile: a harmless reload keeps the issue unconditional)
      const int kf = min(t + 1 + RING, nt - 1) * BN;
      kn.load(ksrc, kf);
      vn.load(vsrc, kf);
      prefetch_words(kf, pfn);
    }
    __syncthreads();
  };
  for (int t = 0; t < nt; t += 2) {
    tile(std::integral_constant<int, 1>{}, t);
    if (t + 1 < nt) tile(std::integral_constant<int, 0>{}, t + 1);
  }
  l = xhalf_sum(l);
  if (!qvalid) return;
  const float inv_l = l > 0.f ? inv_keep / l : 0.f;   // dropout 1/(1-p) folded in here
  bf16* op = a.o + (size_t)(b * S + q) * a.ldo + h * D;
#pragma unroll
  for (int d = 0; d < NDB; ++d)
#pragma unroll
    for (int gq = 0; gq < 4; ++gq) {
      bf16x4 v4;
#pragma unroll
      for (int t = 0; t < 4; ++t) v4[t] = (bf16)(oacc[d][4 * gq + t] * inv_l);
      *reinterpret_cast<bf16x4*>(op + d * 32 + 8 * gq + 4 * hh) = v4;
    }
  if (hh == 0) a.lse[(size_t)bh * S + q] = (m + log2f(l)) * kLn2;
}

// Software-pipelined forward (D = 64; DTD_ATTN_FWD=pipe): the score MFMAs of K/V tile t+1 are
// issued BEFORE tile t's softmax, so within one wave the matrix pipe works on S(t+1) while the
// VALU runs tile t's max / exp / dropout / row sums (cdna_hip_programming.md T15) -- the serial
// MFMA -> VALU -> MFMA chain of attn_fwd_kernel leaves the pipe idle unless another wave of the
// SIMD happens to be in its MFMA phase.  Costs a second 32-register score accumulator.
// K runs one tile ahead of V through the LDS double buffers: at the end of tile t the register
// ring stores K(t+2) (into K(t)'s buffer, last read while S(t) was formed during tile t-1) and
// V(t+1) (into V(t-1)'s), then issues the global loads of K(t+3) and V(t+2); one barrier a tile.
// Same math, masking, defer-max and dropout as attn_fwd_kernel.
template <int D, int OCC, int BN>
__global__ void __launch_bounds__(256, OCC) attn_fwd_pipe_kernel(FwdArgs a) {
  constexpr int KP = D + 8, VP = D + 32, NC = D / 16, NDB = D / 32, NKB = BN / 32;
  __shared__ __attribute__((aligned(16))) bf16 Ks[2][BN * KP];
  __shared__ __attribute__((aligned(16))) bf16 Vs[2][BN * VP];

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, hh = lane >> 5, r = lane & 31;
  int tx, ty;
  xcd_tile(tx, ty);
  const int bh = ty, b = bh / a.H, h = bh % a.H;
  const int S = a.S;
  const int qblk = tx * 128, q0 = qblk + w * 32;
  const int q = q0 + r;
  const bool qvalid = q < S;
  const float sl2 = a.slopes ? a.slopes[h] * kLog2e : 0.f;
  const float sc2 = a.scale * kLog2e;
  const bool drop = a.maskA != nullptr;
  const float inv_keep = drop ? 1.f / (1.f - a.p) : 1.f;
  const RowSrc ksrc = row_src<D>(a.k + (size_t)b * S * a.ld + h * D, a.ld, S);
  const RowSrc vsrc = row_src<D>(a.v + (size_t)b * S * a.ld + h * D, a.ld, S);
  const WordSrc wsrc = word_src(drop ? a.maskA + (size_t)bh * a.W * (32 * a.W) : nullptr, a.lse, a.W, qvalid ? q : 0);

  bf16x8 qf[NC];
  {
    const bf16* qp = a.q + ((size_t)(b * S + (qvalid ? q : 0)) * a.ld + h * D);
#pragma unroll
    for (int c = 0; c < NC; ++c) qf[c] = qvalid ? *reinterpret_cast<const bf16x8*>(qp + 16 * c + 8 * hh) : bf16x8{};
  }
  f32x16 oacc[NDB];
#pragma unroll
  for (int d = 0; d < NDB; ++d) oacc[d] = f32x16{};
  float m = -INFINITY, l = 0.f;

  const int kend = a.causal ? min(S, qblk + 128) : S;
  const int nt = (kend + BN - 1) / BN;
  const int last = nt - 1;
  TileLoader<D, BN> kl, vl;
  uint32_t mwc[NKB], mwn[NKB];
  auto load_words = [&](int k0, uint32_t* out) {
#pragma unroll
    for (int j = 0; j < NKB; ++j) out[j] = wsrc.load((k0 >> 5) + j);
  };
  // prologue: K(0), V(0), K(1) to LDS; the ring then holds K(2), V(1) and the keep words of tile 1
  {
    TileLoader<D, BN> k1l;
    load_words(0, mwc);
    kl.load(ksrc, 0);
    vl.load(vsrc, 0);
    k1l.load(ksrc, min(1, last) * BN);
    kl.store(Ks[0], KP);
    vl.store(Vs[0], VP);
    k1l.store(Ks[1], KP);
  }
  kl.load(ksrc, min(2, last) * BN);
  vl.load(vsrc, min(1, last) * BN);
  load_words(min(1, last) * BN, mwn);
  __syncthreads();

  // score MFMAs of key block kb (32 keys) of a K tile
  auto scores_kb = [&](const bf16* K, f32x16 (&sacc)[NKB], int kb) {
    f32x16 acc = f32x16{};
#pragma unroll
    for (int c = 0; c < NC; ++c)
      acc = mfma32(*reinterpret_cast<const bf16x8*>(&K[(kb * 32 + r) * KP + 16 * c + 8 * hh]), qf[c], acc);
    sacc[kb] = acc;
  };
  // Tile t: softmax of `cur` and O += V(t)^T P(t)^T, with the score MFMAs of the next K tile
  // (Knext -> nxt) placed in the same basic blocks as the VALU work: key block 0 beside the row
  // max, key block 1 beside exp / sums / dropout.  On the last tile Knext is a stale buffer and
  // nxt is never read (unconditional issue keeps the MFMAs in the softmax's blocks).
  auto tile_step = [&](f32x16 (&cur)[NKB], f32x16 (&nxt)[NKB], const bf16* Knext, int t) {
    const int k0 = t * BN;
    const bf16* V = Vs[t & 1];
    const bool needmask = (k0 + BN > S) || (a.causal && k0 + BN - 1 > q0);
    const bool slow = needmask || sl2 != 0.f;
    float tmax = -INFINITY;
    scores_kb(Knext, nxt, 0);
    if (slow) {
#pragma unroll
      for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int key = k0 + kb * 32 + crow(i, hh);
          float sv = fmaf(cur[kb][i], sc2, sl2 * (float)key);
          if (needmask && (key >= S || (a.causal && key > q))) sv = -INFINITY;
          cur[kb][i] = sv;
          tmax = fmaxf(tmax, sv);
        }
    } else {
#pragma unroll
      for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
        for (int i = 0; i < 16; ++i) tmax = fmaxf(tmax, cur[kb][i]);
      tmax *= sc2;
    }
    tmax = xhalf_max(tmax);
    if (!__all(tmax - m <= a.thr)) {
      const float mnew = fmaxf(m, tmax);
      const float alpha = m == -INFINITY ? 0.f : fexp2(m - mnew);
      m = mnew;
      l *= alpha;
#pragma unroll
      for (int d = 0; d < NDB; ++d) oacc[d] *= alpha;
    }
    scores_kb(Knext, nxt, 1);
    const float mexp = m == -INFINITY ? 0.f : m;
    const float msc = slow ? 1.f : sc2;
    float ps[4];
#pragma unroll
    for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float pv = fexp2(fmaf(cur[kb][i], msc, -mexp));
        ps[i & 3] = (kb == 0 && i < 4) ? pv : ps[i & 3] + pv;
        cur[kb][i] = pv;
      }
    l += (ps[0] + ps[1]) + (ps[2] + ps[3]);
    if (drop) {
#pragma unroll
      for (int kb = 0; kb < NKB; ++kb) {
        const uint32_t mw = half_word(mwc[kb], hh);
#pragma unroll
        for (int i = 0; i < 16; ++i) cur[kb][i] = keep_bits(cur[kb][i], mw, crow(i, 0));
      }
    }
#pragma unroll
    for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        bf16x8 pf;
#pragma unroll
        for (int j = 0; j < 8; ++j) pf[j] = (bf16)cur[kb][8 * s2 + j];
#pragma unroll
        for (int d = 0; d < NDB; ++d) oacc[d] = mfma32(tr_operand(V, VP, kb * 32 + 16 * s2, d * 32, lane), pf, oacc[d]);
      }
    // end of tile t: K(t+2), V(t+1) from the ring into LDS, next loads, one barrier
    if (t + 1 < nt) {
      if (t + 2 < nt) kl.store(Ks[t & 1], KP);
      vl.store(Vs[(t + 1) & 1], VP);
#pragma unroll
      for (int j = 0; j < NKB; ++j) mwc[j] = mwn[j];
      kl.load(ksrc, min(t + 3, last) * BN);     // clamped: a harmless reload keeps the issue unconditional
      vl.load(vsrc, min(t + 2, last) * BN);
      load_words(min(t + 2, last) * BN, mwn);
    }
    __syncthreads();
  };
  f32x16 sA[NKB], sB[NKB];
#pragma unroll
  for (int kb = 0; kb < NKB; ++kb) scores_kb(Ks[0], sA, kb);
  for (int t = 0; t < nt; t += 2) {
    tile_step(sA, sB, Ks[1], t);                 // K(t+1) is in Ks[(t+1) & 1]
    if (t + 1 < nt) tile_step(sB, sA, Ks[0], t + 1);
  }
  l = xhalf_sum(l);
  if (!qvalid) return;
  const float inv_l = l > 0.f ? inv_keep / l : 0.f;
  bf16* op = a.o + (size_t)(b * S + q) * a.ldo + h * D;
#pragma unroll
  for (int d = 0; d < NDB; ++d)
#pragma unroll
    for (int gq = 0; gq < 4; ++gq) {
      bf16x4 v4;
#pragma unroll
      for (int t = 0; t < 4; ++t) v4[t] = (bf16)(oacc[d][4 * gq + t] * inv_l);
      *reinterpret_cast<bf16x4*>(op + d * 32 + 8 * gq + 4 * hh) = v4;
    }
  if (hh == 0) a.lse[(size_t)bh * S + q] = (m + log2f(l)) * kLn2;
}

struct BwdArgs {
  const bf16* q; const bf16* k; const bf16* v; const bf16* dout; const float* lse; float* delta;
  const bf16* o;   // forward output: the dQ kernel forms delta = rowsum(dO * O) from it
  bf16* dq; bf16* dk; bf16* dv; const float* slopes;
  const uint32_t* maskA; const uint32_t* maskB;  // dropout keep bits (see attn_mask_kernel)
  int B, S, H, ld, ldo, causal, W;
  float scale, p;
  // optional [B * 4 * ceil(S/128)][3 H D] fp32 column partials of dqkv (the qkv bias gradient):
  // one row per (batch, 32-row block of a wave), finished by colsum_finalize
  float* bias_part;
};

// Column sums of a wave's 32 rows x 64 columns of dQ / dK / dV, straight from the accumulators
// (lane r = row of its half-wave, register k = 16 d + i = column d*32 + crow(i, half)): a
// butterfly reduce-scatter over the 32 lanes of each half (ds_swizzle lane ^ s) leaves the sum of
// column index k = r in lane r -- 31 exchanges instead of 32 x 5 -- and one store per wave writes
// the 64 column partials.  This replaces a separate pass over the 3 H D-wide gradient (the qkv
// bias gradient: ~90 us a layer at b256 x 512).
template <int S_>
__device__ __forceinline__ float xswz(float x) {
  return __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(x), (S_ << 10) | 0x1f));
}
template <int S_, int N>
__device__ __forceinline__ void rs_step(const float (&in)[2 * N], float (&out)[N], int r) {
  const bool hi = (r & S_) != 0;
#pragma unroll
  for (int j = 0; j < N; ++j) {
    const float mine = hi ? in[j + N] : in[j];
    const float other = hi ? in[j] : in[j + N];
    out[j] = mine + xswz<S_>(other);
  }
}
__device__ __forceinline__ float colsum32(const float (&v)[32], int r) {
  float a16[16], a8[8], a4[4], a2[2], a1[1];
  rs_step<16, 16>(v, a16, r);
  rs_step<8, 8>(a16, a8, r);
  rs_step<4, 4>(a8, a4, r);
  rs_step<2, 2>(a4, a2, r);
  rs_step<1, 1>(a2, a1, r);
  return a1[0];
}
// column (within the head) of register index k = 16 d + i in lane half hh
__device__ __forceinline__ int colsum_col(int k, int hh) { return (k >> 4) * 32 + crow(k & 15, hh); }

// dK, dV: grid (ceil(S/128), B*H); block 256 = 4 waves x 32 keys ("key on the lane").
// Query tiles of 64 rows (Q, dO row-major in LDS, double-buffered).
// DROP / ALIBI are compile-time so that the hot path has no runtime branch (whose register
// merges cost 16 v_mov per query sub-block) and no bias add without ALiBi.
// MASK = false: the launch knows no block needs the causal / sequence-end mask (not causal, S a
// multiple of 128).  The runtime `needmask` branch alone is not enough: hipcc hoists the 16 key /
// query comparisons and their lane-mask combines above it, 48 VALU + 52 SALU per 32-query
// sub-block executed on every interior block.
template <int D, int OCC, int BM, bool DROP, bool ALIBI, bool MASK = true>
__global__ void __launch_bounds__(256, OCC) attn_bwd_dkdv_kernel(BwdArgs a) {
  constexpr bool SWZ = D == 64;                 // swizzled unpadded image (swz64_off)
  constexpr int QP = SWZ ? D : D + 8, NC = D / 16, NDB = D / 32;
  // One LDS block, row statistics first: placed after the 72 KiB of Q/dO tiles (BM = 128) their
  // ds_read offsets exceed the 16-bit immediate and every read needed a VALU address add.
  struct Smem {
    float lse_s[2][BM], del_s[2][BM];
    bf16 Qs[2][BM * QP];
    bf16 Os[2][BM * QP];
  };
  __shared__ __attribute__((aligned(16))) Smem sm;
  auto& lse_s = sm.lse_s;
  auto& del_s = sm.del_s;
  auto& Qs = sm.Qs;
  auto& Os = sm.Os;

  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), hh = lane >> 5,
            r = lane & 31;
  int tx, ty;
  xcd_tile(tx, ty);
  const int bh = ty, b = bh / a.H, h = bh % a.H;
  const int S = a.S;
  const int kblk = tx * 128;
  const int key = kblk + w * 32 + r;
  const bool kvalid = key < S;
  const float sl2 = a.slopes ? a.slopes[h] * kLog2e : 0.f;
  const float sc2 = a.scale * kLog2e;
  constexpr bool drop = DROP;
  const float inv_keep = drop ? 1.f / (1.f - a.p) : 1.f;
  const float kbias = sl2 * (float)key;   // ALiBi bias of this lane's key (0 without ALiBi)
  // keep masks: this wave's 32 keys are one key word of the query-major layout A, so a 32-query
  // block's masks are 16 aligned 64-bit words (lm_pos) -- scalar loads, one v_cndmask per use
  const int Sp = 32 * a.W;
  const uint32_t* mrow = drop ? a.maskA + ((size_t)bh * a.W + min((kblk >> 5) + w, a.W - 1)) * Sp : nullptr;
  const __amdgpu_buffer_rsrc_t mrs = bounded_rsrc(drop ? (const void*)mrow : (const void*)a.lse, drop ? (uint32_t)Sp * 4u : 0u);
  const RowSrc qsrc = row_src<D>(a.q + (size_t)b * S * a.ld + h * D, a.ld, S);
  const RowSrc osrc = row_src<D>(a.dout + (size_t)b * S * a.ldo + h * D, a.ldo, S);
  const float* lseb = a.lse + (size_t)bh * S;
  const float* delb = a.delta + (size_t)bh * S;

  bf16x8 kf[NC], vf[NC];
  {
    const size_t off = (size_t)(b * S + (kvalid ? key : 0)) * a.ld + h * D;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      kf[c] = kvalid ? *reinterpret_cast<const bf16x8*>(a.k + off + 16 * c + 8 * hh) : bf16x8{};
      vf[c] = kvalid ? *reinterpret_cast<const bf16x8*>(a.v + off + 16 * c + 8 * hh) : bf16x8{};
    }
  }
  f32x16 dk[NDB], dv[NDB];
#pragma unroll
  for (int d = 0; d < NDB; ++d) { dk[d] = f32x16{}; dv[d] = f32x16{}; }

  const int qstart = a.causal ? (kblk / BM) * BM : 0;
  const int nt = (S - qstart + BM - 1) / BM;
  TileLoader<D, BM> ql, ol;
  float lse_r = 0.f, del_r = 0.f;
  auto load_stats = [&](int q0) {
    if (threadIdx.x < BM) {
      const int qq = q0 + threadIdx.x;
      lse_r = qq < S ? -lseb[qq] * kLog2e : 0.f;   // stored negated: P = 2^fma(s, sc2, -lse)
      // dS = P (dP - delta); with dropout the kernel forms dS' = (1 - p) dS = Pm dP - P (1 - p) delta
      // (Pm = P * keep), so delta is stored pre-scaled and dK takes the 1 / (1 - p) at the end
      del_r = qq < S ? -delb[qq] * (DROP ? 1.f - a.p : 1.f) : 0.f;
    }
  };
  // L2 prefetch of the next query tile's keep words (BM words, value unused)
  constexpr int NPF = BM / 64;
  uint32_t pfw[NPF] = {};
  auto prefetch_words = [&](int q0) {
#pragma unroll
    for (int j = 0; j < NPF; ++j) {
      asm volatile("" :: "v"(pfw[j]));
      pfw[j] = __builtin_amdgcn_raw_buffer_load_b32(mrs, (lane + 64 * j) * 4, q0 * 4, 0);
    }
  };
  ql.load(qsrc, qstart);
  ol.load(osrc, qstart);
  load_stats(qstart);
  ql.store_bwd(Qs[0], QP);
  ol.store_bwd(Os[0], QP);
  if (threadIdx.x < BM) { lse_s[0][threadIdx.x] = lse_r; del_s[0][threadIdx.x] = del_r; }
  __syncthreads();
  for (int t = 0; t < nt; ++t) {
    const int buf = t & 1, q0 = qstart + t * BM;
    if (t + 1 < nt) {
      ql.load(qsrc, q0 + BM);
      ol.load(osrc, q0 + BM);
      load_stats(q0 + BM);
      if (drop) prefetch_words(q0 + BM);
    }
    const bf16* Q = Qs[buf];
    const bf16* O = Os[buf];
    // one wave per SIMD (OCC 1, 512 registers): unroll the query sub-blocks so the S/dP MFMAs
    // of sub-block qb+1 can be scheduled under the softmax VALU of qb; at OCC 2 the register
    // budget keeps the sub-blocks serial
    constexpr int kQbUnroll = OCC == 1 ? BM / 32 : 1;
#pragma unroll kQbUnroll
    for (int qb = 0; qb < BM / 32; ++qb) {
      f32x16 sacc = f32x16{}, pacc = f32x16{};
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        if constexpr (SWZ) {
          sacc = mfma32(swz_row_read(Q, qb * 32, r, 2 * c + hh), kf[c], sacc);
          pacc = mfma32(swz_row_read(O, qb * 32, r, 2 * c + hh), vf[c], pacc);
        } else {
          sacc = mfma32(*reinterpret_cast<const bf16x8*>(&Q[(qb * 32 + r) * QP + 16 * c + 8 * hh]), kf[c], sacc);
          pacc = mfma32(*reinterpret_cast<const bf16x8*>(&O[(qb * 32 + r) * QP + 16 * c + 8 * hh]), vf[c], pacc);
        }
      }
      const int qrow0 = q0 + qb * 32;
      // block-uniform predicate (a scalar branch, never a per-element one)
      const bool needmask = MASK && ((kblk + 128 > S) || (qrow0 + 32 > S) || (a.causal && kblk + 127 > qrow0));
      // this query block's keep masks (after the S / dP MFMAs consumed their LDS operands)
      uint64_t mk[16];
      if constexpr (DROP) {
        const cu64* mp = (const cu64*)(uintptr_t)(mrow + keep_off(qrow0, Sp));
#pragma unroll
        for (int i = 0; i < 16; ++i) mk[i] = mp[i];
      }
      // row statistics of this lane's 16 accumulator rows (rows 8g + 4hh + 0..3 are contiguous):
      // 8 ds_read_b128 issued together instead of 32 dependent scalar LDS reads
      f32x4 L4[4], D4[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        L4[g] = *reinterpret_cast<const f32x4*>(&lse_s[buf][qb * 32 + 8 * g + 4 * hh]);
        D4[g] = *reinterpret_cast<const f32x4*>(&del_s[buf][qb * 32 + 8 * g + 4 * hh]);
      }
      // P = 2^(s sc2 + kbias - lse): score pairs (i, i+1) share a row group, so the row terms pair up
      const f32x2 sc2v = pk2(sc2, sc2), kb2 = pk2(kbias, kbias);
#pragma unroll
      for (int i = 0; i < 16; i += 2) {
        f32x2 nl = pk2(L4[i >> 2][i & 3], L4[i >> 2][(i & 3) + 1]);
        if constexpr (ALIBI) nl += kb2;
        const f32x2 x = pk_fma(pk2(sacc[i], sacc[i + 1]), sc2v, nl);
        sacc[i] = fexp2(x.x);
        sacc[i + 1] = fexp2(x.y);
      }
      if (MASK && needmask) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int qq = qrow0 + crow(i, hh);
          const bool ok = kvalid && qq < S && !(a.causal && key > qq);
          sacc[i] = ok ? sacc[i] : 0.f;
        }
      }
#pragma unroll
      for (int i = 0; i < 16; i += 2) {
        const f32x2 nd = pk2(D4[i >> 2][i & 3], D4[i >> 2][(i & 3) + 1]);
        if constexpr (DROP) {
          // 2 VALU issues per score instead of 3: one keep select (Pm feeds both dV and dS')
          const f32x2 pm = pk2(sel_keep(sacc[i], mk[i]), sel_keep(sacc[i + 1], mk[i + 1]));
          const f32x2 u = pk2(sacc[i], sacc[i + 1]) * nd;                 // -P (1 - p) delta
          const f32x2 ds = pk_fma(pm, pk2(pacc[i], pacc[i + 1]), u);      // dS' = (1 - p) dS
          pacc[i] = ds.x;
          pacc[i + 1] = ds.y;
          sacc[i] = pm.x;                                                 // P*mask (dV)
          sacc[i + 1] = pm.y;
        } else {
          const f32x2 ds = pk2(sacc[i], sacc[i + 1]) * (pk2(pacc[i], pacc[i + 1]) + nd);
          pacc[i] = ds.x;
          pacc[i + 1] = ds.y;
        }
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bf16x8 pb, sb;
#pragma unroll
        for (int j = 0; j < 8; ++j) { pb[j] = (bf16)sacc[8 * s + j]; sb[j] = (bf16)pacc[8 * s + j]; }
#pragma unroll
        for (int d = 0; d < NDB; ++d) {
          if constexpr (SWZ) {
            dv[d] = mfma32(tr_operand_swz(O, qb * 32 + 16 * s, d * 32, lane), pb, dv[d]);
            dk[d] = mfma32(tr_operand_swz(Q, qb * 32 + 16 * s, d * 32, lane), sb, dk[d]);
          } else {
            dv[d] = mfma32(tr_operand(O, QP, qb * 32 + 16 * s, d * 32, lane), pb, dv[d]);
            dk[d] = mfma32(tr_operand(Q, QP, qb * 32 + 16 * s, d * 32, lane), sb, dk[d]);
          }
        }
      }
    }
    if (t + 1 < nt) {
      ql.store_bwd(Qs[buf ^ 1], QP);
      ol.store_bwd(Os[buf ^ 1], QP);
      if (threadIdx.x < BM) { lse_s[buf ^ 1][threadIdx.x] = lse_r; del_s[buf ^ 1][threadIdx.x] = del_r; }
    }
    __syncthreads();
  }
  const float dv_scale = inv_keep;   // the dropped P fed to dV carried keep bits only
  const float dk_scale = a.scale * inv_keep;   // dS' = (1 - p) dS (see load_stats)
  if (a.bias_part && D == 64) {
    float vk[32], vv[32];
#pragma unroll
    for (int d = 0; d < NDB; ++d)
#pragma unroll
      for (int i = 0; i < 16; ++i) {   // the stored (bf16-rounded) values, 0 past S
        vk[16 * d + i] = kvalid ? (float)(bf16)(dk[d][i] * dk_scale) : 0.f;
        vv[16 * d + i] = kvalid ? (float)(bf16)(dv[d][i] * dv_scale) : 0.f;
      }
    const float sk = colsum32(vk, r), sv = colsum32(vv, r);
    float* row = a.bias_part + ((size_t)b * gridDim.x * 4 + (kblk >> 5) + w) * (3 * a.H * D) + h * D + colsum_col(r, hh);
    row[a.H * D] = sk;
    row[2 * a.H * D] = sv;
  }
  if (!kvalid) return;
  bf16* dkp = a.dk + (size_t)(b * S + key) * a.ld + h * D;
  bf16* dvp = a.dv + (size_t)(b * S + key) * a.ld + h * D;
#pragma unroll
  for (int d = 0; d < NDB; ++d)
#pragma unroll
    for (int gq = 0; gq < 4; ++gq) {
      bf16x4 k4, v4;
#pragma unroll
      for (int t = 0; t < 4; ++t) { k4[t] = (bf16)(dk[d][4 * gq + t] * dk_scale); v4[t] = (bf16)(dv[d][4 * gq + t] * dv_scale); }
      *reinterpret_cast<bf16x4*>(dkp + d * 32 + 8 * gq + 4 * hh) = k4;
      *reinterpret_cast<bf16x4*>(dvp + d * 32 + 8 * gq + 4 * hh) = v4;
    }
}

// dQ: grid (ceil(S/128), B*H); block 256 = 4 waves x 32 queries (query on the lane, as in the
// forward); recomputes S^T and dP^T per 64-key tile and accumulates dQ^T = K^T.dS^T in
// registers -- no atomics, no cross-workgroup reduction.
// PK: packed-fp32 exp arguments and dS = P (dP - delta) (v_pk_fma_f32 / v_pk_mul_f32)
template <int D, int OCC, int BN, int RING, bool PK = false>
__global__ void __launch_bounds__(256, OCC) attn_bwd_dq_kernel(BwdArgs a) {
  constexpr bool SWZ = D == 64;                 // swizzled unpadded K / V images (swz64_off)
  constexpr int KP = SWZ ? D : D + 8, NC = D / 16, NDB = D / 32;
  __shared__ __attribute__((aligned(16))) bf16 Ks[2][BN * KP];
  __shared__ __attribute__((aligned(16))) bf16 Vs[2][BN * KP];

  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), hh = lane >> 5,
            r = lane & 31;
  int tx, ty;
  xcd_tile(tx, ty);
  const int bh = ty, b = bh / a.H, h = bh % a.H;
  const int S = a.S;
  const int qblk = tx * 128, q0 = qblk + w * 32;
  const int q = q0 + r;
  const bool qvalid = q < S;
  const float sl2 = a.slopes ? a.slopes[h] * kLog2e : 0.f;
  const float sc2 = a.scale * kLog2e;
  const bool drop = a.maskA != nullptr;
  const float inv_keep = drop ? 1.f / (1.f - a.p) : 1.f;
  const RowSrc ksrc = row_src<D>(a.k + (size_t)b * S * a.ld + h * D, a.ld, S);
  const RowSrc vsrc = row_src<D>(a.v + (size_t)b * S * a.ld + h * D, a.ld, S);
  // keep masks as in attn_fwd_kernel: 64-bit lane masks of the key-major layout, scalar loads
  const int Sp = 32 * a.W;
  const uint32_t* mrow = drop ? a.maskB + ((size_t)bh * a.W + min(q0 >> 5, a.W - 1)) * Sp : nullptr;
  const __amdgpu_buffer_rsrc_t mrs = bounded_rsrc(drop ? (const void*)mrow : (const void*)a.lse, drop ? (uint32_t)Sp * 4u : 0u);

  bf16x8 qf[NC], of[NC];
  {
    const bf16* qp = a.q + ((size_t)(b * S + (qvalid ? q : 0)) * a.ld + h * D);
    const bf16* op = a.dout + ((size_t)(b * S + (qvalid ? q : 0)) * a.ldo + h * D);
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      qf[c] = qvalid ? *reinterpret_cast<const bf16x8*>(qp + 16 * c + 8 * hh) : bf16x8{};
      of[c] = qvalid ? *reinterpret_cast<const bf16x8*>(op + 16 * c + 8 * hh) : bf16x8{};
    }
  }
  const float lse2 = qvalid ? a.lse[(size_t)bh * S + q] * kLog2e : 0.f;
  // delta = rowsum(dO * O) of this lane's query, from the dO fragments already in registers and
  // one O row read (no separate delta pass re-reading dO); stored for the dK/dV kernel, which
  // runs after this one
  float dl;
  {
    const bf16* orow = a.o + ((size_t)(b * S + (qvalid ? q : 0)) * a.ldo + h * D);
    float part = 0.f;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const bf16x8 ov = qvalid ? *reinterpret_cast<const bf16x8*>(orow + 16 * c + 8 * hh) : bf16x8{};
#pragma unroll
      for (int j = 0; j < 8; ++j) part = fmaf((float)ov[j], (float)of[c][j], part);
    }
    dl = xhalf_sum(part);
    if (qvalid && hh == 0) a.delta[(size_t)bh * S + q] = dl;
  }
  f32x16 dq[NDB];
#pragma unroll
  for (int d = 0; d < NDB; ++d) dq[d] = f32x16{};

  const int kend = a.causal ? min(S, qblk + 128) : S;
  const int nt = (kend + BN - 1) / BN;
  // K/V tiles + dropout keep words through a 2-deep register ring (see attn_fwd_kernel)
  constexpr int NKB = BN / 32;
  // RING = 1: one register set in flight (fewer VGPRs -> 3 waves per SIMD), see attn_fwd_kernel
  TileLoader<D, BN> kl0, vl0, kl1r, vl1r;
  TileLoader<D, BN>& kl1 = RING == 2 ? kl1r : kl0;
  TileLoader<D, BN>& vl1 = RING == 2 ? vl1r : vl0;
  uint32_t pf0 = 0, pf1r = 0;   // L2 prefetch of keep words (value unused)
  uint32_t& pf1 = RING == 2 ? pf1r : pf0;
  auto prefetch_words = [&](int k0, uint32_t& out) {
    asm volatile("" :: "v"(out));
    out = __builtin_amdgcn_raw_buffer_load_b32(mrs, lane * 4, k0 * 4, 0);
  };
  kl0.load(ksrc, 0);
  vl0.load(vsrc, 0);
  kl0.store_bwd(Ks[0], KP);
  vl0.store_bwd(Vs[0], KP);
  {
    const int k1 = min(1, nt - 1) * BN, k2 = min(2, nt - 1) * BN;
    kl1.load(ksrc, k1); vl1.load(vsrc, k1); prefetch_words(k1, pf1);
    if constexpr (RING == 2) { kl0.load(ksrc, k2); vl0.load(vsrc, k2); prefetch_words(k2, pf0); }
  }
  __syncthreads();
  auto tile = [&](auto set_c, int t) {
    constexpr int SET = decltype(set_c)::value;
    TileLoader<D, BN>& kn = SET ? kl1 : kl0;
    TileLoader<D, BN>& vn = SET ? vl1 : vl0;
    uint32_t& pfn = SET ? pf1 : pf0;
    const int buf = t & 1, k0 = t * BN;
    const bf16* K = Ks[buf];
    const bf16* V = Vs[buf];
    const bool needmask = !qvalid || (k0 + BN > S) || (a.causal && k0 + BN - 1 > q0);
#pragma unroll
    for (int kb = 0; kb < BN / 32; ++kb) {
      f32x16 sacc = f32x16{}, pacc = f32x16{};
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        if constexpr (SWZ) {
          sacc = mfma32(swz_row_read(K, kb * 32, r, 2 * c + hh), qf[c], sacc);
          pacc = mfma32(swz_row_read(V, kb * 32, r, 2 * c + hh), of[c], pacc);
        } else {
          sacc = mfma32(*reinterpret_cast<const bf16x8*>(&K[(kb * 32 + r) * KP + 16 * c + 8 * hh]), qf[c], sacc);
          pacc = mfma32(*reinterpret_cast<const bf16x8*>(&V[(kb * 32 + r) * KP + 16 * c + 8 * hh]), of[c], pacc);
        }
      }
      // this block's keep masks (after the S / dP MFMAs consumed their LDS operands)
      uint64_t mk[16];
      if (drop) {
        const cu64* mp = (const cu64*)(uintptr_t)(mrow + keep_off(k0 + kb * 32, Sp));
#pragma unroll
        for (int i = 0; i < 16; ++i) mk[i] = mp[i];
      }
      // P = exp2(s*log2e - lse): 2 VALU on interior tiles without ALiBi
      if (needmask || sl2 != 0.f) {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int key = k0 + kb * 32 + crow(i, hh);
          float pv = fexp2(fmaf(sacc[i], sc2, sl2 * (float)key - lse2));
          if (needmask && (!qvalid || key >= S || (a.causal && key > q))) pv = 0.f;
          sacc[i] = pv;
        }
      } else if constexpr (PK) {
        const f32x2 sc22 = pk2(sc2, sc2), nl2 = pk2(-lse2, -lse2);
#pragma unroll
        for (int i = 0; i < 16; i += 2) {
          const f32x2 x = pk_fma(pk2(sacc[i], sacc[i + 1]), sc22, nl2);
          sacc[i] = fexp2(x.x);
          sacc[i + 1] = fexp2(x.y);
        }
      } else {
#pragma unroll
        for (int i = 0; i < 16; ++i) sacc[i] = fexp2(fmaf(sacc[i], sc2, -lse2));
      }
      // dS^T = P * (dP - delta), dP = dropout(dP') (keep bit, 1/(1-p))
      if constexpr (PK) {
        const f32x2 ik2 = pk2(drop ? inv_keep : 1.f, drop ? inv_keep : 1.f), nd2 = pk2(-dl, -dl);
#pragma unroll
        for (int i = 0; i < 16; i += 2) {
          f32x2 dp = pk2(pacc[i], pacc[i + 1]);
          if (drop) dp = pk2(sel_keep(pacc[i], mk[i]), sel_keep(pacc[i + 1], mk[i + 1]));
          const f32x2 ds = pk2(sacc[i], sacc[i + 1]) * pk_fma(dp, ik2, nd2);
          sacc[i] = ds.x;
          sacc[i + 1] = ds.y;
        }
      } else if (drop) {
#pragma unroll
        for (int i = 0; i < 16; ++i) sacc[i] *= fmaf(sel_keep(pacc[i], mk[i]), inv_keep, -dl);
      } else {
#pragma unroll
        for (int i = 0; i < 16; ++i) sacc[i] *= pacc[i] - dl;
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bf16x8 sb;
#pragma unroll
        for (int j = 0; j < 8; ++j) sb[j] = (bf16)sacc[8 * s + j];
#pragma unroll
        for (int d = 0; d < NDB; ++d) {
          if constexpr (SWZ) dq[d] = mfma32(tr_operand_swz(K, kb * 32 + 16 * s, d * 32, lane), sb, dq[d]);
          else dq[d] = mfma32(tr_operand(K, KP, kb * 32 + 16 * s, d * 32, lane), sb, dq[d]);
        }
      }
    }
    if (t + 1 < nt) {
      kn.store_bwd(Ks[buf ^ 1], KP);
      vn.store_bwd(Vs[buf ^ 1], KP);
      // tile t+1+RING (clamped to the last tile: a harmless reload keeps the issue unconditional)
      const int kf = min(t + 1 + RING, nt - 1) * BN;
      kn.load(ksrc, kf);
      vn.load(vsrc, kf);
      prefetch_words(kf, pfn);
    }
    __syncthreads();
  };
  for (int t = 0; t < nt; t += 2) {
    tile(std::integral_constant<int, 1>{}, t);
    if (t + 1 < nt) tile(std::integral_constant<int, 0>{}, t + 1);
  }
  if (a.bias_part && D == 64) {
    float vq[32];
#pragma unroll
    for (int d = 0; d < NDB; ++d)
#pragma unroll
      for (int i = 0; i < 16; ++i) vq[16 * d + i] = qvalid ? (float)(bf16)(dq[d][i] * a.scale) : 0.f;
    const float sq = colsum32(vq, r);
    a.bias_part[((size_t)b * gridDim.x * 4 + (qblk >> 5) + w) * (3 * a.H * D) + h * D + colsum_col(r, hh)] = sq;
  }
  if (!qvalid) return;
  bf16* qp = a.dq + (size_t)(b * S + q) * a.ld + h * D;
#pragma unroll
  for (int d = 0; d < NDB; ++d)
#pragma unroll
    for (int gq = 0; gq < 4; ++gq) {
      bf16x4 v4;
#pragma unroll
      for (int t = 0; t < 4; ++t) v4[t] = (bf16)(dq[d][4 * gq + t] * a.scale);
      *reinterpret_cast<bf16x4*>(qp + d * 32 + 8 * gq + 4 * hh) = v4;
    }
}

#if DTD_ATTN_FUSED_BWD   // experimental builds only (DTD_BUILD_EXPERIMENTAL=1, ops/build.py): the
                        // one-kernel backward forms measured no faster than the split kernels
                        // (profiles/r4_attn_fused_bwd_ab.jsonl), so the default library omits them
// ---------------------------------------------------------------------------------------------
// Fused backward (D = 64, no causal mask, no ALiBi, S = 128 NKB <= 512): ONE workgroup per
// (batch, head) owns every key, so dQ needs neither atomics nor a second kernel that recomputes
// the softmax.  Five MFMA products per score tile instead of the split kernels' seven, and the
// per-score VALU work (exp, dropout select, dS) done once instead of twice.
//   * wave w keeps dK^T / dV^T of its KPW = S/4 keys in accumulator registers (key on the lane,
//     as in attn_bwd_dkdv_kernel: 256 of the 512 registers at S = 512); the whole K and V of the
//     head sit in LDS (swizzled 128-byte rows): row reads for S and dP, transposed reads of K for dQ;
//   * the workgroup sweeps 32-row query tiles.  Per round of KH key blocks per wave: S, dP ->
//     P, dS per 32-key block; dV^T += dO^T.P, dK^T += Q^T.dS; dS^T goes to LDS as a
//     [key][query] image; barrier; dQ^T (64 x 32) += K^T . dS^T over the round's keys with
//     16x16x32 MFMAs (wave w: head dims 16w .. 16w+15 of both 16-query halves -- no partial
//     sums across waves); barrier.  After the last round each wave stores its dQ slice (and its
//     qkv-bias column sums) and the next tile is staged.
//   * delta = rowsum(dO * O) of the next tile is formed while it is staged (no separate pass).
// LDS 154 KiB at S = 512: one workgroup per CU, one wave per SIMD.
__device__ __forceinline__ f32x4 mfma16(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// dK^T / dV^T update with the accumulator pinned to the accumulator file ("+a"): at 256 live
// accumulator registers the compiler kept some of them in arch VGPRs and copied them into and out
// of AGPRs around every MFMA (and spilled).  s_nop 1: the A / B operands may be fresh VALU results
// (cdna_hip_programming.md §5.7 item 2); the accumulate chain itself needs no wait states.  hipcc
// takes the statement as complete at its end, so the results must be waited out before anything
// but the next MFMA of the chain touches them (the s_nop 15 + pin statements in the kernel;
// scripts/diag/audit_fused_bwd_asm.py checks the built ISA for such early reads).
__device__ __forceinline__ void mfma32_a(f32x16& acc, bf16x8 a, bf16x8 b) {
  asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}

// S / dP products with the accumulator in arch VGPRs ("v": the builtin put them in the accumulator
// file, which the dK/dV accumulators fill, and every softmax read then cost a v_accvgpr_read).
// C = 0 for the first product of a chain; mfma_vgpr_wait() (12 wait states, 8-pass XDL) before
// the VALU reads the chain's result.
__device__ __forceinline__ void mfma32_v0(f32x16& acc, bf16x8 a, bf16x8 b) {
  asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=&v"(acc) : "v"(a), "v"(b));
}
__device__ __forceinline__ void mfma32_v(f32x16& acc, bf16x8 a, bf16x8 b) {
  asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b));
}
__device__ __forceinline__ void mfma_vgpr_wait(f32x16& x, f32x16& y) {
  asm volatile("s_nop 11" : "+v"(x), "+v"(y));
}
// dQ^T 16x16x32 products, accumulator in arch VGPRs for the same reason (4-pass XDL: the
// s_nop 7 statement after the chain covers the result's readers)
__device__ __forceinline__ void mfma16_v(f32x4& acc, bf16x8 a, bf16x8 b) {
  asm volatile("s_nop 1\n\tv_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(acc) : "v"(a), "v"(b));
}

template <int NKB, bool DROP>
__global__ void __launch_bounds__(256, 1) attn_bwd_fused_kernel(BwdArgs a) {
  constexpr int D = 64, NC = 4, NDB = 2, SK = 128 * NKB, KPW = 32 * NKB, NT = SK / 32;
  constexpr int KH = NKB % 2 == 0 ? 2 : 1, NH = NKB / KH;   // key blocks per round, rounds per tile
  constexpr int DSP = 36;                                   // dS^T image pitch (bf16): 72-byte rows
  constexpr int DSR = 4 * KH * 32;                          // dS^T image rows (keys of one round)
  struct Smem {
    float lse_s[32], del_s[32];
    bf16 Qs[32 * 64];
    bf16 Os[32 * 64];
    bf16 DS[DSR * DSP];
    bf16 Ks[SK * 64];
    bf16 Vs[SK * 64];
  };
  __shared__ __attribute__((aligned(16))) Smem sm;

  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6), hh = lane >> 5,
            r = lane & 31;
  const int bh = blockIdx.x, b = bh / a.H, h = bh % a.H;
  const int S = a.S;   // == SK (host-checked)
  const float sc2 = a.scale * kLog2e;
  const float inv_keep = DROP ? 1.f / (1.f - a.p) : 1.f;
  const int kw0 = w * KPW;
  const int Sp = 32 * a.W;
  const float* lseb = a.lse + (size_t)bh * S;
  const RowSrc qsrc = row_src<D>(a.q + (size_t)b * S * a.ld + h * D, a.ld, S);
  const RowSrc dsrc = row_src<D>(a.dout + (size_t)b * S * a.ldo + h * D, a.ldo, S);
  const RowSrc osrc = row_src<D>(a.o + (size_t)b * S * a.ldo + h * D, a.ldo, S);
  {
    const RowSrc ksrc = row_src<D>(a.k + (size_t)b * S * a.ld + h * D, a.ld, S);
    const RowSrc vsrc = row_src<D>(a.v + (size_t)b * S * a.ld + h * D, a.ld, S);
#pragma unroll
    for (int half = 0; half < 2; ++half) {   // 64 rows per thread-round x 2 operands, in 2 passes
      TileLoader<D, SK / 2> kl, vl;
      kl.load(ksrc, half * (SK / 2));
      vl.load(vsrc, half * (SK / 2));
      kl.store_swz(sm.Ks + half * (SK / 2) * 64);
      vl.store_swz(sm.Vs + half * (SK / 2) * 64);
    }
  }
  // query-tile staging: Q / dO rows (swizzled), -lse*log2e and -delta of the 32 rows
  TileLoader<D, 32> ql, dl, ol;
  float lse_n = 0.f;
  auto fetch = [&](int q0) {
    ql.load(qsrc, q0);
    dl.load(dsrc, q0);
    ol.load(osrc, q0);
    if (tid < 32) lse_n = lseb[q0 + tid];
  };
  auto stage = [&]() {
    // thread tid holds row tid >> 3, columns 8 (tid & 7) .. +7 of dO and O
    float part = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) part = fmaf((float)dl.reg[0][j], (float)ol.reg[0][j], part);
    part += __shfl_xor(part, 1, 64);
    part += __shfl_xor(part, 2, 64);
    part += __shfl_xor(part, 4, 64);
    ql.store_swz(sm.Qs);
    dl.store_swz(sm.Os);
    if ((tid & 7) == 0) sm.del_s[tid >> 3] = -part;
    if (tid < 32) sm.lse_s[tid] = -lse_n * kLog2e;
  };
  fetch(0);
  stage();

  f32x16 dk[NKB][NDB], dv[NKB][NDB];
#pragma unroll
  for (int kb = 0; kb < NKB; ++kb)
#pragma unroll
    for (int d = 0; d < NDB; ++d) { dk[kb][d] = f32x16{}; dv[kb][d] = f32x16{}; }
  // dQ operand addressing (16x16x32 transposed reads): lane group g16 = lane >> 4 takes keys
  // 8 g16 .. +7 of a 32-key step; lane 4 qq + pp of the group addresses row 8 g16 + qq (+4)
  const int g16 = lane >> 4, l16 = lane & 15, qq = l16 >> 2, pp = l16 & 3;
  const int kcol = 16 * w + 4 * pp;   // K^T rows of this wave: head dims 16w .. 16w+15
  __syncthreads();

  for (int t = 0; t < NT; ++t) {
    const int q0 = t * 32;
    if (t + 1 < NT) fetch(q0 + 32);
    f32x4 dq2[2] = {f32x4{}, f32x4{}};
#pragma unroll
    for (int hf = 0; hf < NH; ++hf) {
#pragma unroll
      for (int kk = 0; kk < KH; ++kk) {
        const int kb = hf * KH + kk;
        const int key0 = kw0 + 32 * kb;
        f32x16 sacc, pacc;
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          // Q / dO row fragments re-read per key block (LDS bandwidth to spare; registers not)
          const bf16x8 qa = swz_row_read(sm.Qs, 0, r, 2 * c + hh), kr = swz_row_read(sm.Ks, key0, r, 2 * c + hh);
          const bf16x8 oa = swz_row_read(sm.Os, 0, r, 2 * c + hh), vr = swz_row_read(sm.Vs, key0, r, 2 * c + hh);
          if (c == 0) { mfma32_v0(sacc, qa, kr); mfma32_v0(pacc, oa, vr); }
          else { mfma32_v(sacc, qa, kr); mfma32_v(pacc, oa, vr); }
        }
        mfma_vgpr_wait(sacc, pacc);
        uint64_t mk[16];
        if constexpr (DROP) {
          const cu64* mp = (const cu64*)(uintptr_t)(a.maskA + ((size_t)bh * a.W + min(w * NKB + kb, a.W - 1)) * Sp +
                                                    keep_off(q0, Sp));
#pragma unroll
          for (int i = 0; i < 16; ++i) mk[i] = mp[i];
        }
        // -lse*log2e / -delta of this lane's 16 accumulator rows (rows 8g + 4hh + 0..3)
        f32x4 L4[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) L4[g] = *reinterpret_cast<const f32x4*>(&sm.lse_s[8 * g + 4 * hh]);
        const f32x2 sc2v = pk2(sc2, sc2);
#pragma unroll
        for (int i = 0; i < 16; i += 2) {
          const f32x2 x = pk_fma(pk2(sacc[i], sacc[i + 1]), sc2v, pk2(L4[i >> 2][i & 3], L4[i >> 2][(i & 3) + 1]));
          sacc[i] = fexp2(x.x);
          sacc[i + 1] = fexp2(x.y);
        }
        f32x4 D4[4];
#pragma unroll
        for (int g = 0; g < 4; ++g) D4[g] = *reinterpret_cast<const f32x4*>(&sm.del_s[8 * g + 4 * hh]);
#pragma unroll
        for (int i = 0; i < 16; i += 2) {
          const f32x2 nd = pk2(D4[i >> 2][i & 3], D4[i >> 2][(i & 3) + 1]);
          if constexpr (DROP) {
            const f32x2 tt = pk_fma(pk2(sel_keep(pacc[i], mk[i]), sel_keep(pacc[i + 1], mk[i + 1])),
                                    pk2(inv_keep, inv_keep), nd);
            const f32x2 ds = pk2(sacc[i], sacc[i + 1]) * tt;                 // dS
            pacc[i] = ds.x;
            pacc[i + 1] = ds.y;
            sacc[i] = sel_keep(sacc[i], mk[i]);                              // P*mask (dV)
            sacc[i + 1] = sel_keep(sacc[i + 1], mk[i + 1]);
          } else {
            const f32x2 ds = pk2(sacc[i], sacc[i + 1]) * (pk2(pacc[i], pacc[i + 1]) + nd);
            pacc[i] = ds.x;
            pacc[i + 1] = ds.y;
          }
        }
        bf16* dsrow = sm.DS + ((w * KH + kk) * 32 + r) * DSP + 4 * hh;
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          bf16x8 pb, sb;
#pragma unroll
          for (int j = 0; j < 8; ++j) { pb[j] = (bf16)sacc[8 * s2 + j]; sb[j] = (bf16)pacc[8 * s2 + j]; }
#pragma unroll
          for (int d = 0; d < NDB; ++d) {
            if constexpr (NKB == 4) {
              mfma32_a(dv[kb][d], tr_operand_swz(sm.Os, 16 * s2, d * 32, lane), pb);
              mfma32_a(dk[kb][d], tr_operand_swz(sm.Qs, 16 * s2, d * 32, lane), sb);
            } else {
              dv[kb][d] = mfma32(tr_operand_swz(sm.Os, 16 * s2, d * 32, lane), pb, dv[kb][d]);
              dk[kb][d] = mfma32(tr_operand_swz(sm.Qs, 16 * s2, d * 32, lane), sb, dk[kb][d]);
            }
          }
          // dS^T image: registers 8 s2 + 4 jj .. +3 are queries 8 (2 s2 + jj) + 4 hh + 0..3
          *reinterpret_cast<bf16x4*>(dsrow + 16 * s2) = __builtin_shufflevector(sb, sb, 0, 1, 2, 3);
          *reinterpret_cast<bf16x4*>(dsrow + 16 * s2 + 8) = __builtin_shufflevector(sb, sb, 4, 5, 6, 7);
        }
        // one key block's live range at a time: the dK/dV accumulators take half the register file
        __builtin_amdgcn_sched_barrier(0);
      }
      if constexpr (NKB == 4) {
        // the asm MFMAs' results land up to 12 wait states after their issue, which hipcc does not
        // know: wait them out before the barrier (below S = 512 the builtin form is used: enough
        // registers, and hipcc pads its own hazards)
        asm volatile("s_nop 15");
      }
      __syncthreads();   // the round's dS^T image complete
      // dQ^T rows 16w .. 16w+15 x the tile's 32 queries over the round's 4 KH 32 keys
#pragma unroll 2
      for (int k0 = 0; k0 < DSR; k0 += 32) {
        const int key = (k0 / (KH * 32)) * KPW + hf * KH * 32 + (k0 % (KH * 32)) + 8 * g16 + qq;
        const bf16* ka = sm.Ks + key * 64 + 8 * ((kcol >> 3) ^ swz64(key)) + (kcol & 7);
        const bf16* kb4 = sm.Ks + (key + 4) * 64 + 8 * ((kcol >> 3) ^ swz64(key + 4)) + (kcol & 7);
        const bf16x8 A = cat(tr_read(ka), tr_read(kb4));
        const int lr = k0 + 8 * g16 + qq;
#pragma unroll
        for (int qh = 0; qh < 2; ++qh) {
          const bf16* dp = sm.DS + lr * DSP + 16 * qh + 4 * pp;
          mfma16_v(dq2[qh], A, cat(tr_read(dp), tr_read(dp + 4 * DSP)));
        }
      }
      asm volatile("s_nop 7" : "+v"(dq2[0]), "+v"(dq2[1]));
      if (hf == NH - 1 && t + 1 < NT) stage();
      __syncthreads();   // the image consumed (and, after the last round, the next tile staged)
    }
    if constexpr (NKB == 4) {
      // pin every accumulator in the accumulator file at the loop back edge: no compiler copy of
      // one can be placed between an asm MFMA and the wait above
#pragma unroll
      for (int kb = 0; kb < NKB; ++kb)
        asm volatile("" : "+a"(dk[kb][0]), "+a"(dk[kb][1]), "+a"(dv[kb][0]), "+a"(dv[kb][1]));
    }
    // lane: query q0 + 16 qh + l16, head dims 16w + 4 g16 + 0..3
    float cs[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int qh = 0; qh < 2; ++qh) {
      bf16x4 v4;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        v4[j] = (bf16)(dq2[qh][j] * a.scale);
        cs[j] += (float)v4[j];
      }
      *reinterpret_cast<bf16x4*>(a.dq + (size_t)(b * S + q0 + 16 * qh + l16) * a.ld + h * D + 16 * w + 4 * g16) = v4;
    }
    if (a.bias_part) {
      // column sums over the tile's 32 queries: the 16 lanes of a group x both halves
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        cs[j] += __shfl_xor(cs[j], 1, 64);
        cs[j] += __shfl_xor(cs[j], 2, 64);
        cs[j] += __shfl_xor(cs[j], 4, 64);
        cs[j] += __shfl_xor(cs[j], 8, 64);
      }
      if (l16 == 0)
        *reinterpret_cast<f32x4*>(a.bias_part + ((size_t)b * (S / 32) + t) * (3 * a.H * D) + h * D + 16 * w + 4 * g16) =
            f32x4{cs[0], cs[1], cs[2], cs[3]};
    }
  }
  if constexpr (NKB == 4) {
    // the accumulators stay pinned in the accumulator file into the epilogue (without this hipcc
    // re-homed them and spilled)
#pragma unroll
    for (int kb = 0; kb < NKB; ++kb)
      asm volatile("s_nop 0" : "+a"(dk[kb][0]), "+a"(dk[kb][1]), "+a"(dv[kb][0]), "+a"(dv[kb][1]));
  }
  const float dv_scale = inv_keep;   // the dropped P fed to dV carried keep bits only
  // epilogue one accumulator tile at a time (the sched barriers keep the compiler from
  // interleaving them, whose pressure made it spill the dK/dV accumulators inside the main loop)
  auto put = [&](const f32x16 (&acc)[NDB], float sc, bf16* dst, int colbase, int kb) {
    if (a.bias_part) {
      float vk[32];
#pragma unroll
      for (int d = 0; d < NDB; ++d)
#pragma unroll
        for (int i = 0; i < 16; ++i) vk[16 * d + i] = (float)(bf16)(acc[d][i] * sc);
      const float sk = colsum32(vk, r);
      a.bias_part[((size_t)b * (S / 32) + w * NKB + kb) * (3 * a.H * D) + colbase + h * D + colsum_col(r, hh)] = sk;
    }
    bf16* p = dst + (size_t)(b * S + kw0 + 32 * kb + r) * a.ld + h * D;
#pragma unroll
    for (int d = 0; d < NDB; ++d)
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        bf16x4 k4;
#pragma unroll
        for (int j = 0; j < 4; ++j) k4[j] = (bf16)(acc[d][4 * gq + j] * sc);
        *reinterpret_cast<bf16x4*>(p + d * 32 + 8 * gq + 4 * hh) = k4;
      }
  };
#pragma unroll
  for (int kb = 0; kb < NKB; ++kb) {
    put(dk[kb], a.scale, a.dk, a.H * D, kb);
    __builtin_amdgcn_sched_barrier(0);
    put(dv[kb], dv_scale, a.dv, 2 * a.H * D, kb);
    __builtin_amdgcn_sched_barrier(0);
  }
}

// Eight-wave form of the fused backward (S = 256 or 512): two waves per SIMD, so one wave's
// softmax VALU runs under the other's MFMAs (the 4-wave form's single wave per SIMD serialises its
// MFMA -> VALU -> MFMA chain: 1.6 ms against the split pair's 1.18 ms at B 256 x H 12).  Wave w
// owns KPW = S / 8 keys (dK^T / dV^T of one or two 32-key blocks: 64 or 128 accumulator
// registers); one key block per wave per round (dS^T image of 256 keys, 18 KiB); the dQ^T
// 16x16x32 blocks: wave w takes head dims 16 (w & 3) .. +15 of query half w >> 2 over every key
// of the round, so each block is a complete sum; the query-half pairs combine only their
// qkv-bias column sums, through LDS.  The tile staging (Q, dO, O rows, lse, delta) runs on the
// first 256 threads.
template <int NKBW, bool DROP>
__global__ void __launch_bounds__(512, 1) attn_bwd_fused8_kernel(BwdArgs a) {
  constexpr int D = 64, NC = 4, NDB = 2, KPW = 32 * NKBW, SK = 8 * KPW, NT = SK / 32, NH = NKBW;
  constexpr int DSP = 36, DSR = 8 * 32;
  struct Smem {
    float lse_s[32], del_s[32];
    float csq[64];           // query-half-1 dQ column sums, per head dim
    bf16 Qs[32 * 64];
    bf16 Os[32 * 64];
    bf16 DS[DSR * DSP];
    bf16 Ks[SK * 64];
    bf16 Vs[SK * 64];
  };
  __shared__ __attribute__((aligned(16))) Smem sm;

  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6), hh = lane >> 5,
            r = lane & 31;
  const bool stager = tid < 256;
  const int bh = blockIdx.x, b = bh / a.H, h = bh % a.H;
  const int S = a.S;   // == SK (host-checked)
  const float sc2 = a.scale * kLog2e;
  const float inv_keep = DROP ? 1.f / (1.f - a.p) : 1.f;
  const int kw0 = w * KPW;
  const int Sp = 32 * a.W;
  const float* lseb = a.lse + (size_t)bh * S;
  const RowSrc qsrc = row_src<D>(a.q + (size_t)b * S * a.ld + h * D, a.ld, S);
  const RowSrc dsrc = row_src<D>(a.dout + (size_t)b * S * a.ldo + h * D, a.ldo, S);
  const RowSrc osrc = row_src<D>(a.o + (size_t)b * S * a.ldo + h * D, a.ldo, S);
  if (stager) {
    const RowSrc ksrc = row_src<D>(a.k + (size_t)b * S * a.ld + h * D, a.ld, S);
    const RowSrc vsrc = row_src<D>(a.v + (size_t)b * S * a.ld + h * D, a.ld, S);
#pragma unroll
    for (int part = 0; part < SK / 128; ++part) {
      TileLoader<D, 128> kl, vl;
      kl.load(ksrc, part * 128);
      vl.load(vsrc, part * 128);
      kl.store_swz(sm.Ks + part * 128 * 64);
      vl.store_swz(sm.Vs + part * 128 * 64);
    }
  }
  TileLoader<D, 32> ql, dl, ol;
  float lse_n = 0.f;
  auto fetch = [&](int q0) {
    if (!stager) return;
    ql.load(qsrc, q0);
    dl.load(dsrc, q0);
    ol.load(osrc, q0);
    if (tid < 32) lse_n = lseb[q0 + tid];
  };
  auto stage = [&]() {
    if (!stager) return;
    float part = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) part = fmaf((float)dl.reg[0][j], (float)ol.reg[0][j], part);
    part += __shfl_xor(part, 1, 64);
    part += __shfl_xor(part, 2, 64);
    part += __shfl_xor(part, 4, 64);
    ql.store_swz(sm.Qs);
    dl.store_swz(sm.Os);
    if ((tid & 7) == 0) sm.del_s[tid >> 3] = -part;
    if (tid < 32) sm.lse_s[tid] = -lse_n * kLog2e;
  };
  fetch(0);
  stage();

  f32x16 dk[NKBW][NDB], dv[NKBW][NDB];
#pragma unroll
  for (int kb = 0; kb < NKBW; ++kb)
#pragma unroll
    for (int d = 0; d < NDB; ++d) { dk[kb][d] = f32x16{}; dv[kb][d] = f32x16{}; }
  const int g16 = lane >> 4, l16 = lane & 15, qq = l16 >> 2, pp = l16 & 3;
  const int dd = w & 3, qh = w >> 2;
  const int kcol = 16 * dd + 4 * pp;
  __syncthreads();

  for (int t = 0; t < NT; ++t) {
    const int q0 = t * 32;
    if (t + 1 < NT) fetch(q0 + 32);
    f32x4 dq1 = f32x4{};
#pragma unroll
    for (int kb = 0; kb < NH; ++kb) {
      const int key0 = kw0 + 32 * kb;
      f32x16 sacc = f32x16{}, pacc = f32x16{};
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        sacc = mfma32(swz_row_read(sm.Qs, 0, r, 2 * c + hh), swz_row_read(sm.Ks, key0, r, 2 * c + hh), sacc);
        pacc = mfma32(swz_row_read(sm.Os, 0, r, 2 * c + hh), swz_row_read(sm.Vs, key0, r, 2 * c + hh), pacc);
      }
      // fragments read just ahead of their MFMAs (4 reads, 2 MFMAs per group): hoisting all 16
      // reads made this block the register peak (dK/dV accumulators + 64 fragment registers)
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
      }
      uint64_t mk[16];
      if constexpr (DROP) {
        const cu64* mp = (const cu64*)(uintptr_t)(a.maskA + ((size_t)bh * a.W + min(w * NKBW + kb, a.W - 1)) * Sp +
                                                  keep_off(q0, Sp));
#pragma unroll
        for (int i = 0; i < 16; ++i) mk[i] = mp[i];
      }
      f32x4 L4[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) L4[g] = *reinterpret_cast<const f32x4*>(&sm.lse_s[8 * g + 4 * hh]);
      const f32x2 sc2v = pk2(sc2, sc2);
#pragma unroll
      for (int i = 0; i < 16; i += 2) {
        const f32x2 x = pk_fma(pk2(sacc[i], sacc[i + 1]), sc2v, pk2(L4[i >> 2][i & 3], L4[i >> 2][(i & 3) + 1]));
        sacc[i] = fexp2(x.x);
        sacc[i + 1] = fexp2(x.y);
      }
      f32x4 D4[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) D4[g] = *reinterpret_cast<const f32x4*>(&sm.del_s[8 * g + 4 * hh]);
#pragma unroll
      for (int i = 0; i < 16; i += 2) {
        const f32x2 nd = pk2(D4[i >> 2][i & 3], D4[i >> 2][(i & 3) + 1]);
        if constexpr (DROP) {
          const f32x2 tt = pk_fma(pk2(sel_keep(pacc[i], mk[i]), sel_keep(pacc[i + 1], mk[i + 1])),
                                  pk2(inv_keep, inv_keep), nd);
          const f32x2 ds = pk2(sacc[i], sacc[i + 1]) * tt;
          pacc[i] = ds.x;
          pacc[i + 1] = ds.y;
          sacc[i] = sel_keep(sacc[i], mk[i]);
          sacc[i + 1] = sel_keep(sacc[i + 1], mk[i + 1]);
        } else {
          const f32x2 ds = pk2(sacc[i], sacc[i + 1]) * (pk2(pacc[i], pacc[i + 1]) + nd);
          pacc[i] = ds.x;
          pacc[i + 1] = ds.y;
        }
      }
      bf16* dsrow = sm.DS + (w * 32 + r) * DSP + 4 * hh;
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        bf16x8 pb, sb;
#pragma unroll
        for (int j = 0; j < 8; ++j) { pb[j] = (bf16)sacc[8 * s2 + j]; sb[j] = (bf16)pacc[8 * s2 + j]; }
#pragma unroll
        for (int d = 0; d < NDB; ++d) {
          dv[kb][d] = mfma32(tr_operand_swz(sm.Os, 16 * s2, d * 32, lane), pb, dv[kb][d]);
          dk[kb][d] = mfma32(tr_operand_swz(sm.Qs, 16 * s2, d * 32, lane), sb, dk[kb][d]);
        }
        *reinterpret_cast<bf16x4*>(dsrow + 16 * s2) = __builtin_shufflevector(sb, sb, 0, 1, 2, 3);
        *reinterpret_cast<bf16x4*>(dsrow + 16 * s2 + 8) = __builtin_shufflevector(sb, sb, 4, 5, 6, 7);
      }
      __syncthreads();   // the round's dS^T image complete
      // dQ^T rows 16 dd .. +15 x queries 16 qh .. +15 over the round's 256 keys (32 of each wave)
#pragma unroll 1
      for (int k0 = 0; k0 < DSR; k0 += 32) {
        const int key = (k0 / 32) * KPW + kb * 32 + 8 * g16 + qq;
        const bf16* ka = sm.Ks + key * 64 + 8 * ((kcol >> 3) ^ swz64(key)) + (kcol & 7);
        const bf16* kb4 = sm.Ks + (key + 4) * 64 + 8 * ((kcol >> 3) ^ swz64(key + 4)) + (kcol & 7);
        const int lr = k0 + 8 * g16 + qq;
        const bf16* dp = sm.DS + lr * DSP + 16 * qh + 4 * pp;
        dq1 = mfma16(cat(tr_read(ka), tr_read(kb4)), cat(tr_read(dp), tr_read(dp + 4 * DSP)), dq1);
      }
      float cs[4] = {0.f, 0.f, 0.f, 0.f};
      if (kb == NH - 1) {
        // lane: query q0 + 16 qh + l16, head dims 16 dd + 4 g16 + 0..3 -- a complete sum
        bf16x4 v4;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          v4[j] = (bf16)(dq1[j] * a.scale);
          cs[j] = (float)v4[j];
        }
        *reinterpret_cast<bf16x4*>(a.dq + (size_t)(b * S + q0 + 16 * qh + l16) * a.ld + h * D + 16 * dd + 4 * g16) = v4;
        if (a.bias_part) {
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            cs[j] += __shfl_xor(cs[j], 1, 64);
            cs[j] += __shfl_xor(cs[j], 2, 64);
            cs[j] += __shfl_xor(cs[j], 4, 64);
            cs[j] += __shfl_xor(cs[j], 8, 64);
          }
          if (qh == 1 && l16 == 0)
            *reinterpret_cast<f32x4*>(&sm.csq[16 * dd + 4 * g16]) = f32x4{cs[0], cs[1], cs[2], cs[3]};
        }
        if (t + 1 < NT) stage();
      }
      __syncthreads();   // the image consumed (after the last round: the next tile staged, the
                         // query-half-1 column sums published)
      if (kb == NH - 1 && a.bias_part && qh == 0 && l16 == 0) {
        const f32x4 o4 = *reinterpret_cast<const f32x4*>(&sm.csq[16 * dd + 4 * g16]);
        *reinterpret_cast<f32x4*>(a.bias_part + ((size_t)b * (S / 32) + t) * (3 * a.H * D) + h * D + 16 * dd + 4 * g16) =
            f32x4{cs[0] + o4[0], cs[1] + o4[1], cs[2] + o4[2], cs[3] + o4[3]};
      }
    }
  }
  const float dv_scale = inv_keep;
  auto put = [&](const f32x16 (&acc)[NDB], float sc, bf16* dst, int colbase, int kb) {
    if (a.bias_part) {
      float vk[32];
#pragma unroll
      for (int d = 0; d < NDB; ++d)
#pragma unroll
        for (int i = 0; i < 16; ++i) vk[16 * d + i] = (float)(bf16)(acc[d][i] * sc);
      const float sk = colsum32(vk, r);
      a.bias_part[((size_t)b * (S / 32) + w * NKBW + kb) * (3 * a.H * D) + colbase + h * D + colsum_col(r, hh)] = sk;
    }
    bf16* p = dst + (size_t)(b * S + kw0 + 32 * kb + r) * a.ld + h * D;
#pragma unroll
    for (int d = 0; d < NDB; ++d)
#pragma unroll
      for (int gq = 0; gq < 4; ++gq) {
        bf16x4 k4;
#pragma unroll
        for (int j = 0; j < 4; ++j) k4[j] = (bf16)(acc[d][4 * gq + j] * sc);
        *reinterpret_cast<bf16x4*>(p + d * 32 + 8 * gq + 4 * hh) = k4;
      }
  };
#pragma unroll
  for (int kb = 0; kb < NKBW; ++kb) {
    put(dk[kb], a.scale, a.dk, a.H * D, kb);
    __builtin_amdgcn_sched_barrier(0);
    put(dv[kb], dv_scale, a.dv, 2 * a.H * D, kb);
    __builtin_amdgcn_sched_barrier(0);
  }
}

#endif  // DTD_ATTN_FUSED_BWD

}  // namespace

// Waves per SIMD the head_dim-64 kernels are compiled for (register budget 512/OCC per lane):
// fwd, dK/dV, dQ.  The kernels are latency-bound (dependent MFMA -> softmax -> MFMA chains per
// wave), so waves per SIMD matter more than in-flight tile loads: at 3 waves the forward and dQ
// keep ONE register set of the next K/V tile in flight (RING = 1, 166-168 VGPRs, no spills)
// instead of two -- forward 233 -> 188 us at B=128 (scripts/bench_attn.py), +1.4 % whole-step
// throughput same-box (profiles/r1_ab_attn_occ.jsonl).  dK/dV stays at 2 (255 VGPRs).
// Override with DTD_ATTN_OCC="f,kv,q" for tuning runs.
static int occupancy(int which) {
  static const int defaults[3] = {3, 2, 3};
  const char* env = getenv("DTD_ATTN_OCC");
  if (!env) return defaults[which];
  int v[3] = {defaults[0], defaults[1], defaults[2]};
  sscanf(env, "%d,%d,%d", &v[0], &v[1], &v[2]);
  return v[which];
}

// Forward form (D = 64): DTD_ATTN_FWD=pipe selects attn_fwd_pipe_kernel (S(t+1) MFMAs under
// tile t's softmax); anything else the single-stage attn_fwd_kernel.
static bool fwd_pipe() {
  const char* e = getenv("DTD_ATTN_FWD");
  return e != nullptr && strcmp(e, "pipe") == 0;
}

// DTD_ATTN_FWD_PK=1: the packed-fp32 softmax forms of attn_fwd_kernel and attn_bwd_dq_kernel (PK)
static bool fwd_pk() {
  const char* e = getenv("DTD_ATTN_FWD_PK");
  return e != nullptr && e[0] == '1';
}

// Keys per K/V tile of the dQ kernel (which=1; the forward uses 64): 64 (37 KB LDS) or 128
// (74 KB LDS; half the barriers per key, but 2 waves/SIMD at most).  64 with the 3-wave kernel
// (128-key dQ at 2 waves: 3 % slower backward).  Measured and dropped: 128-key forward tiles
// (spill at 2 waves), 32-key forward tiles at 4 waves/SIMD (120 VGPRs; 7 % slower than 64 at 3).
// DTD_ATTN_TILE="f,q" overrides for tuning runs.
static int tile_keys(int which) {
  static const int defaults[2] = {64, 64};
  const char* env = getenv("DTD_ATTN_TILE");
  if (!env) return defaults[which];
  int v[2] = {defaults[0], defaults[1]};
  sscanf(env, "%d,%d", &v[0], &v[1]);
  return v[which];
}

// Backward form (D = 64, non-causal, no ALiBi, S % 128 == 0, S <= 512): DTD_ATTN_BWD=fused selects
// attn_bwd_fused_kernel (one workgroup per head, dQ reduced in LDS); anything else the dQ + dK/dV
// kernel pair.
// form: 0 = split pair, 1 = fused (8 waves at S = 512, else 4), 2 = fused, 4 waves always.
// Measured at B 256 x H 12 x S 512 (scripts/bench_attn.py): split 1.16-1.17 ms, fused 8-wave
// 1.18 ms, fused 4-wave 1.60 ms -- the split pair stays the default.
// DTD_ATTN_BWD=fused / fused4 / split; dtd_attn_set_bwd_form at run time.
static int g_bwd_form = -1;
static int bwd_form() {
  if (g_bwd_form < 0) {
    const char* e = getenv("DTD_ATTN_BWD");
    g_bwd_form = !e ? 0 : strcmp(e, "fused") == 0 ? 1 : strcmp(e, "fused4") == 0 ? 2 : 0;
  }
  return g_bwd_form;
}
static bool bwd_fused() { return bwd_form() != 0; }
static bool bwd_fused8() { return bwd_form() == 1; }

// q,k,v,o: bf16 views with row stride ld (q/k/v) / ldo (o); lse: [B,H,S] fp32.
// masks: [2][B*H*S*W] uint32 (W = ceil(S/32)) written here when p > 0 (read by the backward).
// The tile loads address one (batch, head)'s rows through 32-bit buffer offsets (RowSrc).
static bool offsets_fit(int S, int ld, int ldo) {
  const long long lim = 0x7fffffffLL;
  const long long W = (S + 31) / 32;
  return (long long)S * ld * 2 < lim && (long long)S * ldo * 2 < lim && 32 * W * W * 4 < lim;
}

DTD_EXPORT int dtd_attn_fwd(const void* q, const void* k, const void* v, void* o, float* lse, const float* slopes,
                            uint32_t* masks, int B, int S, int H, int D, int ld, int ldo, int causal, float scale,
                            float p, const uint64_t* rng, uint32_t sid, hipStream_t s) {
  if (B * S * H == 0) return 0;
  if (!offsets_fit(S, ld, ldo)) return (int)hipErrorInvalidValue;
  const int W = (S + 31) / 32;
  uint32_t* mA = nullptr;
  if (p > 0.f) {
    if (!masks) return (int)hipErrorInvalidValue;
    mA = masks;
    // rng == nullptr: the masks were generated ahead of time by dtd_attn_masks (on a side
    // stream, overlapping the QKV GEMM)
    if (rng) {
      uint32_t* mB = masks + (size_t)B * H * (32 * W) * W;
      hipLaunchKernelGGL(attn_mask_kernel, dim3((S + 255) / 256, B * H), dim3(256), 0, s, mA, mB, S, W, rng, sid,
                         keep_threshold(p));
    }
  }
  const char* thr_env = getenv("DTD_ATTN_RESCALE_THR");
  const float thr = thr_env ? (float)atof(thr_env) : kRescaleThr;
  const uint32_t* mBk = mA ? mA + (size_t)B * H * (32 * W) * W : nullptr;
  FwdArgs a{(const bf16*)q, (const bf16*)k, (const bf16*)v, (bf16*)o, lse, slopes, mA, mBk, B, S, H, ld, ldo, causal, W,
            scale, p, thr};
  dim3 grid((S + 127) / 128, B * H);
  if (D == 64 && fwd_pipe()) {
    // two score tiles live: 198 VGPRs, 2 waves / SIMD (at 3 it spills)
    hipLaunchKernelGGL((attn_fwd_pipe_kernel<64, 2, 64>), grid, dim3(256), 0, s, a);
  } else if (D == 64) {
    const int o = occupancy(0);
    if (o >= 3 && fwd_pk()) hipLaunchKernelGGL((attn_fwd_kernel<64, 3, 64, 1, true>), grid, dim3(256), 0, s, a);
    else if (o >= 3) hipLaunchKernelGGL((attn_fwd_kernel<64, 3, 64, 1>), grid, dim3(256), 0, s, a);
    else if (o == 2) hipLaunchKernelGGL((attn_fwd_kernel<64, 2, 64, 2>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((attn_fwd_kernel<64, 1, 64, 2>), grid, dim3(256), 0, s, a);
  } else if (D == 128) {
    hipLaunchKernelGGL((attn_fwd_kernel<128, 1, 64, 2>), grid, dim3(256), 0, s, a);
  } else {
    return (int)hipErrorInvalidValue;
  }
  DTD_LAUNCH_CHECK();
}

// 0 = the dQ + dK/dV pair, 1 = fused where it applies, 2 = fused, 4-wave form; returns the previous
DTD_EXPORT int dtd_attn_fused_bwd_built() { return DTD_ATTN_FUSED_BWD; }

DTD_EXPORT int dtd_attn_set_bwd_form(int f) {
  const int old = bwd_form();
  g_bwd_form = f < 0 || f > 2 ? 0 : f;
  return old;
}

// Dropout keep-bit masks of one attention call ([2][B*H*S*W] uint32), VALU-only: launched on a
// side stream so it runs concurrently with the (MFMA-bound) QKV projection GEMM.
DTD_EXPORT int dtd_attn_masks(uint32_t* masks, int B, int S, int H, float p, const uint64_t* rng, uint32_t sid,
                              hipStream_t s) {
  if (B * S * H == 0 || p <= 0.f) return 0;
  if (!masks || !rng) return (int)hipErrorInvalidValue;
  const int W = (S + 31) / 32;
  hipLaunchKernelGGL(attn_mask_kernel, dim3((S + 255) / 256, B * H), dim3(256), 0, s, masks,
                     masks + (size_t)B * H * (32 * W) * W, S, W, rng, sid, keep_threshold(p));
  DTD_LAUNCH_CHECK();
}

template <int D, int OCC, int BM>
static void launch_dkdv(dim3 grid, hipStream_t s, const BwdArgs& a) {
  const bool drop = a.maskB != nullptr, alibi = a.slopes != nullptr;
  if (!a.causal && a.S % 128 == 0 && !alibi) {   // no block needs the mask (BERT: S = 512)
    if (drop) hipLaunchKernelGGL((attn_bwd_dkdv_kernel<D, OCC, BM, true, false, false>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((attn_bwd_dkdv_kernel<D, OCC, BM, false, false, false>), grid, dim3(256), 0, s, a);
    return;
  }
  if (drop && alibi) hipLaunchKernelGGL((attn_bwd_dkdv_kernel<D, OCC, BM, true, true>), grid, dim3(256), 0, s, a);
  else if (drop) hipLaunchKernelGGL((attn_bwd_dkdv_kernel<D, OCC, BM, true, false>), grid, dim3(256), 0, s, a);
  else if (alibi) hipLaunchKernelGGL((attn_bwd_dkdv_kernel<D, OCC, BM, false, true>), grid, dim3(256), 0, s, a);
  else hipLaunchKernelGGL((attn_bwd_dkdv_kernel<D, OCC, BM, false, false>), grid, dim3(256), 0, s, a);
}

// dq/dk/dv: bf16 views with row stride ld into dqkv.  `delta` is [B,H,S] fp32 scratch.
DTD_EXPORT int dtd_attn_bwd(const void* q, const void* k, const void* v, const void* o, const void* dout,
                            const float* lse, float* delta, const uint32_t* masks, void* dq, void* dk, void* dv,
                            const float* slopes, int B, int S, int H, int D, int ld, int ldo, int causal, float scale,
                            float p, float* bias_part, hipStream_t s) {
  if (B * S * H == 0) return 0;
  if (D != 64 && D != 128) return (int)hipErrorInvalidValue;
  if (!offsets_fit(S, ld, ldo)) return (int)hipErrorInvalidValue;
  const int W = (S + 31) / 32;
  const uint32_t* mA = (p > 0.f) ? masks : nullptr;
  const uint32_t* mB = (p > 0.f) ? masks + (size_t)B * H * (32 * W) * W : nullptr;
  if (p > 0.f && !masks) return (int)hipErrorInvalidValue;
  dim3 grid((S + 127) / 128, B * H);
  BwdArgs a{(const bf16*)q, (const bf16*)k, (const bf16*)v, (const bf16*)dout, lse, delta, (const bf16*)o,
            (bf16*)dq, (bf16*)dk, (bf16*)dv, slopes, mA, mB, B, S, H, ld, ldo, causal, W, scale, p,
            D == 64 ? bias_part : nullptr};
#if DTD_ATTN_FUSED_BWD
  if (D == 64 && !causal && !slopes && S % 128 == 0 && S <= 512 && bwd_fused()) {
    const bool drop = mA != nullptr;
    const dim3 g1(B * H);
    // (the one-key-block-per-wave instantiation, S = 256, gave wrong, run-to-run varying dS rows
    // with dropout on the box -- unresolved, so it is not launched: S = 256 takes the 4-wave form)
    if (S == 512 && bwd_fused8()) {
      if (drop) hipLaunchKernelGGL((attn_bwd_fused8_kernel<2, true>), g1, dim3(512), 0, s, a);
      else hipLaunchKernelGGL((attn_bwd_fused8_kernel<2, false>), g1, dim3(512), 0, s, a);
      DTD_LAUNCH_CHECK();
    }
    switch (S / 128) {
      case 1: if (drop) hipLaunchKernelGGL((attn_bwd_fused_kernel<1, true>), g1, dim3(256), 0, s, a);
              else hipLaunchKernelGGL((attn_bwd_fused_kernel<1, false>), g1, dim3(256), 0, s, a); break;
      case 2: if (drop) hipLaunchKernelGGL((attn_bwd_fused_kernel<2, true>), g1, dim3(256), 0, s, a);
              else hipLaunchKernelGGL((attn_bwd_fused_kernel<2, false>), g1, dim3(256), 0, s, a); break;
      case 3: if (drop) hipLaunchKernelGGL((attn_bwd_fused_kernel<3, true>), g1, dim3(256), 0, s, a);
              else hipLaunchKernelGGL((attn_bwd_fused_kernel<3, false>), g1, dim3(256), 0, s, a); break;
      default: if (drop) hipLaunchKernelGGL((attn_bwd_fused_kernel<4, true>), g1, dim3(256), 0, s, a);
               else hipLaunchKernelGGL((attn_bwd_fused_kernel<4, false>), g1, dim3(256), 0, s, a); break;
    }
    DTD_LAUNCH_CHECK();
  }
#endif
  // dQ first: it also produces delta = rowsum(dO * O), which the dK/dV kernel then reads
  if (D == 64) {
    const int o = occupancy(2);
    if (tile_keys(1) == 128) hipLaunchKernelGGL((attn_bwd_dq_kernel<64, 2, 128, 2>), grid, dim3(256), 0, s, a);
    else if (o >= 3 && fwd_pk()) hipLaunchKernelGGL((attn_bwd_dq_kernel<64, 3, 64, 1, true>), grid, dim3(256), 0, s, a);
    else if (o >= 3) hipLaunchKernelGGL((attn_bwd_dq_kernel<64, 3, 64, 1>), grid, dim3(256), 0, s, a);
    else if (o == 2) hipLaunchKernelGGL((attn_bwd_dq_kernel<64, 2, 64, 2>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((attn_bwd_dq_kernel<64, 1, 64, 2>), grid, dim3(256), 0, s, a);
    // query tile of the dK/dV loop: 128 rows halves the barriers / exposed load latency per
    // query row at 2 blocks per CU (75 KB LDS each); DTD_ATTN_DKDV_BM=64 selects the old tile
    const int bm = getenv("DTD_ATTN_DKDV_BM") ? atoi(getenv("DTD_ATTN_DKDV_BM")) : 128;
    if (bm == 128 && occupancy(1) == 1) launch_dkdv<64, 1, 128>(grid, s, a);
    else if (bm == 128) launch_dkdv<64, 2, 128>(grid, s, a);
    else if (occupancy(1) >= 2) launch_dkdv<64, 2, 64>(grid, s, a);
    else launch_dkdv<64, 1, 64>(grid, s, a);
  } else {
    hipLaunchKernelGGL((attn_bwd_dq_kernel<128, 1, 64, 2>), grid, dim3(256), 0, s, a);
    launch_dkdv<128, 1, 64>(grid, s, a);
  }
  DTD_LAUNCH_CHECK();
}
