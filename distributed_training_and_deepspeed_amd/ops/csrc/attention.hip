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
// operand permutes its k order (element j of half h <-> row 16s + 8(j>>2) + 4h + (j&3)), so
// V is staged transposed in LDS and read in that permuted order (two 8-byte reads).
//
// Backward (FA2 structure, "key on the lane"): one workgroup = 4 waves = 128 keys of one
// (batch, head); each wave keeps its 32 keys' K/V fragments in registers and dK^T/dV^T
// accumulators for the whole sweep over query tiles; P is recomputed from the forward LSE;
// S and dP accumulators are the B operands of dV^T += dO^T.P and dK^T += Q^T.dS; dS crosses
// LDS once for dQ = dS.K, which is accumulated across key blocks with fp32 atomics into a
// [B,H,S,D] buffer (rounded to bf16 once at the end).
//
// Features: causal mask, ALiBi (bias = slope_h * key), attention-probability dropout with the
// counter RNG (mask index ((b*H+h)*S + q)*S + key, regenerated in backward), arbitrary S
// (bounds-masked), head_dim 64 or 128.  q/k/v/o are strided views (row stride `ld`) into the
// fused [B*S, 3*H*D] projection output, so no transpose/copy kernels are needed.
#include "common.h"

using namespace dtd;

typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace {

constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;

__device__ __forceinline__ f32x16 mfma32(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ int crow(int i, int h) { return (i & 3) + 8 * (i >> 2) + 4 * h; }

__device__ __forceinline__ float drop_keep(const DropoutRng& g, uint64_t e, uint32_t thr) {
  const uint32_t b = g.bits(e >> 1);
  const uint32_t h16 = (e & 1) ? (b >> 16) : (b & 0xffffu);
  return h16 >= thr ? 1.f : 0.f;
}

struct FwdArgs {
  const bf16* q; const bf16* k; const bf16* v; bf16* o; float* lse; const float* slopes;
  int B, S, H, ld, ldo, causal;
  float scale, p; const uint64_t* rng; uint32_t sid;
};

// grid: (ceil(S/128), B*H); block 256 = 4 waves x 32 queries.
template <int D>
__global__ void __launch_bounds__(256) attn_fwd_kernel(FwdArgs a) {
  constexpr int BN = 64;                 // keys per KV tile
  constexpr int KP = D + 8;              // padded K row (elements)
  constexpr int VP = BN + 8;             // padded V^T row
  constexpr int NC = D / 16;             // 16-wide d chunks (QK^T k-steps)
  constexpr int NDB = D / 32;            // 32-row d blocks of O^T
  __shared__ __attribute__((aligned(16))) bf16 Ks[BN * KP];
  __shared__ __attribute__((aligned(16))) bf16 Vt[D * VP];

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, hh = lane >> 5, r = lane & 31;
  const int bh = blockIdx.y, b = bh / a.H, h = bh % a.H;
  const int S = a.S;
  const int q0 = blockIdx.x * 128 + w * 32;
  const int q = q0 + r;                  // this lane's query (column of S^T)
  const bool qvalid = q < S;
  const float sl2 = a.slopes ? a.slopes[h] * kLog2e : 0.f;
  const float sc2 = a.scale * kLog2e;
  const bool drop = a.p > 0.f;
  DropoutRng g(a.rng, a.sid);
  const uint32_t thr = keep_threshold(a.p);
  const float inv_keep = drop ? 1.f / (1.f - a.p) : 1.f;

  // Q fragments (B operand of S^T = K.Q^T): Q[q][16c + 8hh + j]
  bf16x8 qf[NC];
  {
    const bf16* qp = a.q + ((size_t)(b * S + (qvalid ? q : 0)) * a.ld + h * D);
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      qf[c] = *reinterpret_cast<const bf16x8*>(qp + 16 * c + 8 * hh);
      if (!qvalid) qf[c] = bf16x8{};
    }
  }
  f32x16 oacc[NDB];
#pragma unroll
  for (int d = 0; d < NDB; ++d) oacc[d] = f32x16{};
  float m = -INFINITY, l = 0.f;

  int kend = S;
  if (a.causal) kend = min(S, blockIdx.x * 128 + 128);
  for (int k0 = 0; k0 < kend; k0 += BN) {
    // ---- stage K (row-major) and V (transposed) tiles: 16-byte global loads ----
    __syncthreads();
    for (int cidx = threadIdx.x; cidx < BN * D / 8; cidx += 256) {
      const int key = cidx / (D / 8), dc = (cidx % (D / 8)) * 8;
      const int kg = k0 + key;
      bf16x8 kv = bf16x8{}, vv = bf16x8{};
      if (kg < S) {
        const size_t off = (size_t)(b * S + kg) * a.ld + h * D + dc;
        kv = *reinterpret_cast<const bf16x8*>(a.k + off);
        vv = *reinterpret_cast<const bf16x8*>(a.v + off);
      }
      *reinterpret_cast<bf16x8*>(&Ks[key * KP + dc]) = kv;
#pragma unroll
      for (int j = 0; j < 8; ++j) Vt[(dc + j) * VP + key] = vv[j];
    }
    __syncthreads();

    // ---- S^T tile: two 32-key blocks x 32 queries ----
    f32x16 sacc[2];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      f32x16 acc = f32x16{};
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const bf16x8 kf = *reinterpret_cast<const bf16x8*>(&Ks[(kb * 32 + r) * KP + 16 * c + 8 * hh]);
        acc = mfma32(kf, qf[c], acc);
      }
      sacc[kb] = acc;
    }
    // ---- scale, bias, masks; online softmax (log2 domain) ----
    float tmax = -INFINITY;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int key = k0 + kb * 32 + crow(i, hh);
        float s = sacc[kb][i] * sc2 + sl2 * (float)key;
        if (key >= S || (a.causal && key > q)) s = -INFINITY;
        sacc[kb][i] = s;
        tmax = fmaxf(tmax, s);
      }
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
    const float mnew = fmaxf(m, tmax);
    const float alpha = (m == -INFINITY) ? 0.f : exp2f(m - mnew);
    m = mnew;
    float psum = 0.f;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float pv = (mnew == -INFINITY) ? 0.f : exp2f(sacc[kb][i] - mnew);
        psum += pv;
        sacc[kb][i] = pv;
      }
    psum += __shfl_xor(psum, 32, 64);
    l = l * alpha + psum;
#pragma unroll
    for (int d = 0; d < NDB; ++d) oacc[d] *= alpha;
    if (drop) {
      const uint64_t rowbase = ((uint64_t)bh * S + (uint64_t)q) * (uint64_t)S;
#pragma unroll
      for (int kb = 0; kb < 2; ++kb)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int key = k0 + kb * 32 + crow(i, hh);
          sacc[kb][i] *= drop_keep(g, rowbase + key, thr) * inv_keep;
        }
    }
    // ---- O^T += V^T . P^T (P^T = score accumulator as B operand) ----
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        bf16x8 pf;
#pragma unroll
        for (int j = 0; j < 8; ++j) pf[j] = (bf16)sacc[kb][8 * s + j];
        const int kk = kb * 32 + 16 * s + 4 * hh;
#pragma unroll
        for (int d = 0; d < NDB; ++d) {
          const bf16* vr = &Vt[(d * 32 + r) * VP + kk];
          const bf16x4 lo = *reinterpret_cast<const bf16x4*>(vr);
          const bf16x4 hi = *reinterpret_cast<const bf16x4*>(vr + 8);
          bf16x8 vf;
          vf[0] = lo[0]; vf[1] = lo[1]; vf[2] = lo[2]; vf[3] = lo[3];
          vf[4] = hi[0]; vf[5] = hi[1]; vf[6] = hi[2]; vf[7] = hi[3];
          oacc[d] = mfma32(vf, pf, oacc[d]);
        }
      }
  }
  // ---- epilogue: O = O^T^T / l, LSE (natural log) ----
  if (!qvalid) return;
  const float inv_l = l > 0.f ? 1.f / l : 0.f;
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

// delta[b,h,q] = sum_d dO[q,d] * O[q,d]  (one wave per (row, head))
template <int D>
__global__ void __launch_bounds__(256) attn_bwd_delta_kernel(const bf16* __restrict__ o, const bf16* __restrict__ dout,
                                                             float* __restrict__ delta, int B, int S, int H, int ldo) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int row = blockIdx.x;  // b*S + s
  const int b = row / S, s = row % S;
  for (int h = w; h < H; h += 4) {
    float acc = 0.f;
    const size_t off = (size_t)row * ldo + h * D;
#pragma unroll
    for (int d = lane; d < D; d += 64) acc += (float)o[off + d] * (float)dout[off + d];
    acc = wave_sum(acc);
    if (lane == 0) delta[((size_t)b * H + h) * S + s] = acc;
  }
}

struct BwdArgs {
  const bf16* q; const bf16* k; const bf16* v; const bf16* dout; const float* lse; const float* delta;
  float* dq_acc; bf16* dk; bf16* dv; const float* slopes;
  int B, S, H, ld, ldo, causal;
  float scale, p; const uint64_t* rng; uint32_t sid;
};

// grid: (ceil(S/128), B*H); block 256 = 4 waves x 32 keys.
template <int D>
__global__ void __launch_bounds__(256) attn_bwd_kernel(BwdArgs a) {
  constexpr int NC = D / 16, NDB = D / 32;
  constexpr int QP = D + 8;      // row-major [32][D] tiles
  constexpr int TP = 32 + 8;     // transposed [D][32] tiles
  constexpr int KTP = 128 + 8;   // K^T [D][128]
  constexpr int SP = 32 + 8;     // dS [32 q][32 keys] per wave
  __shared__ __attribute__((aligned(16))) bf16 Kt[D * KTP];
  __shared__ __attribute__((aligned(16))) bf16 Qs[32 * QP];
  __shared__ __attribute__((aligned(16))) bf16 Qt[D * TP];
  __shared__ __attribute__((aligned(16))) bf16 Os[32 * QP];   // dO row-major
  __shared__ __attribute__((aligned(16))) bf16 Ot[D * TP];    // dO transposed
  __shared__ __attribute__((aligned(16))) bf16 dSs[4 * 32 * SP];
  __shared__ float lse_s[32], del_s[32];

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, hh = lane >> 5, r = lane & 31;
  const int bh = blockIdx.y, b = bh / a.H, h = bh % a.H;
  const int S = a.S;
  const int kblk = blockIdx.x * 128;
  const int key = kblk + w * 32 + r;     // this lane's key (column of S / dP)
  const bool kvalid = key < S;
  const float sl2 = a.slopes ? a.slopes[h] * kLog2e : 0.f;
  const float sc2 = a.scale * kLog2e;
  const bool drop = a.p > 0.f;
  DropoutRng g(a.rng, a.sid);
  const uint32_t thr = keep_threshold(a.p);
  const float inv_keep = drop ? 1.f / (1.f - a.p) : 1.f;

  // K^T of the block's 128 keys into LDS (B operand of dQ = dS.K)
  for (int cidx = threadIdx.x; cidx < 128 * D / 8; cidx += 256) {
    const int kk = cidx / (D / 8), dc = (cidx % (D / 8)) * 8;
    bf16x8 kv = bf16x8{};
    if (kblk + kk < S) kv = *reinterpret_cast<const bf16x8*>(a.k + (size_t)(b * S + kblk + kk) * a.ld + h * D + dc);
#pragma unroll
    for (int j = 0; j < 8; ++j) Kt[(dc + j) * KTP + kk] = kv[j];
  }
  // this wave's K, V fragments as B operands: B[k = d][col = key] = K[key][16c + 8hh + j]
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

  const int qstart = a.causal ? (kblk / 32) * 32 : 0;
  for (int q0 = qstart; q0 < S; q0 += 32) {
    __syncthreads();
    // ---- stage Q, dO tiles (row-major + transposed), lse, delta ----
    for (int cidx = threadIdx.x; cidx < 32 * D / 8; cidx += 256) {
      const int qq = cidx / (D / 8), dc = (cidx % (D / 8)) * 8;
      bf16x8 qv = bf16x8{}, ov = bf16x8{};
      if (q0 + qq < S) {
        qv = *reinterpret_cast<const bf16x8*>(a.q + (size_t)(b * S + q0 + qq) * a.ld + h * D + dc);
        ov = *reinterpret_cast<const bf16x8*>(a.dout + (size_t)(b * S + q0 + qq) * a.ldo + h * D + dc);
      }
      *reinterpret_cast<bf16x8*>(&Qs[qq * QP + dc]) = qv;
      *reinterpret_cast<bf16x8*>(&Os[qq * QP + dc]) = ov;
#pragma unroll
      for (int j = 0; j < 8; ++j) { Qt[(dc + j) * TP + qq] = qv[j]; Ot[(dc + j) * TP + qq] = ov[j]; }
    }
    if (threadIdx.x < 32) {
      const int qq = q0 + threadIdx.x;
      lse_s[threadIdx.x] = qq < S ? a.lse[(size_t)bh * S + qq] * kLog2e : 0.f;
      del_s[threadIdx.x] = qq < S ? a.delta[(size_t)bh * S + qq] : 0.f;
    }
    __syncthreads();

    // ---- S = Q.K^T and dP = dO.V^T (rows = queries, lane = key) ----
    f32x16 sacc = f32x16{}, pacc = f32x16{};
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const bf16x8 qa = *reinterpret_cast<const bf16x8*>(&Qs[r * QP + 16 * c + 8 * hh]);
      const bf16x8 oa = *reinterpret_cast<const bf16x8*>(&Os[r * QP + 16 * c + 8 * hh]);
      sacc = mfma32(qa, kf[c], sacc);
      pacc = mfma32(oa, vf[c], pacc);
    }
    // ---- P, dropout, dS ----
    f32x16 pd, ds;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int qr = crow(i, hh);
      const int qq = q0 + qr;
      float s = sacc[i] * sc2 + sl2 * (float)key;
      const bool valid = kvalid && qq < S && !(a.causal && key > qq);
      const float pv = valid ? exp2f(s - lse_s[qr]) : 0.f;
      float keep = 1.f;
      if (drop) keep = drop_keep(g, ((uint64_t)bh * S + (uint64_t)qq) * (uint64_t)S + key, thr) * inv_keep;
      pd[i] = pv * keep;
      ds[i] = pv * (pacc[i] * keep - del_s[qr]);
    }
    // ---- dV^T += dO^T . Pd ; dK^T += Q^T . dS  (accumulators as B operands) ----
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 pb, sb;
#pragma unroll
      for (int j = 0; j < 8; ++j) { pb[j] = (bf16)pd[8 * s + j]; sb[j] = (bf16)ds[8 * s + j]; }
      const int kk = 16 * s + 4 * hh;
#pragma unroll
      for (int d = 0; d < NDB; ++d) {
        const bf16* orow = &Ot[(d * 32 + r) * TP + kk];
        const bf16* qrow = &Qt[(d * 32 + r) * TP + kk];
        const bf16x4 ol = *reinterpret_cast<const bf16x4*>(orow), oh = *reinterpret_cast<const bf16x4*>(orow + 8);
        const bf16x4 ql = *reinterpret_cast<const bf16x4*>(qrow), qh = *reinterpret_cast<const bf16x4*>(qrow + 8);
        bf16x8 oa, qa;
        oa[0] = ol[0]; oa[1] = ol[1]; oa[2] = ol[2]; oa[3] = ol[3]; oa[4] = oh[0]; oa[5] = oh[1]; oa[6] = oh[2]; oa[7] = oh[3];
        qa[0] = ql[0]; qa[1] = ql[1]; qa[2] = ql[2]; qa[3] = ql[3]; qa[4] = qh[0]; qa[5] = qh[1]; qa[6] = qh[2]; qa[7] = qh[3];
        dv[d] = mfma32(oa, pb, dv[d]);
        dk[d] = mfma32(qa, sb, dk[d]);
      }
    }
    // ---- dS to LDS ([q][key] per wave), then dQ_partial = dS . K_w ----
    bf16* dsw = &dSs[w * 32 * SP];
#pragma unroll
    for (int i = 0; i < 16; ++i) dsw[crow(i, hh) * SP + r] = (bf16)ds[i];
    __syncthreads();
    f32x16 dq[NDB];
#pragma unroll
    for (int d = 0; d < NDB; ++d) dq[d] = f32x16{};
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const bf16x8 sa = *reinterpret_cast<const bf16x8*>(&dsw[r * SP + 16 * s + 8 * hh]);
#pragma unroll
      for (int d = 0; d < NDB; ++d) {
        const bf16x8 kb = *reinterpret_cast<const bf16x8*>(&Kt[(d * 32 + r) * KTP + w * 32 + 16 * s + 8 * hh]);
        dq[d] = mfma32(sa, kb, dq[d]);
      }
    }
    // rows = queries, lane = d column: two 128-byte row segments per atomic wave-instruction
#pragma unroll
    for (int d = 0; d < NDB; ++d)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int qq = q0 + crow(i, hh);
        if (qq < S) atomicAdd(&a.dq_acc[((size_t)bh * S + qq) * D + d * 32 + r], dq[d][i] * a.scale);
      }
  }
  // ---- write dK = scale * dK^T^T, dV (lane = key, regs = d rows in groups of 4) ----
  if (!kvalid) return;
  bf16* dkp = a.dk + (size_t)(b * S + key) * a.ld + h * D;
  bf16* dvp = a.dv + (size_t)(b * S + key) * a.ld + h * D;
#pragma unroll
  for (int d = 0; d < NDB; ++d)
#pragma unroll
    for (int gq = 0; gq < 4; ++gq) {
      bf16x4 k4, v4;
#pragma unroll
      for (int t = 0; t < 4; ++t) { k4[t] = (bf16)(dk[d][4 * gq + t] * a.scale); v4[t] = (bf16)dv[d][4 * gq + t]; }
      *reinterpret_cast<bf16x4*>(dkp + d * 32 + 8 * gq + 4 * hh) = k4;
      *reinterpret_cast<bf16x4*>(dvp + d * 32 + 8 * gq + 4 * hh) = v4;
    }
}

// dq (strided bf16 view into dqkv) = dq_acc [B,H,S,D] fp32
template <int D>
__global__ void __launch_bounds__(256) attn_dq_store_kernel(const float* __restrict__ acc, bf16* __restrict__ dq, int B,
                                                            int S, int H, int ld) {
  const int row = blockIdx.x;  // b*S + s
  const int b = row / S, s = row % S;
  for (int e = threadIdx.x * 4; e < H * D; e += blockDim.x * 4) {
    const int h = e / D, d = e % D;
    const float4 v = *reinterpret_cast<const float4*>(acc + (((size_t)b * H + h) * S + s) * D + d);
    bf16x4 o;
    o[0] = (bf16)v.x; o[1] = (bf16)v.y; o[2] = (bf16)v.z; o[3] = (bf16)v.w;
    *reinterpret_cast<bf16x4*>(dq + (size_t)row * ld + e) = o;
  }
}

}  // namespace

// q,k,v,o: bf16 views with row stride ld (q/k/v) / ldo (o); lse: [B,H,S] fp32.
DTD_EXPORT int dtd_attn_fwd(const void* q, const void* k, const void* v, void* o, float* lse, const float* slopes,
                            int B, int S, int H, int D, int ld, int ldo, int causal, int r0, int r1, float scale,
                            float p, const uint64_t* rng, uint32_t sid, hipStream_t s) {
  (void)r0; (void)r1;
  if (B * S * H == 0) return 0;
  FwdArgs a{(const bf16*)q, (const bf16*)k, (const bf16*)v, (bf16*)o, lse, slopes, B, S, H, ld, ldo, causal,
            scale, p, rng, sid};
  dim3 grid((S + 127) / 128, B * H);
  if (D == 64) hipLaunchKernelGGL(attn_fwd_kernel<64>, grid, dim3(256), 0, s, a);
  else if (D == 128) hipLaunchKernelGGL(attn_fwd_kernel<128>, grid, dim3(256), 0, s, a);
  else return (int)hipErrorInvalidValue;
  DTD_LAUNCH_CHECK();
}

DTD_EXPORT int dtd_attn_bwd(const void* q, const void* k, const void* v, const void* o, const void* dout,
                            const float* lse, float* delta, float* dq_acc, void* dq, void* dk, void* dv,
                            const float* slopes, int B, int S, int H, int D, int ld, int ldo, int causal, int r0,
                            int r1, float scale, float p, const uint64_t* rng, uint32_t sid, hipStream_t s) {
  (void)r0; (void)r1;
  if (B * S * H == 0) return 0;
  if (D != 64 && D != 128) return (int)hipErrorInvalidValue;
  if (D == 64) hipLaunchKernelGGL(attn_bwd_delta_kernel<64>, dim3(B * S), dim3(256), 0, s, (const bf16*)o, (const bf16*)dout, delta, B, S, H, ldo);
  else hipLaunchKernelGGL(attn_bwd_delta_kernel<128>, dim3(B * S), dim3(256), 0, s, (const bf16*)o, (const bf16*)dout, delta, B, S, H, ldo);
  BwdArgs a{(const bf16*)q, (const bf16*)k, (const bf16*)v, (const bf16*)dout, lse, delta, dq_acc, (bf16*)dk, (bf16*)dv,
            slopes, B, S, H, ld, ldo, causal, scale, p, rng, sid};
  dim3 grid((S + 127) / 128, B * H);
  if (D == 64) {
    hipLaunchKernelGGL(attn_bwd_kernel<64>, grid, dim3(256), 0, s, a);
    hipLaunchKernelGGL(attn_dq_store_kernel<64>, dim3(B * S), dim3(256), 0, s, dq_acc, (bf16*)dq, B, S, H, ld);
  } else {
    hipLaunchKernelGGL(attn_bwd_kernel<128>, grid, dim3(256), 0, s, a);
    hipLaunchKernelGGL(attn_dq_store_kernel<128>, dim3(B * S), dim3(256), 0, s, dq_acc, (bf16*)dq, B, S, H, ld);
  }
  DTD_LAUNCH_CHECK();
}
