// Flash-style attention at the reference's precision (fp32 in, fp32 out) on the gfx950 f32 MFMA.
//
// The reference trains in fp32 throughout (reference model/transformer.py:80-86 and
// HF BertSelfAttention: matmul -> softmax -> dropout -> matmul, materialising the S x S scores).
// These kernels keep the scores in registers like the bf16 family in attention.hip, but run the
// products on v_mfma_f32_32x32x2_f32: exact fp32 products with fp32 accumulation (one rounding per
// product, cdna_hip_programming.md §3 "FP32-input MFMA"), so the --dtype fp32 path is not a
// reduced-precision shortcut.  At the f32 rate (64 FLOP/clk/SIMD, 1/16 of bf16) the products
// dominate the per-score softmax VALU work, so the kernels are simple: one LDS stage per tile,
// two workgroups per CU to overlap one's staging with the other's MFMAs.
//
// Operand maps of 32x32x2 f32 (cdna_hip_programming.md §3): lane l holds A[i = l&31][k = l>>5] and
// B[k = l>>5][j = l&31]; C/D register i of lane l is row crow(i, l>>5), column l&31.  A dot product
// over d in k-steps of 2 may visit d in any order as long as both operands use the same one:
// step s of lane half h takes d = dperm(s, h) = 8(s/4) + 4h + s%4, so each lane reads its
// operand rows as float4 (4 steps per 16-byte read).  A score accumulator is the B operand of
// the following product as is: its register s holds, for lane half h, row crow(s, h) -- which is
// exactly "k-step s, half h" of a 32-deep sum.
//
//  forward   query on the lane: S^T = K Q^T (K rows from LDS, Q in registers), online softmax,
//            O^T += V^T P^T (V rows from LDS, P^T = the score registers)
//  dQ        query on the lane: S^T, dP^T = V dO^T, dS^T = P^T (dP^T keep/(1-p) - delta),
//            dQ^T += K^T dS^T; also writes delta = rowsum(dO * O) for the dK/dV kernel
//  dK / dV   key on the lane: S = Q K^T, dP = dO V^T (Q / dO rows from LDS, K / V in registers),
//            dV^T += dO^T (P keep), dK^T += Q^T dS
// Dropout keep bits come from attention.hip's generator (same layouts, same stream), so the fp32
// and bf16 paths drop the same elements.  Causal masking and ALiBi as in the bf16 kernels.
#include "common.h"

using namespace dtd;

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;

__device__ __forceinline__ f32x16 mfma_f32(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ int crow(int i, int h) { return (i & 3) + 8 * (i >> 2) + 4 * h; }
// keep-word position of a query / key inside its [32 W] row (attention.hip lm_pos)
__device__ __forceinline__ int lm_pos(int x) {
  const int c = x & 31;
  return (x & ~31) | (c & 24) | ((c & 3) << 1) | ((c >> 2) & 1);
}
__device__ __forceinline__ float xhalf_max(float x) { return fmaxf(x, __shfl_xor(x, 32, 64)); }
__device__ __forceinline__ float xhalf_sum(float x) { return x + __shfl_xor(x, 32, 64); }
__device__ __forceinline__ float4 ld4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ float comp(const float4& v, int c) { return c == 0 ? v.x : c == 1 ? v.y : c == 2 ? v.z : v.w; }

struct F32Args {
  const float* q; const float* k; const float* v; float* o; float* lse; const float* slopes;
  const uint32_t* maskA;   // [B*H][W][32 W]: bit j of word (w, lm_pos(q)) = key 32 w + j kept
  const uint32_t* maskB;   // [B*H][W][32 W]: bit j of word (w, lm_pos(key)) = query 32 w + j kept
  const float* dout; float* delta; float* dq; float* dk; float* dv;
  int B, S, H, ld, ldo, causal, W;
  float scale, p;
};

// rows [row0, row0 + 64) x D of one (batch, head) -> LDS with row pitch P (rows past S read 0)
template <int D, int P>
__device__ __forceinline__ void stage_rows(float* dst, const float* base, int ld, int row0, int S) {
  constexpr int C4 = D / 4;
  for (int i = threadIdx.x; i < 64 * C4; i += 256) {
    const int r = i / C4, c = (i % C4) * 4, row = row0 + r;
    const float4 v = row < S ? ld4(base + (size_t)row * ld + c) : make_float4(0.f, 0.f, 0.f, 0.f);
    *reinterpret_cast<float4*>(dst + r * P + c) = v;
  }
}

// grid (ceil(S/128), B*H), 256 threads = 4 waves x 32 queries; 64-key tiles
template <int D, int OCC>
__global__ void __launch_bounds__(256, OCC) attn_fwd_f32_kernel(F32Args a) {
  constexpr int KP = D + 4, NG = D / 8, NDB = D / 32;
  __shared__ __attribute__((aligned(16))) float Ks[64 * KP];
  __shared__ __attribute__((aligned(16))) float Vs[64 * KP];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, hh = lane >> 5, r = lane & 31;
  const int bh = blockIdx.y, b = bh / a.H, h = bh % a.H, S = a.S;
  const int qblk = blockIdx.x * 128, q = qblk + w * 32 + r;
  const bool qv = q < S;
  const float sc2 = a.scale * kLog2e, sl2 = a.slopes ? a.slopes[h] * kLog2e : 0.f;
  const bool drop = a.maskA != nullptr;
  const int Sp = 32 * a.W;
  float4 qf[NG];
  {
    const float* qp = a.q + (size_t)(b * S + (qv ? q : 0)) * a.ld + h * D + 4 * hh;
#pragma unroll
    for (int g = 0; g < NG; ++g) qf[g] = qv ? ld4(qp + 8 * g) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  const float* kb_ = a.k + (size_t)b * S * a.ld + h * D;
  const float* vb_ = a.v + (size_t)b * S * a.ld + h * D;
  f32x16 oacc[NDB];
#pragma unroll
  for (int d = 0; d < NDB; ++d) oacc[d] = f32x16{};
  float m = -INFINITY, l = 0.f;
  const int kend = a.causal ? min(S, qblk + 128) : S;
  for (int k0 = 0; k0 < kend; k0 += 64) {
    __syncthreads();
    stage_rows<D, KP>(Ks, kb_, a.ld, k0, S);
    stage_rows<D, KP>(Vs, vb_, a.ld, k0, S);
    __syncthreads();
    f32x16 sc[2];
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      f32x16 acc = f32x16{};
      const float* kr = Ks + (kb * 32 + r) * KP + 4 * hh;
#pragma unroll
      for (int g = 0; g < NG; ++g) {
        const float4 kv = ld4(kr + 8 * g);
#pragma unroll
        for (int c = 0; c < 4; ++c) acc = mfma_f32(comp(kv, c), comp(qf[g], c), acc);
      }
      sc[kb] = acc;
    }
    // log2-domain scores, masked; tile max over this lane's 32 keys and its partner half's
    float tmax = -INFINITY;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int key = k0 + kb * 32 + crow(i, hh);
        float x = fmaf(sc[kb][i], sc2, sl2 * (float)key);
        if (key >= S || (a.causal && key > q)) x = -INFINITY;
        sc[kb][i] = x;
        tmax = fmaxf(tmax, x);
      }
    tmax = xhalf_max(tmax);
    const float mnew = fmaxf(m, tmax);
    const float alpha = m == -INFINITY ? 0.f : exp2f(m - mnew);
    m = mnew;
    l *= alpha;
#pragma unroll
    for (int d = 0; d < NDB; ++d) oacc[d] *= alpha;
    const float mexp = m == -INFINITY ? 0.f : m;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      const uint32_t word = drop ? a.maskA[((size_t)bh * a.W + (k0 >> 5) + kb) * Sp + lm_pos(qv ? q : 0)] : 0u;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float pv = exp2f(sc[kb][i] - mexp);
        l += pv;                                             // the softmax sums undropped P
        sc[kb][i] = (!drop || ((word >> crow(i, hh)) & 1u)) ? pv : 0.f;
      }
    }
    // O^T += V^T P^T: k-step s = key kb*32 + crow(s, hh) of this lane's half
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        const float* vr = Vs + (kb * 32 + crow(s, hh)) * KP + r;
#pragma unroll
        for (int d = 0; d < NDB; ++d) oacc[d] = mfma_f32(vr[d * 32], sc[kb][s], oacc[d]);
      }
  }
  l = xhalf_sum(l);
  if (!qv) return;
  const float inv = l > 0.f ? (drop ? 1.f / (1.f - a.p) : 1.f) / l : 0.f;
  float* op = a.o + (size_t)(b * S + q) * a.ldo + h * D + 4 * hh;
#pragma unroll
  for (int d = 0; d < NDB; ++d)
#pragma unroll
    for (int g = 0; g < 4; ++g)
      *reinterpret_cast<float4*>(op + d * 32 + 8 * g) =
          make_float4(oacc[d][4 * g] * inv, oacc[d][4 * g + 1] * inv, oacc[d][4 * g + 2] * inv, oacc[d][4 * g + 3] * inv);
  if (hh == 0) a.lse[(size_t)bh * S + q] = (m + log2f(l)) * kLn2;
}

// dQ (+ delta): grid (ceil(S/128), B*H), 4 waves x 32 queries, 64-key tiles
template <int D, int OCC>
__global__ void __launch_bounds__(256, OCC) attn_bwd_dq_f32_kernel(F32Args a) {
  constexpr int KP = D + 4, NG = D / 8, NDB = D / 32;
  __shared__ __attribute__((aligned(16))) float Ks[64 * KP];
  __shared__ __attribute__((aligned(16))) float Vs[64 * KP];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, hh = lane >> 5, r = lane & 31;
  const int bh = blockIdx.y, b = bh / a.H, h = bh % a.H, S = a.S;
  const int qblk = blockIdx.x * 128, q = qblk + w * 32 + r;
  const bool qv = q < S;
  const int qs = qv ? q : 0;
  const float sc2 = a.scale * kLog2e, sl2 = a.slopes ? a.slopes[h] * kLog2e : 0.f;
  const bool drop = a.maskA != nullptr;
  const float inv_keep = drop ? 1.f / (1.f - a.p) : 1.f;
  const int Sp = 32 * a.W;
  float4 qf[NG], of[NG];
  float dl = 0.f;
  {
    const float* qp = a.q + (size_t)(b * S + qs) * a.ld + h * D + 4 * hh;
    const float* dp = a.dout + (size_t)(b * S + qs) * a.ldo + h * D + 4 * hh;
    const float* opp = a.o + (size_t)(b * S + qs) * a.ldo + h * D + 4 * hh;
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      qf[g] = qv ? ld4(qp + 8 * g) : make_float4(0.f, 0.f, 0.f, 0.f);
      of[g] = qv ? ld4(dp + 8 * g) : make_float4(0.f, 0.f, 0.f, 0.f);
      const float4 ov = qv ? ld4(opp + 8 * g) : make_float4(0.f, 0.f, 0.f, 0.f);
      dl = fmaf(ov.x, of[g].x, fmaf(ov.y, of[g].y, fmaf(ov.z, of[g].z, fmaf(ov.w, of[g].w, dl))));
    }
  }
  dl = xhalf_sum(dl);
  if (qv && hh == 0) a.delta[(size_t)bh * S + q] = dl;
  const float lse2 = qv ? a.lse[(size_t)bh * S + q] * kLog2e : 0.f;
  const float* kb_ = a.k + (size_t)b * S * a.ld + h * D;
  const float* vb_ = a.v + (size_t)b * S * a.ld + h * D;
  f32x16 dq[NDB];
#pragma unroll
  for (int d = 0; d < NDB; ++d) dq[d] = f32x16{};
  const int kend = a.causal ? min(S, qblk + 128) : S;
  for (int k0 = 0; k0 < kend; k0 += 64) {
    __syncthreads();
    stage_rows<D, KP>(Ks, kb_, a.ld, k0, S);
    stage_rows<D, KP>(Vs, vb_, a.ld, k0, S);
    __syncthreads();
#pragma unroll
    for (int kb = 0; kb < 2; ++kb) {
      f32x16 st = f32x16{}, dpt = f32x16{};
      const float* kr = Ks + (kb * 32 + r) * KP + 4 * hh;
      const float* vr = Vs + (kb * 32 + r) * KP + 4 * hh;
#pragma unroll
      for (int g = 0; g < NG; ++g) {
        const float4 kv = ld4(kr + 8 * g), vv = ld4(vr + 8 * g);
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          st = mfma_f32(comp(kv, c), comp(qf[g], c), st);
          dpt = mfma_f32(comp(vv, c), comp(of[g], c), dpt);
        }
      }
      const uint32_t word = drop ? a.maskA[((size_t)bh * a.W + (k0 >> 5) + kb) * Sp + lm_pos(qs)] : 0u;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int key = k0 + kb * 32 + crow(i, hh);
        const bool ok = qv && key < S && !(a.causal && key > q);
        const float pv = ok ? exp2f(fmaf(st[i], sc2, fmaf(sl2, (float)key, -lse2))) : 0.f;
        const bool keep = !drop || ((word >> crow(i, hh)) & 1u);
        const float dpe = keep ? dpt[i] * inv_keep : 0.f;
        st[i] = pv * (dpe - dl);                              // dS^T
      }
      // dQ^T += K^T dS^T: k-step s = key kb*32 + crow(s, hh)
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        const float* kr2 = Ks + (kb * 32 + crow(s, hh)) * KP + r;
#pragma unroll
        for (int d = 0; d < NDB; ++d) dq[d] = mfma_f32(kr2[d * 32], st[s], dq[d]);
      }
    }
  }
  if (!qv) return;
  float* gp = a.dq + (size_t)(b * S + q) * a.ld + h * D + 4 * hh;
#pragma unroll
  for (int d = 0; d < NDB; ++d)
#pragma unroll
    for (int g = 0; g < 4; ++g)
      *reinterpret_cast<float4*>(gp + d * 32 + 8 * g) =
          make_float4(dq[d][4 * g] * a.scale, dq[d][4 * g + 1] * a.scale, dq[d][4 * g + 2] * a.scale,
                      dq[d][4 * g + 3] * a.scale);
}

// dK, dV: grid (ceil(S/128), B*H), 4 waves x 32 keys, 64-query tiles (Q, dO, lse, delta in LDS)
template <int D, int OCC>
__global__ void __launch_bounds__(256, OCC) attn_bwd_dkdv_f32_kernel(F32Args a) {
  constexpr int KP = D + 4, NG = D / 8, NDB = D / 32;
  __shared__ __attribute__((aligned(16))) float Qs[64 * KP];
  __shared__ __attribute__((aligned(16))) float Os[64 * KP];
  __shared__ float Ls[64], Ds[64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, hh = lane >> 5, r = lane & 31;
  const int bh = blockIdx.y, b = bh / a.H, h = bh % a.H, S = a.S;
  const int kblk = blockIdx.x * 128, key = kblk + w * 32 + r;
  const bool kv_ = key < S;
  const int ks = kv_ ? key : 0;
  const float sc2 = a.scale * kLog2e, sl2 = a.slopes ? a.slopes[h] * kLog2e : 0.f;
  const float kbias = sl2 * (float)key;
  const bool drop = a.maskB != nullptr;
  const float inv_keep = drop ? 1.f / (1.f - a.p) : 1.f;
  const int Sp = 32 * a.W;
  float4 kf[NG], vf[NG];
  {
    const float* kp = a.k + (size_t)(b * S + ks) * a.ld + h * D + 4 * hh;
    const float* vp = a.v + (size_t)(b * S + ks) * a.ld + h * D + 4 * hh;
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      kf[g] = kv_ ? ld4(kp + 8 * g) : make_float4(0.f, 0.f, 0.f, 0.f);
      vf[g] = kv_ ? ld4(vp + 8 * g) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  const float* qb_ = a.q + (size_t)b * S * a.ld + h * D;
  const float* ob_ = a.dout + (size_t)b * S * a.ldo + h * D;
  f32x16 dk[NDB], dv[NDB];
#pragma unroll
  for (int d = 0; d < NDB; ++d) { dk[d] = f32x16{}; dv[d] = f32x16{}; }
  const int qstart = a.causal ? kblk : 0;
  for (int q0 = qstart; q0 < S; q0 += 64) {
    __syncthreads();
    stage_rows<D, KP>(Qs, qb_, a.ld, q0, S);
    stage_rows<D, KP>(Os, ob_, a.ldo, q0, S);
    if (threadIdx.x < 64) {
      const int qq = q0 + threadIdx.x;
      Ls[threadIdx.x] = qq < S ? a.lse[(size_t)bh * S + qq] * kLog2e : 0.f;
      Ds[threadIdx.x] = qq < S ? a.delta[(size_t)bh * S + qq] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) {
      f32x16 sa = f32x16{}, dpa = f32x16{};
      const float* qr = Qs + (qb * 32 + r) * KP + 4 * hh;
      const float* orr = Os + (qb * 32 + r) * KP + 4 * hh;
#pragma unroll
      for (int g = 0; g < NG; ++g) {
        const float4 qv = ld4(qr + 8 * g), ov = ld4(orr + 8 * g);
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          sa = mfma_f32(comp(qv, c), comp(kf[g], c), sa);     // S[q][key]
          dpa = mfma_f32(comp(ov, c), comp(vf[g], c), dpa);   // dP[q][key]
        }
      }
      const int qw = (q0 >> 5) + qb;
      const uint32_t word = drop ? a.maskB[((size_t)bh * a.W + qw) * Sp + lm_pos(ks)] : 0u;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int ql = qb * 32 + crow(i, hh), qq = q0 + ql;
        const bool ok = kv_ && qq < S && !(a.causal && key > qq);
        const float pv = ok ? exp2f(fmaf(sa[i], sc2, kbias - Ls[ql])) : 0.f;
        const bool keep = !drop || ((word >> crow(i, hh)) & 1u);
        const float dpe = keep ? dpa[i] * inv_keep : 0.f;
        dpa[i] = pv * (dpe - Ds[ql]);                         // dS
        sa[i] = keep ? pv : 0.f;                              // P with the dropped entries zeroed
      }
      // dV^T += dO^T P_keep, dK^T += Q^T dS: k-step s = query qb*32 + crow(s, hh)
#pragma unroll
      for (int s = 0; s < 16; ++s) {
        const int row = (qb * 32 + crow(s, hh)) * KP + r;
#pragma unroll
        for (int d = 0; d < NDB; ++d) {
          dv[d] = mfma_f32(Os[row + d * 32], sa[s], dv[d]);
          dk[d] = mfma_f32(Qs[row + d * 32], dpa[s], dk[d]);
        }
      }
    }
  }
  if (!kv_) return;
  float* kp = a.dk + (size_t)(b * S + key) * a.ld + h * D + 4 * hh;
  float* vp = a.dv + (size_t)(b * S + key) * a.ld + h * D + 4 * hh;
#pragma unroll
  for (int d = 0; d < NDB; ++d)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      *reinterpret_cast<float4*>(kp + d * 32 + 8 * g) =
          make_float4(dk[d][4 * g] * a.scale, dk[d][4 * g + 1] * a.scale, dk[d][4 * g + 2] * a.scale,
                      dk[d][4 * g + 3] * a.scale);
      *reinterpret_cast<float4*>(vp + d * 32 + 8 * g) =
          make_float4(dv[d][4 * g] * inv_keep, dv[d][4 * g + 1] * inv_keep, dv[d][4 * g + 2] * inv_keep,
                      dv[d][4 * g + 3] * inv_keep);
    }
}

bool f32_offsets_ok(int S, int ld, int ldo) {
  // row offsets are formed in 32-bit ints inside a (batch, head): keep them in range
  return (long long)S * ld < (1ll << 31) && (long long)S * ldo < (1ll << 31);
}

}  // namespace

// q/k/v/o: fp32 views with row stride ld (q, k, v) / ldo (o) elements; masks as dtd_attn_fwd's
// (generated ahead by dtd_attn_masks; required when p > 0)
DTD_EXPORT int dtd_attn_fwd_f32(const float* q, const float* k, const float* v, float* o, float* lse,
                                const float* slopes, const uint32_t* masks, int B, int S, int H, int D, int ld,
                                int ldo, int causal, float scale, float p, hipStream_t s) {
  if (B * S * H == 0) return 0;
  if ((D != 64 && D != 128) || ld % 4 || ldo % 4 || !f32_offsets_ok(S, ld, ldo)) return (int)hipErrorInvalidValue;
  if (p > 0.f && !masks) return (int)hipErrorInvalidValue;
  const int W = (S + 31) / 32;
  F32Args a{q, k, v, o, lse, slopes, p > 0.f ? masks : nullptr, p > 0.f ? masks + (size_t)B * H * (32 * W) * W : nullptr,
            nullptr, nullptr, nullptr, nullptr, nullptr, B, S, H, ld, ldo, causal, W, scale, p};
  const dim3 grid((S + 127) / 128, B * H);
  if (D == 64) hipLaunchKernelGGL((attn_fwd_f32_kernel<64, 2>), grid, dim3(256), 0, s, a);
  else hipLaunchKernelGGL((attn_fwd_f32_kernel<128, 1>), grid, dim3(256), 0, s, a);
  DTD_LAUNCH_CHECK();
}

// dq/dk/dv: fp32 views with row stride ld; dout / o row stride ldo; delta [B,H,S] fp32 scratch
DTD_EXPORT int dtd_attn_bwd_f32(const float* q, const float* k, const float* v, const float* o, const float* dout,
                                const float* lse, float* delta, const uint32_t* masks, float* dq, float* dk, float* dv,
                                const float* slopes, int B, int S, int H, int D, int ld, int ldo, int causal,
                                float scale, float p, hipStream_t s) {
  if (B * S * H == 0) return 0;
  if ((D != 64 && D != 128) || ld % 4 || ldo % 4 || !f32_offsets_ok(S, ld, ldo)) return (int)hipErrorInvalidValue;
  if (p > 0.f && !masks) return (int)hipErrorInvalidValue;
  const int W = (S + 31) / 32;
  F32Args a{q, k, v, const_cast<float*>(o), const_cast<float*>(lse), slopes, p > 0.f ? masks : nullptr,
            p > 0.f ? masks + (size_t)B * H * (32 * W) * W : nullptr, dout, delta, dq, dk, dv,
            B, S, H, ld, ldo, causal, W, scale, p};
  const dim3 grid((S + 127) / 128, B * H);
  // dQ first: it writes delta = rowsum(dO * O), which the dK/dV kernel reads
  if (D == 64) {
    hipLaunchKernelGGL((attn_bwd_dq_f32_kernel<64, 2>), grid, dim3(256), 0, s, a);
    hipLaunchKernelGGL((attn_bwd_dkdv_f32_kernel<64, 2>), grid, dim3(256), 0, s, a);
  } else {
    hipLaunchKernelGGL((attn_bwd_dq_f32_kernel<128, 1>), grid, dim3(256), 0, s, a);
    hipLaunchKernelGGL((attn_bwd_dkdv_f32_kernel<128, 1>), grid, dim3(256), 0, s, a);
  }
  DTD_LAUNCH_CHECK();
}
