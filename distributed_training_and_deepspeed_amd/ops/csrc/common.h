// Shared device helpers for the gfx950 (MI355X / CDNA4) kernels of this framework.
//
// Conventions (every .hip file in this directory):
//  * wave = 64 lanes; block sizes are multiples of 64.
//  * bf16 is the native clang `__bf16` type: `(__bf16)f` lowers to the hardware
//    v_cvt_pk_bf16_f32 (round-to-nearest-even, NaN preserving) on gfx950.
//  * memory-bound kernels move 8-16 B per lane per access (bf16x4 / bf16x8 vectors).
//  * exported entry points are `extern "C" int dtd_*(..., hipStream_t)` returning the
//    hipError_t of the launch; the Python side (ops/_lib.py) binds them with ctypes and
//    passes torch's current HIP stream, so every launch is graph-capturable.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define DTD_EXPORT extern "C" __attribute__((visibility("default")))

typedef __bf16 bf16;
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

namespace dtd {

constexpr int kWave = 64;

// ---- dtype codes shared with python (ops/_lib.py) ----
enum DType : int { kF32 = 0, kBF16 = 1 };

// ---- vector load/store of N elements of T, converted to/from fp32 ----
template <typename T, int N> struct Vec;
template <int N> struct Vec<float, N> {
  static __device__ __forceinline__ void load(const float* p, float* out) {
    if constexpr (N % 4 == 0) {
#pragma unroll
      for (int i = 0; i < N; i += 4) {
        float4 v = *reinterpret_cast<const float4*>(p + i);
        out[i] = v.x; out[i + 1] = v.y; out[i + 2] = v.z; out[i + 3] = v.w;
      }
    } else if constexpr (N % 2 == 0) {
#pragma unroll
      for (int i = 0; i < N; i += 2) {
        float2 v = *reinterpret_cast<const float2*>(p + i);
        out[i] = v.x; out[i + 1] = v.y;
      }
    } else {
#pragma unroll
      for (int i = 0; i < N; ++i) out[i] = p[i];
    }
  }
  static __device__ __forceinline__ void store(float* p, const float* in) {
    if constexpr (N % 4 == 0) {
#pragma unroll
      for (int i = 0; i < N; i += 4)
        *reinterpret_cast<float4*>(p + i) = make_float4(in[i], in[i + 1], in[i + 2], in[i + 3]);
    } else if constexpr (N % 2 == 0) {
#pragma unroll
      for (int i = 0; i < N; i += 2) *reinterpret_cast<float2*>(p + i) = make_float2(in[i], in[i + 1]);
    } else {
#pragma unroll
      for (int i = 0; i < N; ++i) p[i] = in[i];
    }
  }
};
template <int N> struct Vec<bf16, N> {
  static __device__ __forceinline__ void load(const bf16* p, float* out) {
    if constexpr (N % 8 == 0) {
#pragma unroll
      for (int i = 0; i < N; i += 8) {
        bf16x8 v = *reinterpret_cast<const bf16x8*>(p + i);
#pragma unroll
        for (int j = 0; j < 8; ++j) out[i + j] = (float)v[j];
      }
    } else if constexpr (N % 4 == 0) {
#pragma unroll
      for (int i = 0; i < N; i += 4) {
        bf16x4 v = *reinterpret_cast<const bf16x4*>(p + i);
#pragma unroll
        for (int j = 0; j < 4; ++j) out[i + j] = (float)v[j];
      }
    } else if constexpr (N % 2 == 0) {
#pragma unroll
      for (int i = 0; i < N; i += 2) {
        bf16x2 v = *reinterpret_cast<const bf16x2*>(p + i);
        out[i] = (float)v[0]; out[i + 1] = (float)v[1];
      }
    } else {
#pragma unroll
      for (int i = 0; i < N; ++i) out[i] = (float)p[i];
    }
  }
  static __device__ __forceinline__ void store(bf16* p, const float* in) {
    if constexpr (N % 8 == 0) {
#pragma unroll
      for (int i = 0; i < N; i += 8) {
        bf16x8 v;
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = (bf16)in[i + j];
        *reinterpret_cast<bf16x8*>(p + i) = v;
      }
    } else if constexpr (N % 4 == 0) {
#pragma unroll
      for (int i = 0; i < N; i += 4) {
        bf16x4 v;
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = (bf16)in[i + j];
        *reinterpret_cast<bf16x4*>(p + i) = v;
      }
    } else if constexpr (N % 2 == 0) {
#pragma unroll
      for (int i = 0; i < N; i += 2) {
        bf16x2 v; v[0] = (bf16)in[i]; v[1] = (bf16)in[i + 1];
        *reinterpret_cast<bf16x2*>(p + i) = v;
      }
    } else {
#pragma unroll
      for (int i = 0; i < N; ++i) p[i] = (bf16)in[i];
    }
  }
};

template <typename T, int N> __device__ __forceinline__ void vload(const T* p, float* o) { Vec<T, N>::load(p, o); }
template <typename T, int N> __device__ __forceinline__ void vstore(T* p, const float* i) { Vec<T, N>::store(p, i); }

// Access form of the streaming elementwise kernels (GELU fwd/bwd, bias-grad, LayerNorm wave
// kernels): non-temporal 16/8-byte loads AND stores of the [rows, h] tensors (NT = 3) and one
// vector per thread -- +0.35 % whole-step, same box, two A/B sessions (profiles/r1_ab_ew_mode.jsonl;
// NT loads only, NT stores only and plain one-vector-per-thread all measured lower).
// DTD_EW_MODE=0 selects the plain grid-stride form (tuning runs).
inline int ew_mode() {
  const char* e = getenv("DTD_EW_MODE");
  return e ? atoi(e) : 2;
}
inline int ew_nt_bits() { return ew_mode() == 2 ? 3 : 0; }

// Streaming (non-temporal) forms for bf16 tensors touched once per pass: the 16-byte accesses
// carry the nt hint, so a pass over a tensor larger than L2 + MALL does not evict what the
// next kernel re-reads.  Other types / widths fall back to the plain forms.
template <typename T, int N> __device__ __forceinline__ void vload_nt(const T* p, float* o) {
  if constexpr (sizeof(T) == 2 && N % 8 == 0) {
#pragma unroll
    for (int i = 0; i < N; i += 8) {
      const bf16x8 v = __builtin_nontemporal_load(reinterpret_cast<const bf16x8*>(p + i));
#pragma unroll
      for (int j = 0; j < 8; ++j) o[i + j] = (float)v[j];
    }
  } else if constexpr (sizeof(T) == 2 && N % 4 == 0) {
#pragma unroll
    for (int i = 0; i < N; i += 4) {
      const bf16x4 v = __builtin_nontemporal_load(reinterpret_cast<const bf16x4*>(p + i));
#pragma unroll
      for (int j = 0; j < 4; ++j) o[i + j] = (float)v[j];
    }
  } else {
    vload<T, N>(p, o);
  }
}
template <typename T, int N> __device__ __forceinline__ void vstore_nt(T* p, const float* in) {
  if constexpr (sizeof(T) == 2 && N % 8 == 0) {
#pragma unroll
    for (int i = 0; i < N; i += 8) {
      bf16x8 v;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = (bf16)in[i + j];
      __builtin_nontemporal_store(v, reinterpret_cast<bf16x8*>(p + i));
    }
  } else if constexpr (sizeof(T) == 2 && N % 4 == 0) {
#pragma unroll
    for (int i = 0; i < N; i += 4) {
      bf16x4 v;
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = (bf16)in[i + j];
      __builtin_nontemporal_store(v, reinterpret_cast<bf16x4*>(p + i));
    }
  } else {
    vstore<T, N>(p, in);
  }
}

// ---- wave / block reductions (64-wide waves) ----
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
// Block-wide sum; `sh` must hold >= blockDim.x/64 floats. All threads get the result.
__device__ __forceinline__ float block_sum(float v, float* sh) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) sh[w] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < nw; ++i) t += sh[i];
  return t;
}
__device__ __forceinline__ float block_max(float v, float* sh) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_max(v);
  __syncthreads();
  if (lane == 0) sh[w] = v;
  __syncthreads();
  float t = -INFINITY;
  for (int i = 0; i < nw; ++i) t = fmaxf(t, sh[i]);
  return t;
}

// ---- counter-based RNG for dropout ----
// A dropout mask element is a pure function of (seed, step, stream id, element index) so the
// backward pass (and activation recompute) regenerates it instead of storing a mask.
// `rng` points at device memory {seed, step}: the step is bumped on device once per training
// step, which keeps masks fresh under hipGraph replay (host scalars would be frozen).
__device__ __forceinline__ uint32_t mix32(uint32_t h) {
  h ^= h >> 16; h *= 0x7feb352dU; h ^= h >> 15; h *= 0x846ca68bU; h ^= h >> 16;
  return h;
}
struct DropoutRng {
  uint32_t k0, k1;
  __device__ __forceinline__ DropoutRng(const uint64_t* rng, uint32_t stream_id) {
    const uint64_t seed = rng[0], step = rng[1];
    k0 = mix32((uint32_t)seed ^ mix32((uint32_t)(seed >> 32) + 0x9e3779b9U));
    k1 = mix32((uint32_t)step * 0x85ebca6bU ^ mix32(stream_id + 0x632be5abU) ^ k0);
  }
  // 32 random bits for 64-bit element index i (one mix32 per pair of dropout decisions:
  // the attention kernels draw B*H*S*S of them per layer, so the hash is kept short -- the
  // counter enters the bijective mix32 finalizer directly, 2 integer multiplies per hash;
  // v_mul_lo_u32 is a quarter-rate VALU op on CDNA, and it bounds the mask generator).
  __device__ __forceinline__ uint32_t bits(uint64_t i) const {
    return mix32(((uint32_t)i ^ k0) + hi_term((uint32_t)(i >> 32)));
  }
  __device__ __forceinline__ uint32_t hi_term(uint32_t hi) const { return (hi * 0xc2b2ae35U) ^ k1; }
  // bits() for consecutive counters sharing one precomputed hi_term (the caller guarantees the
  // high word does not change across the run)
  __device__ __forceinline__ uint32_t bits_lo(uint32_t lo, uint32_t ht) const { return mix32((lo ^ k0) + ht); }
};
// Two keep-decisions per 32 random bits (16-bit thresholds: p quantised to 1/65536).
__host__ __device__ __forceinline__ uint32_t keep_threshold(float p) {
  float t = p * 65536.0f;
  return t >= 65536.0f ? 65536u : (uint32_t)(t + 0.5f);
}

// One LDS-DMA piece (buffer_load_dwordx4 ... lds: 16 bytes per lane to LDS address lds + 16 lane)
// as inline asm.  Issued through the builtin, hipcc's wait-count pass treats every later LDS read
// (and the next LDS-DMA) as a possible alias of the in-flight DMA and drains the whole vector-memory
// queue before it (s_waitcnt vmcnt(0)): the counted waits of a multi-stage LDS ring are then dead
// letters and every stage lands before the next is issued.  Hidden in asm the DMA is counted only by
// the kernel's own s_waitcnt vmcnt(N) (a compiler-visible load or store in between only makes those
// waits stricter: the counter retires in issue order).  M0 is set inside the statement (the
// compiler does not preserve it around asm) and restored after it; the s_nop covers the
// M0-write -> LDS-DMA hazard.
// LDS byte address of a pointer into a __shared__ array (32-bit, wave-uniform)
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)p);
}
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, uint32_t lds, int voff, int soff) {
  // the LDS address and the scalar offset must be wave-uniform (SGPR operands): readfirstlane makes
  // that provable where the caller's expression is not (a no-op on values already in SGPRs)
  const uint32_t m = __builtin_amdgcn_readfirstlane(lds);
  soff = __builtin_amdgcn_readfirstlane(soff);
#ifdef DTD_DMA_BUILTIN   // A/B builds only: the builtin form (hipcc's drains included)
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)(uintptr_t)m, 16, voff, soff,
                                           0, 0);
  return;
#endif
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tbuffer_load_dwordx4 %2, %3, %4 offen lds\n\t"
               "s_mov_b32 m0, %0"
               : "=&s"(keep) : "s"(m), "v"(voff), "s"(r), "s"(soff) : "memory");
}
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, const void* lds, int voff, int soff) {
  dma16(r, lds_addr(lds), voff, soff);
}

}  // namespace dtd

#define DTD_LAUNCH_CHECK() return (int)hipGetLastError()
