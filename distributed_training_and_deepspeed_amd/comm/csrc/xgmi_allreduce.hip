// Peer-mapped all-reduce over the xGMI full mesh of an MI355X node.
//
// RCCL's ring all-reduce runs each ring over ONE xGMI link per GPU (~153 GB/s) and pays a
// per-hop latency, which dominates small buckets (the last DDP buckets, ZeRO scalars, grad-norm
// reductions).  Inside a node every MI355X has a direct link to each of its 7 peers, so a kernel
// that reads the peers' buffers directly (IPC-mapped into this process) finishes in ONE (one-shot)
// or TWO (two-shot) link latencies and uses all 7 links at once:
//
//   one-shot : every rank copies its input into its staging buffer, barrier, then reads the
//              element range of each workgroup from ALL n staging buffers and sums (fp32) --
//              (n-1) x message bytes read per GPU, lowest latency (small messages);
//   two-shot : reduce-scatter (rank r sums chunk r of every peer's staging buffer into its result
//              buffer), barrier, all-gather (read chunk p of peer p's result) -- 2(n-1)/n x bytes
//              per GPU, the bandwidth-optimal direct algorithm (medium messages).
//
// Synchronisation (CDNA4 memory model): workgroup b of every rank handles the same element set
// in every phase, so the barrier is per workgroup: lanes 0..n-1 of workgroup b store the call's
// epoch into slot [b][my rank] of peer lane's signal array with a system-scope RELEASE (after a
// system-scope fence by every thread that wrote staging data), then spin with system-scope
// ACQUIRE loads on their own slot [b][peer].  Signals live in fine-grained uncached memory
// (hipDeviceMallocUncached) so remote stores are visible without cache maintenance; staging
// buffers are ordinary device memory made visible by the release/acquire fences (L2 writeback
// on release, L2 invalidate on acquire).  Staging is double-buffered by epoch parity: a rank can
// only reach call k+1's barrier after it finished reading call k's buffers, so one barrier per
// phase suffices.  Every spin is bounded (kSpinLimit polls): a missing peer sets an error flag and
// the kernel still drains instead of hanging the GPU.
//
// The same kernel runs in "local" mode for testing: gridDim.y virtual ranks inside one process on
// one device (views of n buffers on the same GPU), which exercises the indexing, the epoch/parity
// protocol and the barrier on a 1-GPU box; the real mode maps peers with hipIpcOpenMemHandle.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include "common.h"

using namespace dtd;

namespace {

constexpr int kMaxRanks = 8;
constexpr int kMaxBlocks = 64;          // workgroups per rank (barrier slots)
constexpr int kThreads = 512;
constexpr uint32_t kSpinLimit = 1u << 26;

struct XArgs {
  const void* in[kMaxRanks];            // per virtual rank (real mode: [0] only)
  void* out[kMaxRanks];
  char* staging[kMaxRanks];             // rank i's staging base as mapped here: [2 parity][2 (in,res)][max_bytes]
  uint32_t* sig[kMaxRanks];             // rank i's signal base: [2 phases][kMaxBlocks][kMaxRanks]
  uint32_t* err;                        // local error flag (spin timeout)
  long long max_bytes;
  long long numel;
  int world, rank_base;
  uint32_t epoch;
  float scale;                          // y = scale * sum (1/world: DDP's average)
};

__device__ __forceinline__ void signal_and_wait(const XArgs& a, int rank, int phase) {
  // every thread: make this thread's staging writes visible at system scope before the flag
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");   // "" = system scope
  __syncthreads();
  const int t = threadIdx.x;
  if (t < a.world) {
    uint32_t* remote = a.sig[t] + ((size_t)phase * kMaxBlocks + blockIdx.x) * kMaxRanks + rank;
    __hip_atomic_store(remote, a.epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    const uint32_t* mine = a.sig[rank] + ((size_t)phase * kMaxBlocks + blockIdx.x) * kMaxRanks + t;
    uint32_t n = 0;
    while ((int32_t)(__hip_atomic_load(mine, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) - a.epoch) < 0) {
      __builtin_amdgcn_s_sleep(1);
      if (++n == kSpinLimit) {
        __hip_atomic_store(a.err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
  }
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
}

// 8 elements = one (bf16) or two (fp32) 16-byte moves
template <typename T>
__device__ __forceinline__ void copy8(T* d, const T* s) {
  const uint4* src = reinterpret_cast<const uint4*>(s);
  uint4* dst = reinterpret_cast<uint4*>(d);
#pragma unroll
  for (int i = 0; i < (int)(8 * sizeof(T) / 16); ++i) dst[i] = src[i];
}

template <typename T>
__device__ __forceinline__ void load8(const T* p, float* o) { vload<T, 8>(p, o); }
template <typename T>
__device__ __forceinline__ void store8(T* p, const float* i) { vstore<T, 8>(p, i); }

// Element set of workgroup b: 8-element vectors v with v % gridDim.x == b (strided by thread).
template <typename T, bool TWO_SHOT>
__global__ void __launch_bounds__(kThreads) xgmi_allreduce_kernel(XArgs a) {
  const int vr = blockIdx.y;
  const int rank = a.rank_base + vr;
  const int n = a.world;
  const int parity = a.epoch & 1;
  const size_t region = (size_t)a.max_bytes;
  auto in_buf = [&](int r) { return reinterpret_cast<T*>(a.staging[r] + (size_t)(parity * 2 + 0) * region); };
  auto res_buf = [&](int r) { return reinterpret_cast<T*>(a.staging[r] + (size_t)(parity * 2 + 1) * region); };
  const T* x = reinterpret_cast<const T*>(a.in[vr]);
  T* y = reinterpret_cast<T*>(a.out[vr]);
  const size_t nvec = (size_t)a.numel / 8;
  const size_t stride = (size_t)gridDim.x * blockDim.x;

  if constexpr (!TWO_SHOT) {
    T* mine = in_buf(rank);
    for (size_t v = (size_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += stride)
      copy8<T>(mine + v * 8, x + v * 8);
    signal_and_wait(a, rank, 0);
    for (size_t v = (size_t)blockIdx.x * blockDim.x + threadIdx.x; v < nvec; v += stride) {
      float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      for (int p = 0; p < n; ++p) {      // fixed order: bitwise-identical results on every rank
        float u[8];
        load8<T>(in_buf(p) + v * 8, u);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += u[j];
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] *= a.scale;
      store8<T>(y + v * 8, acc);
    }
  } else {
    // chunk c = vectors [c*cv, (c+1)*cv); the host guarantees numel % (8 n) == 0
    const size_t cv = nvec / n;
    T* mine = in_buf(rank);
    for (int c = 0; c < n; ++c)
      for (size_t v = (size_t)blockIdx.x * blockDim.x + threadIdx.x; v < cv; v += stride) {
        const size_t e = (c * cv + v) * 8;
        copy8<T>(mine + e, x + e);
      }
    signal_and_wait(a, rank, 0);
    T* res = res_buf(rank);
    for (size_t v = (size_t)blockIdx.x * blockDim.x + threadIdx.x; v < cv; v += stride) {
      const size_t e = (rank * cv + v) * 8;
      float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      for (int p = 0; p < n; ++p) {
        float u[8];
        load8<T>(in_buf(p) + e, u);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += u[j];
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] *= a.scale;
      store8<T>(res + e, acc);
      store8<T>(y + e, acc);
    }
    signal_and_wait(a, rank, 1);
    for (int q = 1; q < n; ++q) {
      const int c = (rank + q) % n;
      const T* src = res_buf(c);
      for (size_t v = (size_t)blockIdx.x * blockDim.x + threadIdx.x; v < cv; v += stride) {
        const size_t e = (c * cv + v) * 8;
        copy8<T>(y + e, src + e);
      }
    }
  }
}

struct Ctx {
  int rank, world, local;               // local: number of virtual ranks in this process (0 = real mode)
  long long max_bytes;
  char* staging[kMaxRanks];             // mapped bases (own allocation at [rank], or all in local mode)
  uint32_t* sig[kMaxRanks];
  bool opened[kMaxRanks];
  uint32_t* err;
};

int alloc_rank_buffers(long long max_bytes, char** staging, uint32_t** sig) {
  hipError_t e = hipMalloc(reinterpret_cast<void**>(staging), (size_t)max_bytes * 4);
  if (e != hipSuccess) return (int)e;
  const size_t sbytes = sizeof(uint32_t) * 2 * kMaxBlocks * kMaxRanks;
  e = hipExtMallocWithFlags(reinterpret_cast<void**>(sig), sbytes, hipDeviceMallocUncached);
  if (e != hipSuccess) return (int)e;
  return (int)hipMemset(*sig, 0, sbytes);
}

}  // namespace

// ---- C ABI (bound from comm/xgmi.py) ----

DTD_EXPORT int dtd_xgmi_max_ranks() { return kMaxRanks; }

// Real mode: allocate this rank's staging + signal buffers.  `handles_out` receives two
// hipIpcMemHandle_t (staging, signal) = 2 * sizeof(hipIpcMemHandle_t) bytes.
DTD_EXPORT int dtd_xgmi_create(int rank, int world, long long max_bytes, void** ctx_out, void* handles_out) {
  if (world < 1 || world > kMaxRanks || rank < 0 || rank >= world || max_bytes <= 0) return -1;
  Ctx* c = new Ctx();
  memset(c, 0, sizeof(Ctx));
  c->rank = rank; c->world = world; c->local = 0; c->max_bytes = max_bytes;
  int rc = alloc_rank_buffers(max_bytes, &c->staging[rank], &c->sig[rank]);
  if (rc) { delete c; return rc; }
  if (hipMalloc(reinterpret_cast<void**>(&c->err), sizeof(uint32_t)) != hipSuccess) { delete c; return -2; }
  hipMemset(c->err, 0, sizeof(uint32_t));
  hipIpcMemHandle_t* h = reinterpret_cast<hipIpcMemHandle_t*>(handles_out);
  hipError_t e = hipIpcGetMemHandle(&h[0], c->staging[rank]);
  if (e == hipSuccess) e = hipIpcGetMemHandle(&h[1], c->sig[rank]);
  *ctx_out = c;
  return (int)e;
}

DTD_EXPORT int dtd_xgmi_handle_bytes() { return (int)(2 * sizeof(hipIpcMemHandle_t)); }

// Map every peer's buffers (handles: world x 2 hipIpcMemHandle_t, own entry ignored).
DTD_EXPORT int dtd_xgmi_open(void* ctx, const void* handles) {
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  const hipIpcMemHandle_t* h = reinterpret_cast<const hipIpcMemHandle_t*>(handles);
  for (int p = 0; p < c->world; ++p) {
    if (p == c->rank) continue;
    void* s = nullptr; void* g = nullptr;
    hipError_t e = hipIpcOpenMemHandle(&s, h[2 * p], hipIpcMemLazyEnablePeerAccess);
    if (e != hipSuccess) return (int)e;
    e = hipIpcOpenMemHandle(&g, h[2 * p + 1], hipIpcMemLazyEnablePeerAccess);
    if (e != hipSuccess) return (int)e;
    c->staging[p] = reinterpret_cast<char*>(s);
    c->sig[p] = reinterpret_cast<uint32_t*>(g);
    c->opened[p] = true;
  }
  return 0;
}

// Local mode: `world` virtual ranks in this process on the current device (testing).
DTD_EXPORT int dtd_xgmi_create_local(int world, long long max_bytes, void** ctx_out) {
  if (world < 1 || world > kMaxRanks || max_bytes <= 0) return -1;
  Ctx* c = new Ctx();
  memset(c, 0, sizeof(Ctx));
  c->rank = 0; c->world = world; c->local = world; c->max_bytes = max_bytes;
  for (int r = 0; r < world; ++r) {
    int rc = alloc_rank_buffers(max_bytes, &c->staging[r], &c->sig[r]);
    if (rc) return rc;
  }
  if (hipMalloc(reinterpret_cast<void**>(&c->err), sizeof(uint32_t)) != hipSuccess) return -2;
  hipMemset(c->err, 0, sizeof(uint32_t));
  *ctx_out = c;
  return 0;
}

DTD_EXPORT int dtd_xgmi_destroy(void* ctx) {
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  if (!c) return 0;
  hipDeviceSynchronize();
  for (int p = 0; p < kMaxRanks; ++p) {
    if (c->opened[p]) {
      hipIpcCloseMemHandle(c->staging[p]);
      hipIpcCloseMemHandle(c->sig[p]);
    } else if (c->staging[p] && (c->local || p == c->rank)) {
      hipFree(c->staging[p]);
      hipFree(c->sig[p]);
    }
  }
  hipFree(c->err);
  delete c;
  return 0;
}

DTD_EXPORT int dtd_xgmi_error(void* ctx, hipStream_t s) {
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  uint32_t v = 0;
  hipMemcpyAsync(&v, c->err, sizeof(uint32_t), hipMemcpyDeviceToHost, s);
  hipStreamSynchronize(s);
  return (int)v;
}

// Non-blocking form: queue a copy of the error flag into `host_dst` (pinned host memory) on `s`.
// The caller reads the value one step later, so no host synchronisation is needed per step.
DTD_EXPORT int dtd_xgmi_error_poll(void* ctx, uint32_t* host_dst, hipStream_t s) {
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  return (int)hipMemcpyAsync(host_dst, c->err, sizeof(uint32_t), hipMemcpyDeviceToHost, s);
}

// y = scale * sum over ranks of x (per virtual rank in local mode: ins/outs arrays of `local` pointers).
// dtype: 0 fp32, 1 bf16.  mode: 0 one-shot, 1 two-shot.  numel % 8 == 0 (two-shot: % (8 world)).
DTD_EXPORT int dtd_xgmi_allreduce(void* ctx, const void* const* ins, void* const* outs, long long numel, int dtype,
                                  int mode, unsigned epoch, float scale, int blocks, hipStream_t s) {
  Ctx* c = reinterpret_cast<Ctx*>(ctx);
  const int es = dtype == kBF16 ? 2 : 4;
  if (numel <= 0) return 0;
  if (numel % 8 || numel * es > c->max_bytes) return -1;
  if (mode == 1 && numel % (8LL * c->world)) return -1;
  XArgs a;
  memset(&a, 0, sizeof(a));
  const int nv = c->local ? c->local : 1;
  for (int i = 0; i < nv; ++i) { a.in[i] = ins[i]; a.out[i] = outs[i]; }
  for (int p = 0; p < c->world; ++p) { a.staging[p] = c->staging[p]; a.sig[p] = c->sig[p]; }
  a.err = c->err; a.max_bytes = c->max_bytes; a.numel = numel; a.world = c->world;
  a.rank_base = c->local ? 0 : c->rank; a.epoch = epoch; a.scale = scale;
  blocks = blocks < 1 ? 1 : (blocks > kMaxBlocks ? kMaxBlocks : blocks);
  dim3 grid(blocks, nv);
  if (dtype == kBF16) {
    if (mode == 1) hipLaunchKernelGGL((xgmi_allreduce_kernel<bf16, true>), grid, dim3(kThreads), 0, s, a);
    else hipLaunchKernelGGL((xgmi_allreduce_kernel<bf16, false>), grid, dim3(kThreads), 0, s, a);
  } else {
    if (mode == 1) hipLaunchKernelGGL((xgmi_allreduce_kernel<float, true>), grid, dim3(kThreads), 0, s, a);
    else hipLaunchKernelGGL((xgmi_allreduce_kernel<float, false>), grid, dim3(kThreads), 0, s, a);
  }
  DTD_LAUNCH_CHECK();
}
