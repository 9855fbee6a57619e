// Timestamped forward-attention run: per workgroup, s_memrealtime (100 MHz) at entry, after the
// prologue barrier, after tile 0 / tile nt-2 / tile nt-1, before and after the epilogue.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../distributed_training_and_deepspeed_amd/ops/csrc
//        attn_trace_main.hip -o attn_trace
#include "attn_fwd_traced.hip"
#include <vector>
#include <cstdio>

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 32, S = argc > 2 ? atoi(argv[2]) : 512, H = 16, D = 64;
  const int ld = 3 * H * D;
  bf16* qkv; bf16* o; float* lse; unsigned long long* tr;
  hipMalloc(&qkv, (size_t)B * S * ld * 2); hipMalloc(&o, (size_t)B * S * H * D * 2);
  hipMalloc(&lse, (size_t)B * H * S * 4);
  hipMemset(qkv, 0, (size_t)B * S * ld * 2);
  const int nwg = ((S + 127) / 128) * B * H;
  hipMalloc(&tr, (size_t)nwg * 8 * 8);
  hipMemcpyToSymbol(HIP_SYMBOL(g_trace), &tr, sizeof(tr));
  for (int it = 0; it < 5; ++it) {
    hipMemset(tr, 0, (size_t)nwg * 64);
    int rc = dtd_attn_fwd(qkv, qkv + H * D, qkv + 2 * H * D, o, lse, nullptr, nullptr, B, S, H, D, ld, H * D, 0,
                          0.125f, 0.f, nullptr, 0, 0);
    hipDeviceSynchronize();
    if (rc) { printf("rc %d\n", rc); return 1; }
  }
  std::vector<unsigned long long> h((size_t)nwg * 8);
  hipMemcpy(h.data(), tr, h.size() * 8, hipMemcpyDeviceToHost);
  FILE* f = fopen(argc > 3 ? argv[3] : "trace.csv", "w");
  fprintf(f, "wg,t0,t1,t2,t3,t4,t5,t6\n");
  for (int w = 0; w < nwg; ++w) {
    fprintf(f, "%d", w);
    for (int k = 0; k < 7; ++k) fprintf(f, ",%llu", h[w * 8 + k]);
    fprintf(f, "\n");
  }
  fclose(f);
  printf("wrote %d workgroups\n", nwg);
  return 0;
}
