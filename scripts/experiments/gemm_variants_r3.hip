// Round-3 GEMM main-loop experiments (NOT compiled into the library; kept for reproducibility).
// Each was built into ops/csrc/gemm.hip as a DTD_GEMM_VARIANT, checked against an fp32 reference
// and timed against the production persistent kernel (v1) and hipBLASLt with
// scripts/bench_gemm_v2.py at the BERT-base b256 projection shapes.  All three lost to v1:
//  * variant 3, direct-store epilogue (no LDS image, v_permlane16_swap 16-byte row pieces, wave
//    rows stay staggered through the epilogue): 0.95-0.99x v1
//    (profiles/r3_gemm_direct_store_epilogue.jsonl) -- the epilogue is not the limiter;
//  * variant 4, four waves / one per SIMD, 128x128 per wave with 256 AGPR accumulators, own LDS
//    reads interleaved between MFMAs, one barrier per K-step: 0.65-0.80x v1
//    (profiles/r3_gemm_w4_experiment.jsonl);
//  * variant 5, deep prefetch (each K-step quarter restaged as soon as it is consumed, two K-steps
//    ahead of its readers): 0.75-0.82x v1 (profiles/r3_gemm_deep_prefetch_experiment.jsonl).
// They need gemm.hip's helpers (stage, stage_offsets, uniform_rsrc, bar, mfma16, tile_of, ...).
// ---------------------------------------------------------------------------------------------
// Persistent form, direct-store epilogue (EPI_STORE, optional bias; DTD_GEMM_VARIANT 3): the
// K-step pipeline of gemm_bt_persistent, but a tile's epilogue neither goes through an LDS image
// nor synchronises the workgroup.  Two packed bf16 fragments of adjacent 16-column blocks are
// exchanged between lane rows by v_permlane16_swap, after which every lane holds 8 consecutive
// columns of one row: 16 16-byte stores per wave (64-byte row segments).  The wave rows stay
// staggered through the epilogue, so one row's epilogue runs beside the other row's MFMAs (the
// last segment of the tile, or the first of the next).  The tile's bias (256 columns) comes into a
// 512-byte LDS slot by LDS-DMA in the tile's last K-step, so no register-destination load sits in
// the counted DMA pipeline (hipcc would drain it with vmcnt(0) at the first use).  Static
// XCD-grouped tile order; K >= 128.
constexpr int BIAS_LDS = LDS_BYTES;                 // 512-byte bias slot after the two K-step buffers
constexpr int LDS3_BYTES = LDS_BYTES + 512;
constexpr int DIRECT_STORES = 16;                   // vector-memory ops of one wave's epilogue

__device__ __forceinline__ uint32_t pack_bf16x2(float a, float b) {
  const bf16x2 v = {(bf16)a, (bf16)b};
  return __builtin_bit_cast(uint32_t, v);
}

// bf16 store of accumulator quadrant (qm, column blocks nb, nb + 1) of one wave: 4 x 16 rows;
// bq[0] / bq[1]: the bias of blocks nb / nb + 1 at the lane's 4 columns
template <bool BIAS>
__device__ __forceinline__ void store_quadrant(const f32x4 (&acc)[8][4], int qm, int nb, const bf16x4 (&bq)[2],
                                               bf16* __restrict__ c, int ldc, int m0, int n0, int wm, int wn, int li,
                                               int lq) {
  const int ecol = (lq & 1) * 16 + (lq >> 1) * 8;
  bf16* base = c + (size_t)(m0 + wm * 128 + qm * 64 + li) * ldc + n0 + wn * 64 + nb * 16 + ecol;
#pragma unroll
  for (int mi = 0; mi < 4; ++mi) {
    f32x4 X = acc[qm * 4 + mi][nb], Y = acc[qm * 4 + mi][nb + 1];
    if constexpr (BIAS) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        X[k] += (float)bq[0][k];
        Y[k] += (float)bq[1][k];
      }
    }
    const uint32_t x0 = pack_bf16x2(X[0], X[1]), x1 = pack_bf16x2(X[2], X[3]);
    const uint32_t y0 = pack_bf16x2(Y[0], Y[1]), y1 = pack_bf16x2(Y[2], Y[3]);
    const auto s0 = __builtin_amdgcn_permlane16_swap(x0, y0, false, false);
    const auto s1 = __builtin_amdgcn_permlane16_swap(x1, y1, false, false);
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 v = {s0[0], s1[0], s0[1], s1[1]};
    *reinterpret_cast<u32x4*>(base + (size_t)mi * 16 * ldc) = v;
  }
}

template <bool BIAS>
__global__ void __launch_bounds__(512, 2) gemm_bt_pers3(GemmArgs g) {
  __shared__ __attribute__((aligned(1024))) char smem[LDS3_BYTES];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int li = lane & 15, lq = lane >> 4, sw = li & 7;
  const int wm = w >> 2, wn = w & 3;
  const int ntn = g.N / BN, ntiles = (g.M / BM) * ntn;
  const int nk = g.K / BK;   // >= 2 (host check)
  const int nwg = gridDim.x, x = blockIdx.x % 8, l = blockIdx.x / 8, per = nwg / 8;
  const int q = ntiles / 8, r = ntiles % 8;
  const int beg = x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q;
  const int end = beg + q + (x < r ? 1 : 0);
  int t = beg + l;
  if (t >= end) return;
  int m0, n0;
  tile_of(t, ntn, m0, n0);
  const StageOffs so = stage_offsets(w, lane, g.lda, g.ldb);
  auto rsa = uniform_rsrc(g.a + (size_t)m0 * g.lda), rsb = uniform_rsrc(g.b + (size_t)n0 * g.ldb);
  const auto rbias = uniform_rsrc(BIAS ? (const void*)g.bias : (const void*)g.a);
  stage<0>(so, rsa, rsb, smem, 0);
  stage<1>(so, rsa, rsb, smem, 0);
  stage<2>(so, rsa, rsb, smem, 0);
  stage<3>(so, rsa, rsb, smem, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (__builtin_amdgcn_readfirstlane(wm) == 1) bar();   // stagger wave row 1

  const int arow = (wm * 128 + li) * 128;
  const int brow = A_BYTES + (wn * 64 + li) * 128;
  const int ch0 = ((0 * 4 + lq) ^ sw) * 16, ch1 = ((1 * 4 + lq) ^ sw) * 16;
  constexpr int BL = BIAS ? 1 : 0;
  // counted waits (a phase retires the quarter DMA of two phases ago; younger are the ops issued
  // since): first K-step after an epilogue, phases 0-1: 2 + 16 stores + 2; the last K-step,
  // phases 0-1: + the bias DMA; the very last K-step (nothing staged): 2 + bias, bias, 0, 0
  constexpr int WAIT_EPI = 4 + DIRECT_STORES;

  bf16x8 af[4][2], b0[2][2], b1[2][2];
  f32x4 acc[8][4];
  int buf = 0;
  bool after_epi = false;
  while (true) {
    const int tn = t + per;
    const bool has_next = tn < end;
    int m1 = 0, n1 = 0;
    if (has_next) tile_of(tn, ntn, m1, n1);
    const auto rsa1 = uniform_rsrc(g.a + (size_t)m1 * g.lda), rsb1 = uniform_rsrc(g.b + (size_t)n1 * g.ldb);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    for (int kt = 0; kt < nk; ++kt) {
      const char* cur = smem + buf * TILE_BYTES;
      char* nxt = smem + (buf ^ 1) * TILE_BYTES;
      buf ^= 1;
      const bool more_here = kt + 1 < nk;
      const bool more = more_here || has_next;
      const auto sra = more_here ? rsa : rsa1, srb = more_here ? rsb : rsb1;
      const int skt = more_here ? kt + 1 : 0;
      const bool first = kt == 0 && after_epi;
      const bool lastk = !more_here;
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        if (p == 0 || p == 2) {
          const int qm = p == 0 ? 0 : 1;
#pragma unroll
          for (int mi = 0; mi < 4; ++mi) {
            const char* rr = cur + arow + (qm * 4 + mi) * 16 * 128;
            af[mi][0] = *reinterpret_cast<const bf16x8*>(rr + ch0);
            af[mi][1] = *reinterpret_cast<const bf16x8*>(rr + ch1);
          }
        }
        if (p == 0 || p == 1) {
#pragma unroll
          for (int ni = 0; ni < 2; ++ni) {
            const char* rr = cur + brow + (p * 2 + ni) * 16 * 128;
            bf16x8 x0 = *reinterpret_cast<const bf16x8*>(rr + ch0);
            bf16x8 x1 = *reinterpret_cast<const bf16x8*>(rr + ch1);
            if (p == 0) { b0[ni][0] = x0; b0[ni][1] = x1; } else { b1[ni][0] = x0; b1[ni][1] = x1; }
          }
        }
        if constexpr (BIAS) {
          if (lastk && p == 0)   // this tile's 256 bias values -> LDS (every wave: 256 of the 512 B)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(rbias, (lds_void*)(smem + BIAS_LDS + (w & 1) * 256), 4,
                                                      (n0 + (w & 1) * 128) * 2 + lane * 4, 0, 0, 0);
        }
        if (more) {
          if (p == 0) stage<0>(so, sra, srb, nxt, skt);
          if (p == 1) stage<1>(so, sra, srb, nxt, skt);
          if (p == 2) stage<2>(so, sra, srb, nxt, skt);
          if (p == 3) stage<3>(so, sra, srb, nxt, skt);
          if (p < 2 && first) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(WAIT_EPI) : "memory");
          else if (p < 2 && lastk) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(4 + BL) : "memory");
          else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        } else if (p == 0) {
          asm volatile("s_waitcnt vmcnt(%0)" :: "n"(2 + BL) : "memory");
        } else if (p == 1) {
          asm volatile("s_waitcnt vmcnt(%0)" :: "n"(BL) : "memory");
        } else {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        bar();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_setprio(1);
        const int qm = (p == 2 || p == 3) ? 1 : 0;
#pragma unroll
        for (int mi = 0; mi < 4; ++mi)
#pragma unroll
          for (int ni = 0; ni < 2; ++ni)
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) {
              const bf16x8 bb = (p == 1 || p == 2) ? b1[ni][ks] : b0[ni][ks];
              const int nn = ((p == 1 || p == 2) ? 2 : 0) + ni;
              acc[qm * 4 + mi][nn] = mfma16(bb, af[mi][ks], acc[qm * 4 + mi][nn]);
            }
        __builtin_amdgcn_s_setprio(0);
        bar();
      }
    }
    // ---- epilogue: registers -> global, no LDS image, no workgroup barrier (the bias DMA of
    //      this tile was retired by the last K-step's phase-2 wait, which every wave passed)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int eqm = e >> 1, enb = (e & 1) * 2;
      bf16x4 bq[2] = {};
      if constexpr (BIAS) {
#pragma unroll
        for (int j = 0; j < 2; ++j)
          bq[j] = *reinterpret_cast<const bf16x4*>(smem + BIAS_LDS + (wn * 64 + (enb + j) * 16 + 4 * lq) * 2);
      }
      store_quadrant<BIAS>(acc, eqm, enb, bq, g.c, g.ldc, m0, n0, wm, wn, li, lq);
    }
    after_epi = true;
    if (!has_next) break;
    t = tn;
    m0 = m1;
    n0 = n1;
    rsa = rsa1;
    rsb = rsb1;
  }
  if (__builtin_amdgcn_readfirstlane(wm) == 0) bar();   // close the stagger
}

// ---------------------------------------------------------------------------------------------
// Deep-prefetch persistent form (DTD_GEMM_VARIANT 5; EPI_STORE, optional bias): the 8-wave
// 4-phase main loop and direct-store epilogue of gemm_bt_pers3, but every quarter of a K-step
// buffer is restaged the moment the current K-step has consumed it: A-lo and B-lo are read only in
// phase 0, B-hi in phase 1, A-hi in phase 2, so K-step i + 2's quarters H0 + H1 go out in phase 1
// of K-step i, H2 in phase 2, H3 in phase 3 -- two K-steps (8 phases) ahead of their readers,
// instead of the 2 phases of the other forms.  Per wave and K-step: phase 0 issues nothing (the
// tile's bias DMA, first K-step only), phase 1 four DMAs, phases 2 and 3 two each.  Waits: phase 3
// retires H0 + H1 of K-step i + 1 (12 younger ops), phase 0 H2 (10), phase 1 H3 (12), phase 2
// none; + 16 after an epilogue in between, + 1 for the bias DMA; the last two K-steps of the
// stream drain with vmcnt(0).  K >= 128.
template <bool BIAS>
__global__ void __launch_bounds__(512, 2) gemm_bt_pers5(GemmArgs g) {
  __shared__ __attribute__((aligned(1024))) char smem[LDS_BYTES + 1024];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int li = lane & 15, lq = lane >> 4, sw = li & 7;
  const int wm = w >> 2, wn = w & 3;
  const int ntn = g.N / BN, ntiles = (g.M / BM) * ntn;
  const int nk = g.K / BK;   // >= 2 (host check)
  const int nwg = gridDim.x, x = blockIdx.x % 8, l = blockIdx.x / 8, per = nwg / 8;
  const int q = ntiles / 8, r = ntiles % 8;
  const int beg = x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q;
  const int end = beg + q + (x < r ? 1 : 0);
  int t = beg + l;
  if (t >= end) return;
  const int ntl = (end - t + per - 1) / per;
  const int G = ntl * nk;   // K-steps of this workgroup's stream
  int m0, n0;
  tile_of(t, ntn, m0, n0);
  const StageOffs so = stage_offsets(w, lane, g.lda, g.ldb);
  auto panel_a = [&](int tile) { int a, b; tile_of(tile, ntn, a, b); return uniform_rsrc(g.a + (size_t)a * g.lda); };
  auto panel_b = [&](int tile) { int a, b; tile_of(tile, ntn, a, b); return uniform_rsrc(g.b + (size_t)b * g.ldb); };
  auto rsa = panel_a(t), rsb = panel_b(t);
  const int t1 = t + per < end ? t + per : t;
  auto rsa1 = panel_a(t1), rsb1 = panel_b(t1);
  const auto rbias = uniform_rsrc(BIAS ? (const void*)g.bias : (const void*)g.a);
  // prologue: K-steps 0 and 1 (both of the first tile), quarters in order
  stage<0>(so, rsa, rsb, smem, 0);
  stage<1>(so, rsa, rsb, smem, 0);
  stage<2>(so, rsa, rsb, smem, 0);
  stage<3>(so, rsa, rsb, smem, 0);
  stage<0>(so, rsa, rsb, smem + TILE_BYTES, 1);
  stage<1>(so, rsa, rsb, smem + TILE_BYTES, 1);
  stage<2>(so, rsa, rsb, smem + TILE_BYTES, 1);
  stage<3>(so, rsa, rsb, smem + TILE_BYTES, 1);
  asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  __syncthreads();
  if (__builtin_amdgcn_readfirstlane(wm) == 1) bar();   // stagger wave row 1

  const int arow = (wm * 128 + li) * 128;
  const int brow = A_BYTES + (wn * 64 + li) * 128;
  const int ch0 = ((0 * 4 + lq) ^ sw) * 16, ch1 = ((1 * 4 + lq) ^ sw) * 16;
  constexpr int BL = BIAS ? 1 : 0;
  bf16x8 af[4][2], b0[2][2], b1[2][2];
  f32x4 acc[8][4];
  int it = 0;
  for (int i = 0; i < G; ++i) {
    const int k = i - it * nk;              // K-step within the tile
    const char* cur = smem + (i & 1) * TILE_BYTES;
    char* cw = smem + (i & 1) * TILE_BYTES;   // K-step i + 2 lands in this same buffer
    const bool st2 = i + 2 < G;             // K-step i + 2 exists
    const bool nxt2 = k + 2 >= nk;          // ... and belongs to the next tile
    const auto sra = nxt2 ? rsa1 : rsa, srb = nxt2 ? rsb1 : rsb;
    const int sk = nxt2 ? k + 2 - nk : k + 2;
    const bool tail = i + 2 >= G;
    const bool e1 = k == 0 && it > 0;       // an epilogue ran right before this K-step
    const bool e2 = k == 1 && it > 0;       // ... right before the previous one
    const bool b1k = BIAS && (k == 0);      // this K-step issues the bias DMA (phase 0)
    const bool b2k = BIAS && (k == 1);      // the previous one did
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      if (p == 0 || p == 2) {
        const int qm = p == 0 ? 0 : 1;
#pragma unroll
        for (int mi = 0; mi < 4; ++mi) {
          const char* rr = cur + arow + (qm * 4 + mi) * 16 * 128;
          af[mi][0] = *reinterpret_cast<const bf16x8*>(rr + ch0);
          af[mi][1] = *reinterpret_cast<const bf16x8*>(rr + ch1);
        }
      }
      if (p == 0 || p == 1) {
#pragma unroll
        for (int ni = 0; ni < 2; ++ni) {
          const char* rr = cur + brow + (p * 2 + ni) * 16 * 128;
          bf16x8 x0 = *reinterpret_cast<const bf16x8*>(rr + ch0);
          bf16x8 x1 = *reinterpret_cast<const bf16x8*>(rr + ch1);
          if (p == 0) { b0[ni][0] = x0; b0[ni][1] = x1; } else { b1[ni][0] = x0; b1[ni][1] = x1; }
        }
      }
      if constexpr (BIAS) {
        if (p == 0 && k == 0)   // this tile's 256 bias values -> its LDS slot (tile parity)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rbias, (lds_void*)(smem + LDS_BYTES + (it & 1) * 512 + (w & 1) * 256),
                                                    4, (n0 + (w & 1) * 128) * 2 + lane * 4, 0, 0, 0);
      }
      if (st2) {   // restage the quarters this K-step has consumed with K-step i + 2
        if (p == 1) { stage<0>(so, sra, srb, cw, sk); stage<1>(so, sra, srb, cw, sk); }
        if (p == 2) stage<2>(so, sra, srb, cw, sk);
        if (p == 3) stage<3>(so, sra, srb, cw, sk);
      }
      if (tail) {
        if (p != 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      } else if (p == 0) {
        if (e1) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(10 + DIRECT_STORES + BL) : "memory");
        else if (e2) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(10 + DIRECT_STORES + BL) : "memory");
        else if (b1k || b2k) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(10 + BL) : "memory");
        else asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
      } else if (p == 1) {
        if (e1 || e2) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(12 + DIRECT_STORES + BL) : "memory");
        else if (b1k || b2k) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(12 + BL) : "memory");
        else asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
      } else if (p == 3) {
        if (e1) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(12 + DIRECT_STORES + BL) : "memory");
        else if (b1k) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(12 + BL) : "memory");
        else asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
      }
      bar();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_setprio(1);
      const int qm = (p == 2 || p == 3) ? 1 : 0;
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int ni = 0; ni < 2; ++ni)
#pragma unroll
          for (int ks = 0; ks < 2; ++ks) {
            const bf16x8 bb = (p == 1 || p == 2) ? b1[ni][ks] : b0[ni][ks];
            const int nn = ((p == 1 || p == 2) ? 2 : 0) + ni;
            const f32x4 z = {0.f, 0.f, 0.f, 0.f};
            acc[qm * 4 + mi][nn] = mfma16(bb, af[mi][ks], (k == 0 && ks == 0) ? z : acc[qm * 4 + mi][nn]);
          }
      __builtin_amdgcn_s_setprio(0);
      bar();
    }
    if (k == nk - 1) {   // tile done: direct-store epilogue (bias retired at its 2nd K-step's phase 3)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int eqm = e >> 1, enb = (e & 1) * 2;
        bf16x4 bq[2] = {};
        if constexpr (BIAS) {
#pragma unroll
          for (int j = 0; j < 2; ++j)
            bq[j] = *reinterpret_cast<const bf16x4*>(smem + LDS_BYTES + (it & 1) * 512 +
                                                     (wn * 64 + (enb + j) * 16 + 4 * lq) * 2);
        }
        store_quadrant<BIAS>(acc, eqm, enb, bq, g.c, g.ldc, m0, n0, wm, wn, li, lq);
      }
      ++it;
      t += per;
      tile_of(t < end ? t : beg, ntn, m0, n0);
      rsa = rsa1;
      rsb = rsb1;
      const int tn = t + per < end ? t + per : t;
      rsa1 = panel_a(tn);
      rsb1 = panel_b(tn);
    }
  }
  if (__builtin_amdgcn_readfirstlane(wm) == 0) bar();   // close the stagger
}

// ---------------------------------------------------------------------------------------------
// W4 form (DTD_GEMM_VARIANT 4; EPI_STORE, optional bias): FOUR waves, one per SIMD, each owning a
// 128 x 128 quarter of the 256 x 256 tile -- 256 fp32 accumulators per lane in AGPRs (a single
// wave per SIMD may use the whole 512-entry register file), so a K-step costs each wave 32 LDS
// fragment reads for 128 MFMAs (0.25 reads per MFMA; the 8-wave 128 x 64 split needs 0.375).
// With no partner wave on the SIMD, each wave hides its own LDS reads and LDS-DMA issue between
// its MFMAs (sched_group_barrier interleave) instead of alternating read / MFMA segments with a
// partner across 8 barriers per K-step: ONE barrier per K-step.
//   K-step g (buffer g & 1): part 1 = MFMAs of k-half 0 (fragments X) while reading k-half 1 (Y);
//   wait for the DMA of K-step g + 1; barrier; part 2 = MFMAs of k-half 1 (Y) while reading
//   k-half 0 of K-step g + 1 (X) and issuing the DMA of K-step g + 2 into buffer g & 1.
// The K-step stream runs across the workgroup's tiles (persistent, XCD-grouped static order);
// a tile's epilogue (bf16 + bias, v_permlane16_swap into 16-byte row pieces, direct stores) sits
// between its last K-step and the next tile's first, whose MFMAs start from C = 0.  The bias of a
// tile reaches a 512-byte LDS slot (tile parity) by LDS-DMA in its first K-step.  K >= 128.
constexpr int W4_LDS = LDS_BYTES + 1024;
constexpr int W4_STORES = 32;   // vector-memory ops of one wave's epilogue

struct W4Ctx {
  int voff;        // per-lane DMA source offset (row L/8 of an 8-row piece, swizzled chunk)
  int abase, bbase;   // per-lane fragment read offsets within a K-step buffer (chunk of k-half 0)
  int kh1;         // byte delta from the k-half 0 chunk to the k-half 1 chunk
  int w, wm, wn, li, lq, lane;
};

// the 16 DMA pieces of one wave for K-step `kk` of the tile whose operand panel is `rs`
__device__ __forceinline__ void w4_stage(const W4Ctx& C, __amdgpu_buffer_rsrc_t rs, int ld, char* buf, int kk,
                                         int i0, int i1) {
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    if (i < i0 || i >= i1) continue;
    const int j = C.w * 16 + i;   // 8-row piece of the [A; B] 512-row image
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(buf + j * 1024), 16, C.voff, kk * BK * 2 + i * 16 * ld, 0,
                                              0);
  }
}

template <bool BIAS>
__device__ __forceinline__ void w4_epilogue(const f32x4 (&acc)[8][8], const char* bias_lds, bf16* __restrict__ c,
                                            int ldc, int m0, int n0, const W4Ctx& C) {
  const int ecol = (C.lq & 1) * 16 + (C.lq >> 1) * 8;
  bf16* base = c + (size_t)(m0 + C.wm * 128 + C.li) * ldc + n0 + C.wn * 128 + ecol;
#pragma unroll
  for (int nb = 0; nb < 8; nb += 2) {
    bf16x4 bx = {}, by = {};
    if constexpr (BIAS) {
      bx = *reinterpret_cast<const bf16x4*>(bias_lds + (C.wn * 128 + nb * 16 + 4 * C.lq) * 2);
      by = *reinterpret_cast<const bf16x4*>(bias_lds + (C.wn * 128 + (nb + 1) * 16 + 4 * C.lq) * 2);
    }
#pragma unroll
    for (int mb = 0; mb < 8; ++mb) {
      f32x4 X = acc[mb][nb], Y = acc[mb][nb + 1];
      if constexpr (BIAS) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          X[k] += (float)bx[k];
          Y[k] += (float)by[k];
        }
      }
      const uint32_t x0 = pack_bf16x2(X[0], X[1]), x1 = pack_bf16x2(X[2], X[3]);
      const uint32_t y0 = pack_bf16x2(Y[0], Y[1]), y1 = pack_bf16x2(Y[2], Y[3]);
      const auto s0 = __builtin_amdgcn_permlane16_swap(x0, y0, false, false);
      const auto s1 = __builtin_amdgcn_permlane16_swap(x1, y1, false, false);
      typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
      const u32x4 v = {s0[0], s1[0], s0[1], s1[1]};
      *reinterpret_cast<u32x4*>(base + (size_t)mb * 16 * ldc + nb * 16) = v;
    }
  }
}

// fragments of one k-half: A[mb] (8) and B[nb] (8) of the wave's quarter
__device__ __forceinline__ void w4_read(const char* buf, const W4Ctx& C, int kh, bf16x8 (&fa)[8], bf16x8 (&fb)[8]) {
  const char* pa = buf + C.abase + kh * C.kh1;
  const char* pb = buf + C.bbase + kh * C.kh1;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    fa[i] = *reinterpret_cast<const bf16x8*>(pa + i * 2048);
    fb[i] = *reinterpret_cast<const bf16x8*>(pb + i * 2048);
  }
}

template <bool ZERO>
__device__ __forceinline__ void w4_mfma(f32x4 (&acc)[8][8], const bf16x8 (&fa)[8], const bf16x8 (&fb)[8]) {
  const f32x4 z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int mb = 0; mb < 8; ++mb)
#pragma unroll
    for (int nb = 0; nb < 8; ++nb) acc[mb][nb] = mfma16(fb[nb], fa[mb], ZERO ? z : acc[mb][nb]);
}

// interleave: per group, `nds` LDS reads, `nvm` VMEM issues, `nmf` MFMAs
__device__ __forceinline__ void w4_sched(int dummy) { (void)dummy; }
#define DTD_W4_SCHED(GROUPS, NDS, NVM, NMF)                                  \
  do {                                                                       \
    _Pragma("unroll") for (int _g = 0; _g < (GROUPS); ++_g) {                \
      if ((NDS) > 0) __builtin_amdgcn_sched_group_barrier(0x100, (NDS), 0);  \
      if ((NVM) > 0) __builtin_amdgcn_sched_group_barrier(0x020, (NVM), 0);  \
      __builtin_amdgcn_sched_group_barrier(0x008, (NMF), 0);                 \
    }                                                                        \
  } while (0)

template <bool BIAS>
__global__ void __launch_bounds__(256, 1) gemm_bt_w4(GemmArgs g) {
  __shared__ __attribute__((aligned(1024))) char smem[W4_LDS];
  // wave index through readfirstlane: provably uniform, so everything derived from it (operand,
  // leading dimension, DMA soffsets) stays in SGPRs -- no waterfall loops around the DMA
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  W4Ctx C;
  C.w = w; C.wm = w >> 1; C.wn = w & 1; C.li = lane & 15; C.lq = lane >> 4; C.lane = lane;
  const int ntn = g.N / BN, ntiles = (g.M / BM) * ntn;
  const int nk = g.K / BK;   // >= 2 (host check)
  const int nwg = gridDim.x, x = blockIdx.x % 8, l = blockIdx.x / 8, per = nwg / 8;
  const int q = ntiles / 8, r = ntiles % 8;
  const int beg = x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q;
  const int end = beg + q + (x < r ? 1 : 0);
  int t = beg + l;
  if (t >= end) return;
  const int ntl = (end - t + per - 1) / per;   // tiles of this workgroup
  const int ng = ntl * nk;                     // its K-steps
  // DMA: waves 0-1 stage A rows, 2-3 B rows; lane L -> row L/8 of an 8-row piece, chunk slot
  // L%8 <- global chunk (L%8) ^ (L/8) (the involutive swizzle of the fragment reads)
  const bool isb = w >= 2;
  const int ld = isb ? g.ldb : g.lda;
  C.voff = ((((w & 1) * 16 * 8) + (lane >> 3)) * ld + (((lane & 7) ^ (lane >> 3)) * 8)) * 2;
  const int sw = C.li & 7;
  C.abase = (C.wm * 128 + C.li) * 128 + ((C.lq ^ sw) * 16);
  C.bbase = A_BYTES + (C.wn * 128 + C.li) * 128 + ((C.lq ^ sw) * 16);
  C.kh1 = (((4 + C.lq) ^ sw) - (C.lq ^ sw)) * 16;
  constexpr int BL = BIAS ? 1 : 0;
  auto panel = [&](int tile) {   // this wave's operand panel of `tile`
    int tm0, tn0;
    tile_of(tile, ntn, tm0, tn0);
    return uniform_rsrc(isb ? (const void*)(g.b + (size_t)tn0 * g.ldb) : (const void*)(g.a + (size_t)tm0 * g.lda));
  };
  const auto rbias = uniform_rsrc(BIAS ? (const void*)g.bias : (const void*)g.a);
  // K-steps 0 and 1 (both of the first tile: nk >= 2)
  auto rs_cur = panel(t);
  w4_stage(C, rs_cur, ld, smem, 0, 0, 16);
  w4_stage(C, rs_cur, ld, smem + TILE_BYTES, 1, 0, 16);
  asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  bar();
  bf16x8 xa[8], xb[8], ya[8], yb[8];
  w4_read(smem, C, 0, xa, xb);
  f32x4 acc[8][8];
  int m0, n0;
  tile_of(t, ntn, m0, n0);
  int it = 0;       // tile iteration of this workgroup
  int kk = 0;       // K-step within the tile
  auto rs_next = panel(t + per < end ? t + per : t);
  (void)kk;
  for (int gs0 = 0; gs0 < ng; gs0 += nk) {   // one tile
    for (int k = 0; k < nk; ++k) {
      const int gs = gs0 + k;
      const char* cur = smem + (gs & 1) * TILE_BYTES;
      char* oth = smem + ((gs & 1) ^ 1) * TILE_BYTES;
      // ---- part 1: k-half 0 MFMAs (X) | k-half 1 reads (Y)
      w4_read(cur, C, 1, ya, yb);
      if (k == 0) w4_mfma<true>(acc, xa, xb);
      else w4_mfma<false>(acc, xa, xb);
      DTD_W4_SCHED(16, 1, 0, 4);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      // the DMA of K-step gs + 1 (issued in part 2 of gs - 1 or the prologue); younger: the
      // epilogue stores of the tile that ended at gs - 1
      if (k == 0 && it > 0) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(W4_STORES) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      bar();
      // ---- part 2: k-half 1 MFMAs (Y) | k-half 0 reads of K-step gs + 1 (X) | DMA of K-step gs + 2
      const bool has1 = gs + 1 < ng, has2 = gs + 2 < ng;
      if (has1) w4_read(oth, C, 0, xa, xb);
      if constexpr (BIAS) {
        if (k == 0)   // this tile's bias -> its LDS slot (waves 0-1: 256 B each)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rbias,
                                                    (lds_void*)(smem + LDS_BYTES + (it & 1) * 512 + (w & 1) * 256), 4,
                                                    (n0 + (w & 1) * 128) * 2 + lane * 4, 0, 0, 0);
      }
      if (has2) {
        // K-step gs + 2: this tile's k + 2, or the next tile's k + 2 - nk
        const bool nxt = k + 2 >= nk;
        const auto rs2 = nxt ? rs_next : rs_cur;
        w4_stage(C, rs2, ld, const_cast<char*>(cur), nxt ? k + 2 - nk : k + 2, 0, 16);
      }
      w4_mfma<false>(acc, ya, yb);
      DTD_W4_SCHED(16, 1, 1, 4);
    }
    // ---- tile done: epilogue, then the next tile
    w4_epilogue<BIAS>(acc, smem + LDS_BYTES + (it & 1) * 512, g.c, g.ldc, m0, n0, C);
    ++it;
    t += per;
    tile_of(t < end ? t : beg, ntn, m0, n0);
    rs_cur = rs_next;
    rs_next = panel(t + per < end ? t + per : t);
  }
}


// ---------------------------------------------------------------------------------------------
// "U2" (DTD_GEMM_VARIANT 2, removed): gemm_bt_persistent's K-step loop unrolled by two (K / 64
// even) so each K-step's LDS buffer is a compile-time constant, every K-step stages (the
// workgroup's last one a duplicate of its tile's K-step 0, drained before exit) so the phases have
// one counted vmcnt and no staging branch.  The constant-buffer fragment addressing needs more
// live address registers: 256 VGPRs with 14-20 spilled INTO the main loop -> 0.74-0.83x v1
// (profiles/r3_gemm_u2_experiment.jsonl).  A layout with both buffers' A (and B) halves within
// one 16-bit ds_read offset of a single base ([A0][A1][B0][B1]) would be the way to retry it.
// The K-step body, as it was written (a macro inside gemm_bt_persistent, CB = buffer, FIRST =
// first K-step after an epilogue):
// // One K-step of the U2 main loop (reads LDS buffer CB, stages the next K-step into the other);
// // used inside gemm_bt_persistent only
// #define DTD_KSTEP(CB, FIRST, KT_)                                                           \
//   do {                                                                                      \
//     constexpr bool first = (FIRST);                                                         \
//     const int kt = (KT_);                                                                   \
//     const char* cur = smem + (CB) * TILE_BYTES; \
//     char* nxt = smem + ((CB) ^ 1) * TILE_BYTES; \
//     const bool more_here = kt + 1 < nk; \
//     const auto sra = more_here ? rsa : (has_next ? rsa1 : rsa); \
//     const auto srb = more_here ? rsb : (has_next ? rsb1 : rsb); \
//     const int skt = more_here ? kt + 1 : 0; \
//     _Pragma("unroll")                                                                      \
//     for (int p = 0; p < 4; ++p) { \
//       if (p == 0 || p == 2) { \
//         const int qm = p == 0 ? 0 : 1; \
//     _Pragma("unroll")                                                                      \
//         for (int mi = 0; mi < 4; ++mi) { \
//           const char* rr = cur + arow + (qm * 4 + mi) * 16 * 128; \
//           af[mi][0] = *reinterpret_cast<const bf16x8*>(rr + ch0); \
//           af[mi][1] = *reinterpret_cast<const bf16x8*>(rr + ch1); \
//         } \
//       } \
//       if (p == 0 || p == 1) { \
//     _Pragma("unroll")                                                                      \
//         for (int ni = 0; ni < 2; ++ni) { \
//           const char* rr = cur + brow + (p * 2 + ni) * 16 * 128; \
//           bf16x8 x0 = *reinterpret_cast<const bf16x8*>(rr + ch0); \
//           bf16x8 x1 = *reinterpret_cast<const bf16x8*>(rr + ch1); \
//           if (p == 0) { b0[ni][0] = x0; b0[ni][1] = x1; } else { b1[ni][0] = x0; b1[ni][1] = x1; } \
//         } \
//       } \
//       if (p == 0) stage<0>(so, sra, srb, nxt, skt); \
//       if (p == 1) stage<1>(so, sra, srb, nxt, skt); \
//       if (p == 2) stage<2>(so, sra, srb, nxt, skt); \
//       if (p == 3) stage<3>(so, sra, srb, nxt, skt); \
//       if (first && p < 2) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(WAIT_FIRST) : "memory"); \
//       else asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); \
//       bar(); \
//       asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); \
//       __builtin_amdgcn_sched_barrier(0); \
//       __builtin_amdgcn_s_setprio(1); \
//       const int qm = (p == 2 || p == 3) ? 1 : 0; \
//     _Pragma("unroll")                                                                      \
//       for (int mi = 0; mi < 4; ++mi) \
//     _Pragma("unroll")                                                                      \
//         for (int ni = 0; ni < 2; ++ni) \
//     _Pragma("unroll")                                                                      \
//           for (int ks = 0; ks < 2; ++ks) { \
//             const bf16x8 bb = (p == 1 || p == 2) ? b1[ni][ks] : b0[ni][ks]; \
//             const int nn = ((p == 1 || p == 2) ? 2 : 0) + ni; \
//             acc[qm * 4 + mi][nn] = mfma16(bb, af[mi][ks], acc[qm * 4 + mi][nn]); \
//           } \
//       __builtin_amdgcn_s_setprio(0); \
//       bar(); \
//     } \
//   } while (0)
// 
//     if constexpr (U2) {
//       // K-step kt reading buffer CB; `first` (compile-time) selects the waits that also cover the
//       // previous tile's epilogue stores
//       DTD_KSTEP(0, true, 0);
//       DTD_KSTEP(1, false, 1);
//       for (int kt2 = 2; kt2 < nk; kt2 += 2) {
//         DTD_KSTEP(0, false, kt2);
//         DTD_KSTEP(1, false, kt2 + 1);
//       }
//       buf = 0;   // the last K-step read buffer 1 (the epilogue's image); buffer 0 holds the next K-step 0
//     } else {

// ---------------------------------------------------------------------------------------------
// Split-buffer form (DTD_GEMM_VARIANT 2, removed): LDS as [A0|A1|B0|B1] so every fragment read of
// either K-step buffer is one base register + a 16-bit immediate, K loop unrolled by two with
// compile-time buffers and branch-free staging -- the main loop compiles to reads / DMA / SALU /
// barriers / MFMAs with no VALU at all, yet 256 VGPRs + 15-18 spilled (stored before the loop,
// reloaded in the epilogue, where the scratch reload's vmcnt wait also drains the next tile's
// K-step-0 DMA): 0.77-0.81x v1 on every BERT shape, fused epilogues included, -3.5 % whole step
// (profiles/r3_gemm_split_experiment.jsonl).  The code as it was:
// 
// // ---- split-buffer form (DTD_GEMM_VARIANT 2, K / 64 even) --------------------------------------
// // LDS as [A0 | A1 | B0 | B1] (32 KiB each) instead of [A0 B0 | A1 B1]: every fragment read of
// // either K-step buffer is then one per-lane base register + a 16-bit immediate (buffer 1 is +32
// // KiB), so the K-step loop can be unrolled by two with compile-time buffers and NO per-phase
// // address arithmetic; every K-step stages (the workgroup's last one a duplicate of its tile's
// // K-step 0, drained before exit), so each phase has one counted vmcnt and no staging branch.
// __device__ __forceinline__ StageOffs stage_offsets2(int w, int lane, int lda, int ldb) {
//   StageOffs o = stage_offsets(w, lane, lda, ldb);
// #pragma unroll
//   for (int h = 0; h < 2; ++h)
// #pragma unroll
//     for (int i = 0; i < 2; ++i) o.lb[h][i] -= A_BYTES;   // B rows relative to their own half
//   return o;
// }
// template <int H>
// __device__ __forceinline__ void stage2(const StageOffs& o, __amdgpu_buffer_rsrc_t ra, __amdgpu_buffer_rsrc_t rb,
//                                        char* abuf, char* bbuf, int kt) {
//   const int so = kt * BK * 2;
// #pragma unroll
//   for (int i = 0; i < 2; ++i) {
//     if constexpr (H == 0 || H == 3) {
//       constexpr int h = H == 3 ? 1 : 0;
//       __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_void*)(abuf + o.la[h][i]), 16, o.a[h][i], so, 0, 0);
//     } else {
//       constexpr int h = H == 2 ? 1 : 0;
//       __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (lds_void*)(bbuf + o.lb[h][i]), 16, o.b[h][i], so, 0, 0);
//     }
//   }
// }
// // one K-step of gemm_bt_persistent2: reads buffer CB, stages the next K-step into buffer CB ^ 1
// #define DTD_KSTEP2(CB, FIRST, KT_)                                                                  \
//   do {                                                                                             \
//     constexpr bool first = (FIRST);                                                                \
//     const int kt = (KT_);                                                                          \
//     const char* ca = smem + (CB) * A_BYTES;                                                         \
//     char* na = smem + ((CB) ^ 1) * A_BYTES;                                                         \
//     char* nb = smem + 2 * A_BYTES + ((CB) ^ 1) * A_BYTES;                                           \
//     const bool more_here = kt + 1 < nk;                                                            \
//     const auto sra = more_here ? rsa : (has_next ? rsa1 : rsa);                                     \
//     const auto srb = more_here ? rsb : (has_next ? rsb1 : rsb);                                     \
//     const int skt = more_here ? kt + 1 : 0;                                                        \
//     _Pragma("unroll") for (int p = 0; p < 4; ++p) {                                                \
//       if (p == 0 || p == 2) {                                                                      \
//         const int qm = p == 0 ? 0 : 1;                                                             \
//         _Pragma("unroll") for (int mi = 0; mi < 4; ++mi) {                                         \
//           const char* rr = ca + arow + (qm * 4 + mi) * 16 * 128;                                   \
//           af[mi][0] = *reinterpret_cast<const bf16x8*>(rr + ch0);                                  \
//           af[mi][1] = *reinterpret_cast<const bf16x8*>(rr + ch1);                                  \
//         }                                                                                          \
//       }                                                                                            \
//       if (p == 0 || p == 1) {                                                                      \
//         _Pragma("unroll") for (int ni = 0; ni < 2; ++ni) {                                         \
//           const char* rr = ca + brow + (p * 2 + ni) * 16 * 128;                                    \
//           const bf16x8 x0 = *reinterpret_cast<const bf16x8*>(rr + ch0);                            \
//           const bf16x8 x1 = *reinterpret_cast<const bf16x8*>(rr + ch1);                            \
//           if (p == 0) { b0[ni][0] = x0; b0[ni][1] = x1; } else { b1[ni][0] = x0; b1[ni][1] = x1; } \
//         }                                                                                          \
//       }                                                                                            \
//       if (p == 0) stage2<0>(so, sra, srb, na, nb, skt);                                            \
//       if (p == 1) stage2<1>(so, sra, srb, na, nb, skt);                                            \
//       if (p == 2) stage2<2>(so, sra, srb, na, nb, skt);                                            \
//       if (p == 3) stage2<3>(so, sra, srb, na, nb, skt);                                            \
//       if (first && p < 2) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(WAIT_FIRST) : "memory");      \
//       else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");                                        \
//       bar();                                                                                       \
//       asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                           \
//       __builtin_amdgcn_sched_barrier(0);                                                           \
//       __builtin_amdgcn_s_setprio(1);                                                               \
//       const int qm = (p == 2 || p == 3) ? 1 : 0;                                                   \
//       _Pragma("unroll") for (int mi = 0; mi < 4; ++mi)                                             \
//         _Pragma("unroll") for (int ni = 0; ni < 2; ++ni)                                           \
//           _Pragma("unroll") for (int ks = 0; ks < 2; ++ks) {                                       \
//             const bf16x8 bb = (p == 1 || p == 2) ? b1[ni][ks] : b0[ni][ks];                        \
//             const int nn = ((p == 1 || p == 2) ? 2 : 0) + ni;                                      \
//             acc[qm * 4 + mi][nn] = mfma16(bb, af[mi][ks], acc[qm * 4 + mi][nn]);                   \
//           }                                                                                        \
//       __builtin_amdgcn_s_setprio(0);                                                               \
//       bar();                                                                                       \
//     }                                                                                              \
//   } while (0)
// 
// template <int EPI, bool DYN>
// __global__ void __launch_bounds__(512, 2) gemm_bt_persistent2(GemmArgs g) {
//   __shared__ __attribute__((aligned(1024))) char smem[LDS_BYTES];
//   // the wave index through readfirstlane: provably uniform, so the LDS-DMA destinations (M0) are
//   // formed with scalar adds instead of a v_readfirstlane per DMA (-11 % VALU; +2-3 % vs hipBLASLt
//   // on the BERT projection shapes, profiles/r3_gemm_u2_experiment.jsonl)
//   const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
//   const int li = lane & 15, lq = lane >> 4, sw = li & 7;
//   const int wm = w >> 2, wn = w & 3;
//   const int ntn = g.N / BN, ntiles = (g.M / BM) * ntn;
//   const int nk = g.K / BK;
//   // tile sequence of this workgroup: XCD group x gets tiles [beg, end), member l takes beg + l + 32 i
//   const int nwg = gridDim.x, x = blockIdx.x % 8, l = blockIdx.x / 8, per = nwg / 8;
//   const int q = ntiles / 8, r = ntiles % 8;
//   const int beg = x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q;
//   const int end = beg + q + (x < r ? 1 : 0);
//   constexpr bool dyn = DYN;   // g.sched != null (a separate instantiation keeps SGPR pressure)
//   // dynamic queue: a workgroup's first two tiles are the static order's (no claims at launch,
//   // where 256 workgroups would contend for 8 counters); queue entry c is tile beg + 2 per + c.
//   // Iteration j >= 1 reads the tile of iteration j + 1 from qslot[j & 1].
//   __shared__ int qslot[2];
//   int t = beg + l;
//   if (t >= end) {   // more workgroups than tiles in this group (small problems) / queue drained
//     if constexpr (DYN) sched_finish(g.sched, nwg, tid);
//     return;
//   }
//   int m0, n0;
//   tile_of(t, ntn, m0, n0);
//   const StageOffs so = stage_offsets2(w, lane, g.lda, g.ldb);
//   auto rsa = uniform_rsrc(g.a + (size_t)m0 * g.lda), rsb = uniform_rsrc(g.b + (size_t)n0 * g.ldb);
//   stage2<0>(so, rsa, rsb, smem, smem + 2 * A_BYTES, 0);
//   stage2<1>(so, rsa, rsb, smem, smem + 2 * A_BYTES, 0);
//   stage2<2>(so, rsa, rsb, smem, smem + 2 * A_BYTES, 0);
//   stage2<3>(so, rsa, rsb, smem, smem + 2 * A_BYTES, 0);
//   asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
//   __syncthreads();
//   if (__builtin_amdgcn_readfirstlane(wm) == 1) bar();   // stagger wave row 1
// 
//   const int arow = (wm * 128 + li) * 128;
//   const int brow = 2 * A_BYTES + (wn * 64 + li) * 128;   // B halves at 64 KiB
//   const int ch0 = ((0 * 4 + lq) ^ sw) * 16, ch1 = ((1 * 4 + lq) ^ sw) * 16;
//   constexpr int S = kStores(EPI);
//   constexpr int WAIT_FIRST = 4 + S > 63 ? 63 : 4 + S;
// 
//   bf16x8 af[4][2], b0[2][2], b1[2][2];
//   f32x4 acc[8][4];
//   int it = 0;
//   STAMP_ID(0);
//   while (true) {
//     STAMP(0, it);
//     const int tn = dyn && it > 0 ? __builtin_amdgcn_readfirstlane(qslot[it & 1]) : t + per;
//     const bool has_next = tn < end;
//     int m1 = 0, n1 = 0;
//     if (has_next) tile_of(tn, ntn, m1, n1);
//     const auto rsa1 = uniform_rsrc(g.a + (size_t)m1 * g.lda), rsb1 = uniform_rsrc(g.b + (size_t)n1 * g.ldb);
// #pragma unroll
//     for (int i = 0; i < 8; ++i)
// #pragma unroll
//       for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
// 
//     // K-steps in pairs: buffer 0 then 1, compile-time (nk is even: host check)
//     DTD_KSTEP2(0, true, 0);
//     DTD_KSTEP2(1, false, 1);
//     for (int kt2 = 2; kt2 < nk; kt2 += 2) {
//       DTD_KSTEP2(0, false, kt2);
//       DTD_KSTEP2(1, false, kt2 + 1);
//     }
// 
//     STAMP(2, it);
//     // ---- epilogue through the free LDS buffer (the last K-step's; the other one holds the
//     //      next tile's K-step 0), in two rounds of 128 rows: the wave row r writes its
//     //      accumulators (fp32 bias / residual, one bf16 rounding) as a [128][512 B] image
//     //      (8-byte slots XOR-swizzled by row & 15), then all 8 waves store 16 rows each as
//     //      512-byte row segments of 16-byte vectors.
//     // accumulators -> packed bf16 first (fp32 bias / residual, one rounding): halves the live
//     // registers for the rest of the epilogue
//     bf16x4 pk[8][4];
//     if constexpr (EPI == EPI_ADD) {
//       const auto rs = uniform_rsrc(g.c + (size_t)(m0 + wm * 128) * g.ldc + n0 + wn * 64);
//       const int voff = (li * g.ldc + 4 * lq) * 2;
// #pragma unroll
//       for (int h = 0; h < 2; ++h) {
//         bf16x4 cin[4][4];
// #pragma unroll
//         for (int mi = 0; mi < 4; ++mi)
// #pragma unroll
//           for (int ni = 0; ni < 4; ++ni)
//             cin[mi][ni] = __builtin_bit_cast(bf16x4, __builtin_amdgcn_raw_buffer_load_b64(
//                                                          rs, voff + ni * 32, (h * 4 + mi) * 16 * g.ldc * 2, 0));
// #pragma unroll
//         for (int mi = 0; mi < 4; ++mi)
// #pragma unroll
//           for (int ni = 0; ni < 4; ++ni)
// #pragma unroll
//             for (int k = 0; k < 4; ++k)
//               pk[h * 4 + mi][ni][k] = (bf16)(acc[h * 4 + mi][ni][k] + (float)cin[mi][ni][k]);
//       }
//     } else {
// #pragma unroll
//       for (int ni = 0; ni < 4; ++ni) {
//         float bv[4] = {0.f, 0.f, 0.f, 0.f};
//         if constexpr (EPI == EPI_STORE || is_gelu_fwd(EPI)) {
//           if (g.bias) {
//             const bf16x4 b4 = *reinterpret_cast<const bf16x4*>(g.bias + n0 + wn * 64 + ni * 16 + 4 * lq);
// #pragma unroll
//             for (int k = 0; k < 4; ++k) bv[k] = (float)b4[k];
//           }
//         }
// #pragma unroll
//         for (int mi = 0; mi < 8; ++mi)
// #pragma unroll
//           for (int k = 0; k < 4; ++k) pk[mi][ni][k] = (bf16)(acc[mi][ni][k] + bv[k]);
//       }
//     }
//     if (__builtin_amdgcn_readfirstlane(wm) == 0) bar();   // close the stagger
//     bar();                                                // every wave is done with `img`
//     // the image in the last K-step's buffer (1): rows 0-63 in its A half, 64-127 in its B half
//     char* const imgA = smem + A_BYTES;
//     char* const imgB = smem + 3 * A_BYTES - 64 * 512;
//     const int c = lane & 31;
//     // row-phase inputs first (GELU_BWD: U), so no later load wait holds back a store
//     bf16x8 uin[2][8];
//     if constexpr (is_gelu_bwd(EPI)) {
//       const auto rs = uniform_rsrc(g.u + (size_t)m0 * g.ldu + n0);
//       const int voff = ((w * 16 + (lane >> 5)) * g.ldu + c * 8) * 2;
// #pragma unroll
//       for (int rr = 0; rr < 2; ++rr)
// #pragma unroll
//         for (int i = 0; i < 8; ++i)
//           uin[rr][i] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(
//                                                       rs, voff, (rr * 128 + 2 * i) * g.ldu * 2, 0));
//     }
//     float colsum[8];
// #pragma unroll
//     for (int j = 0; j < 8; ++j) colsum[j] = 0.f;
//     int claim = 0;
// #pragma unroll
//     for (int rr = 0; rr < 2; ++rr) {
//       // dynamic queue: claim the tile after the next one when the second round starts (every load
//       // of the epilogue is older, so no counted wait for them waits for the atomic as well);
//       // publish it when the round ends
//       if (dyn && rr == 1 && has_next && tid == 0) claim = atomicAdd(&g.sched[x], 1);
//       if (__builtin_amdgcn_readfirstlane(wm) == rr) {
// #pragma unroll
//         for (int ni = 0; ni < 4; ++ni) {
//           const int n = wn * 64 + ni * 16 + 4 * lq;
// #pragma unroll
//           for (int mi = 0; mi < 8; ++mi) {
//             const int m = mi * 16 + li;   // row within the round's 128
//             *reinterpret_cast<bf16x4*>((mi < 4 ? imgA : imgB) + m * 512 + (((n >> 2) ^ (m & 15)) << 3)) = pk[mi][ni];
//           }
//         }
//       }
//       bar();
// #pragma unroll
//       for (int i = 0; i < 8; ++i) {
//         const int r = w * 16 + 2 * i + (lane >> 5);   // row within the round
//         const int x = r & 15;
//         bf16x8 v = *reinterpret_cast<const bf16x8*>((w < 4 ? imgA : imgB) + r * 512 + ((c ^ (x >> 1)) << 4));
//         if (x & 1) v = __builtin_shufflevector(v, v, 4, 5, 6, 7, 0, 1, 2, 3);
//         const size_t off = (size_t)(m0 + rr * 128 + r) * g.ldc + n0 + c * 8;
//         if constexpr (EPI == EPI_STORE || EPI == EPI_ADD) {
//           *reinterpret_cast<bf16x8*>(g.c + off) = v;
//         } else if constexpr (stores_grad(EPI)) {
//           bf16x8 av, dv;
// #pragma unroll
//           for (int j = 0; j < 8; ++j) {
//             float aj, dj;
//             epi_act_and_grad<EPI>((float)v[j], aj, dj);
//             av[j] = (bf16)aj;
//             dv[j] = (bf16)dj;
//           }
//           *reinterpret_cast<bf16x8*>(g.c + off) = dv;
//           *reinterpret_cast<bf16x8*>(g.c2 + off) = av;
//         } else if constexpr (is_gelu_fwd(EPI)) {
//           bf16x8 av;
// #pragma unroll
//           for (int j = 0; j < 8; ++j) av[j] = (bf16)epi_act<EPI>((float)v[j]);
//           *reinterpret_cast<bf16x8*>(g.c + off) = v;
//           *reinterpret_cast<bf16x8*>(g.c2 + off) = av;
//         } else {
//           bf16x8 o;
// #pragma unroll
//           for (int j = 0; j < 8; ++j) {
//             const float du = (float)v[j] * epi_act_grad<EPI>((float)uin[rr][i][j]);
//             o[j] = (bf16)du;
//             colsum[j] += du;
//           }
//           *reinterpret_cast<bf16x8*>(g.c + off) = o;
//         }
//       }
//       if (dyn && rr == 1 && tid == 0) qslot[(it + 1) & 1] = has_next ? beg + 2 * per + claim : end;
//       bar();   // the image is consumed before it is rewritten / restaged
//     }
//     if constexpr (is_gelu_bwd(EPI)) {
//       // lanes c and c+32 hold the same columns; the 8 waves combine through LDS: one fp32
//       // partial row per 256-row tile
// #pragma unroll
//       for (int j = 0; j < 8; ++j) colsum[j] += __shfl_xor(colsum[j], 32, 64);
//       float* red = reinterpret_cast<float*>(imgA);
//       if (lane < 32) {
//         *reinterpret_cast<f32x4*>(red + w * 256 + c * 8) = f32x4{colsum[0], colsum[1], colsum[2], colsum[3]};
//         *reinterpret_cast<f32x4*>(red + w * 256 + c * 8 + 4) = f32x4{colsum[4], colsum[5], colsum[6], colsum[7]};
//       }
//       bar();
//       if (tid < 256 && g.part) {
//         float sum = 0.f;
// #pragma unroll
//         for (int k = 0; k < 8; ++k) sum += red[k * 256 + tid];
//         g.part[(size_t)(m0 >> 8) * g.N + n0 + tid] = sum;
//       }
//       bar();
//     }
//     if (has_next && __builtin_amdgcn_readfirstlane(wm) == 1) bar();   // reopen the stagger
//     STAMP(4, it);
//     ++it;
//     if (!has_next) break;
//     t = tn;
//     m0 = m1;
//     n0 = n1;
//     rsa = rsa1;
//     rsb = rsb1;
//   }
//   asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the last K-step's duplicate stage
//   if constexpr (DYN) sched_finish(g.sched, nwg, tid);
// }
// 
// #undef DTD_KSTEP2
// 


// ---------------------------------------------------------------------------------------------
// Round 3b: register-staged B panel in gemm_bt_persistent (was DTD_GEMM_REGB=1).  After the
// limiter probe (profiles/r3_gemm_limiter_probe.jsonl: LDS-DMA issue is the main-loop limiter,
// ~90 cycles per buffer_load...lds among the phase's ds_reads; halving the DMA count recovers most
// of the gap to the no-staging ceiling), the B half-tiles went through registers: global loads at
// phases 1 / 2 into 2 x 16 B per lane, ds_write_b128 one phase later to the DMA's lane-linear image.
// 252 VGPRs, no spill, tests/test_gemm_gpu.py 39 passed -- and 0.70x the DMA form (qkv 622 vs 443 us,
// fc2 758 vs 471 us): the phase-2 / phase-3 waits retire loads issued one phase earlier, which the
// L2 round trip does not meet (a two-phase register ring needs 16 more VGPRs: spills).  Removed.
//   main loop (non-first K-steps, `more`):
//     p0: stage<0>(A lo DMA);            vmcnt(4)
//     p1: load_b<0>(B lo -> regs);       vmcnt(4)
//     p2: vmcnt(0); store_b<0>(regs -> LDS); load_b<1>(B hi -> regs)
//     p3: stage<3>(A hi DMA); vmcnt(2);  store_b<1>(regs -> LDS)
// // Register-staged form of stage<1> / stage<2> (B rows lo / hi half): the same per-lane source
// // (swizzled chunk) and the same lane-linear LDS destination as the LDS-DMA, as a global load into
// // two 16-byte registers and, one phase later, two ds_write_b128.  An LDS-DMA instruction costs the
// // issuing wave ~90 cycles among the phase's LDS reads (profiles/r3_gemm_limiter_probe.jsonl); the
// // load + store pair a fraction of that.
// template <int HB>
// __device__ __forceinline__ void load_b(const StageOffs& o, __amdgpu_buffer_rsrc_t rb, int kt, bf16x8 (&r)[2]) {
//   const int so = kt * BK * 2;
// #pragma unroll
//   for (int i = 0; i < 2; ++i)
//     r[i] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rb, o.b[HB][i], so, 0));
// }
// template <int HB>
// __device__ __forceinline__ void store_b(const StageOffs& o, char* buf, int lane, const bf16x8 (&r)[2]) {
// #pragma unroll
//   for (int i = 0; i < 2; ++i) *reinterpret_cast<bf16x8*>(buf + o.lb[HB][i] + lane * 16) = r[i];
// }

// ---------------------------------------------------------------------------------------------
// Round 3b: LDS-DMA placement / priority in the persistent main loop (scripts/gemm_diag.py, same
// box, 2 rounds; GEMM tests pass under each): DMA issued BEFORE the phase's fragment reads 0.63x
// (the reads queue behind the DMA's LDS writes and the MFMA segment waits on them); DMA in the
// middle of the MFMA segment 0.78x; no s_setprio around the MFMA segments 0.90x; both 0.75x; one
// barrier per phase without the wave-row stagger 0.95x.  The shipped order (reads, then DMA, then
// the counted wait and barrier; MFMA segment at priority 1) is the best of the set.

// ---------------------------------------------------------------------------------------------
// Round 3b: W4R -- the 4-wave (one per SIMD, 128x128 per wave) form with the operands staged
// through registers instead of LDS-DMA (the LDS-DMA issue cost the W4 form could not hide).
// Built into gemm.hip as DTD_GEMM_VARIANT=4 for EPI_STORE, launched like the persistent kernel
// (nwg workgroups of 256 threads):
//     if (gemm_variant() == 4 && epi == EPI_STORE && K / BK >= 2) {
//       if (bias) hipLaunchKernelGGL((gemm_bt_w4r<true>), dim3(nwg), dim3(256), 0, s, g);
//       else hipLaunchKernelGGL((gemm_bt_w4r<false>), dim3(nwg), dim3(256), 0, s, g);
//     }
// Correct (scripts/bench_gemm_v2.py checks, tests/test_gemm_gpu.py 39 passed under it).  Timing
// (VNEW=4 scripts/bench_gemm_v2.py, same box): first version with the staging / next-step reads
// behind runtime conditions 0.57-0.69x v1 (the branches split the K-step into basic blocks, so the
// sched_group_barrier interleave did not apply: reads, stores and loads clumped beside idle MFMA
// issue); branch-free K-step 0.79-0.89x v1 (e.g. fwd qkv 507 vs 438 us, fc2 542 vs 464 us,
// hipBLASLt 388 / 437).  512 VGPRs (256 accumulators, 128 for the double-buffered X / Y
// fragments, 32 staging): the half-K-step staging ring leaves each load one MFMA part (~1 k cycles)
// before its ds_write, and a lone wave stalls its whole MFMA stream on that vmcnt.  Next step if
// revisited: stream the A fragments per 16-row block (8 instead of 32 registers per k-half), which
// frees the registers for a full K-step staging ring (two parts of load distance).  Upper bound of
// that fix, measured with the loads re-reading an L2-hot K-step (timing only): 0.91-0.97x v1.
// // ---------------------------------------------------------------------------------------------
// // W4R form (DTD_GEMM_VARIANT=4; EPI_STORE, optional bias; K >= 128): FOUR waves, one per SIMD,
// // each owning a 128 x 128 quarter of the 256 x 256 tile in 256 fp32 accumulators (a wave alone on
// // its SIMD may use the whole 512-entry register file).  Per K-step a wave reads 32 fragments for
// // 128 MFMAs (0.25 reads per MFMA against 0.375 in the 8-wave form) and the operands are staged
// // through REGISTERS: 16 global loads into 64 VGPRs and 16 ds_write_b128 a K-step later -- the
// // 8-wave form's limiter is the ~90-cycle issue of each buffer_load...lds (profiles/
// // r3_gemm_limiter_probe.jsonl), and one wave per SIMD has no partner to hide it behind (the
// // LDS-DMA version of this schedule ran 0.65-0.80x, scripts/experiments/gemm_variants_r3.hip).
// //   K-step g (buffer g & 1): part 1 = MFMAs of k-half 0 (fragments X) beside the k-half 1 reads
// //   (Y); barrier; part 2 = MFMAs of k-half 1 (Y) beside the k-half 0 reads of K-step g + 1 (X), the
// //   LDS stores of K-step g + 2 into buffer g & 1 (read out in part 1) and the global loads of
// //   K-step g + 3.  One barrier per K-step plus one per part boundary.
// // The staging image is the LDS-DMA one (lane-linear 1 KiB pieces, source-side chunk swizzle), so
// // the fragment reads are those of the 8-wave kernel.  Persistent XCD-grouped static tile order;
// // a tile's epilogue stores 16-byte row pieces straight from the accumulators (v_permlane16_swap).
// constexpr int W4R_LDS = LDS_BYTES + 1024;
//
// struct W4Ctx {
//   int voff;           // per-lane source offset (row L/8 of an 8-row piece, swizzled chunk)
//   int abase, bbase;   // per-lane fragment read offsets within a K-step buffer (chunk of k-half 0)
//   int kh1;            // byte delta from the k-half 0 chunk to the k-half 1 chunk
//   int w, wm, wn, li, lq, lane;
// };
//
// // half H (8 of this wave's 16 pieces, 1 KiB each) of K-step `kk` of the operand panel `rs` ->
// // registers, and registers -> the lane-linear LDS image of a K-step buffer
// __device__ __forceinline__ void w4r_load(const W4Ctx& C, __amdgpu_buffer_rsrc_t rs, int ld, int kk, int H,
//                                          bf16x8 (&st)[8]) {
// #pragma unroll
//   for (int i = 0; i < 8; ++i)
//     st[i] = __builtin_bit_cast(bf16x8,
//                                __builtin_amdgcn_raw_buffer_load_b128(rs, C.voff, kk * BK * 2 + (H * 8 + i) * 16 * ld, 0));
// }
// __device__ __forceinline__ void w4r_write(const W4Ctx& C, char* buf, int H, const bf16x8 (&st)[8]) {
// #pragma unroll
//   for (int i = 0; i < 8; ++i) *reinterpret_cast<bf16x8*>(buf + (C.w * 16 + H * 8 + i) * 1024 + C.lane * 16) = st[i];
// }
//
// __device__ __forceinline__ uint32_t pack2(float a, float b) {
//   typedef float f32x2_t __attribute__((ext_vector_type(2)));
//   return __builtin_bit_cast(uint32_t, __builtin_convertvector(f32x2_t{a, b}, bf16x2));
// }
//
// template <bool BIAS>
// __device__ __forceinline__ void w4r_epilogue(const f32x4 (&acc)[8][8], const char* bias_lds, bf16* __restrict__ c,
//                                              int ldc, int m0, int n0, const W4Ctx& C) {
//   const int ecol = (C.lq & 1) * 16 + (C.lq >> 1) * 8;
//   bf16* base = c + (size_t)(m0 + C.wm * 128 + C.li) * ldc + n0 + C.wn * 128 + ecol;
// #pragma unroll
//   for (int nb = 0; nb < 8; nb += 2) {
//     f32x4 bx = {0.f, 0.f, 0.f, 0.f}, by = {0.f, 0.f, 0.f, 0.f};
//     if constexpr (BIAS) {
//       bx = __builtin_convertvector(*reinterpret_cast<const bf16x4*>(bias_lds + (C.wn * 128 + nb * 16 + 4 * C.lq) * 2), f32x4);
//       by = __builtin_convertvector(*reinterpret_cast<const bf16x4*>(bias_lds + (C.wn * 128 + (nb + 1) * 16 + 4 * C.lq) * 2), f32x4);
//     }
// #pragma unroll
//     for (int mb = 0; mb < 8; ++mb) {
//       const f32x4 X = acc[mb][nb] + bx, Y = acc[mb][nb + 1] + by;
//       const uint32_t x0 = pack2(X[0], X[1]), x1 = pack2(X[2], X[3]);
//       const uint32_t y0 = pack2(Y[0], Y[1]), y1 = pack2(Y[2], Y[3]);
//       const auto s0 = __builtin_amdgcn_permlane16_swap(x0, y0, false, false);
//       const auto s1 = __builtin_amdgcn_permlane16_swap(x1, y1, false, false);
//       typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
//       const u32x4 v = {s0[0], s1[0], s0[1], s1[1]};
//       *reinterpret_cast<u32x4*>(base + (size_t)mb * 16 * ldc + nb * 16) = v;
//     }
//   }
// }
//
// // fragments of one k-half: A[mb] (8) and B[nb] (8) of the wave's quarter
// __device__ __forceinline__ void w4r_read(const char* buf, const W4Ctx& C, int kh, bf16x8 (&fa)[8], bf16x8 (&fb)[8]) {
//   const char* pa = buf + C.abase + kh * C.kh1;
//   const char* pb = buf + C.bbase + kh * C.kh1;
// #pragma unroll
//   for (int i = 0; i < 8; ++i) {
//     fa[i] = *reinterpret_cast<const bf16x8*>(pa + i * 2048);
//     fb[i] = *reinterpret_cast<const bf16x8*>(pb + i * 2048);
//   }
// }
//
// template <bool ZERO>
// __device__ __forceinline__ void w4r_mfma(f32x4 (&acc)[8][8], const bf16x8 (&fa)[8], const bf16x8 (&fb)[8]) {
// #pragma unroll
//   for (int mb = 0; mb < 8; ++mb)
// #pragma unroll
//     for (int nb = 0; nb < 8; ++nb)
//       acc[mb][nb] = mfma16(fb[nb], fa[mb], ZERO ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[mb][nb]);
// }
//
// // interleave per group: NDS LDS reads, NDW LDS writes, NVM VMEM loads, NMF MFMAs
// #define DTD_W4R_SCHED(GROUPS, NDS, NDW, NVM, NMF)                            \
//   do {                                                                       \
//     _Pragma("unroll") for (int _g = 0; _g < (GROUPS); ++_g) {                \
//       if ((NDS) > 0) __builtin_amdgcn_sched_group_barrier(0x100, (NDS), 0);  \
//       if ((NDW) > 0) __builtin_amdgcn_sched_group_barrier(0x200, (NDW), 0);  \
//       if ((NVM) > 0) __builtin_amdgcn_sched_group_barrier(0x020, (NVM), 0);  \
//       __builtin_amdgcn_sched_group_barrier(0x008, (NMF), 0);                 \
//     }                                                                        \
//   } while (0)
//
// template <bool BIAS>
// __global__ void __launch_bounds__(256, 1) gemm_bt_w4r(GemmArgs g) {
//   __shared__ __attribute__((aligned(1024))) char smem[W4R_LDS];
//   const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
//   W4Ctx C;
//   C.w = w; C.wm = w >> 1; C.wn = w & 1; C.li = lane & 15; C.lq = lane >> 4; C.lane = lane;
//   const int ntn = g.N / BN, ntiles = (g.M / BM) * ntn;
//   const int nk = g.K / BK;   // >= 2 (host check)
//   const int nwg = gridDim.x, x = blockIdx.x % 8, l = blockIdx.x / 8, per = nwg / 8;
//   const int q = ntiles / 8, r = ntiles % 8;
//   const int beg = x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q;
//   const int end = beg + q + (x < r ? 1 : 0);
//   int t = beg + l;
//   if (t >= end) return;
//   const int ntl = (end - t + per - 1) / per;   // tiles of this workgroup
//   const int ng = ntl * nk;                     // its K-steps
//   // staging: waves 0-1 carry A rows, 2-3 B rows; lane L -> row L/8 of an 8-row piece, chunk slot
//   // L%8 <- global chunk (L%8) ^ (L/8) (the involutive swizzle of the fragment reads)
//   const bool isb = w >= 2;
//   const int ld = isb ? g.ldb : g.lda;
//   C.voff = ((((w & 1) * 16 * 8) + (lane >> 3)) * ld + (((lane & 7) ^ (lane >> 3)) * 8)) * 2;
//   const int sw = C.li & 7;
//   C.abase = (C.wm * 128 + C.li) * 128 + ((C.lq ^ sw) * 16);
//   C.bbase = A_BYTES + (C.wn * 128 + C.li) * 128 + ((C.lq ^ sw) * 16);
//   C.kh1 = (((4 + C.lq) ^ sw) - (C.lq ^ sw)) * 16;
//   auto panel = [&](int tile) {   // this wave's operand panel of `tile`
//     int tm0, tn0;
//     tile_of(tile, ntn, tm0, tn0);
//     return uniform_rsrc(isb ? (const void*)(g.b + (size_t)tn0 * g.ldb) : (const void*)(g.a + (size_t)tm0 * g.lda));
//   };
//   const auto rbias = uniform_rsrc(BIAS ? (const void*)g.bias : (const void*)g.a);
//   auto rs_cur = panel(t);
//   auto rs_next = panel(t + per < end ? t + per : t);
//   // source of global K-step gs + d relative to the tile of local step k (the next tile past nk)
//   // staging ring of half a K-step (8 pieces): K-step s's half 0 is loaded in part 1 of K-step
//   // s - 2 and stored in its part 2, half 1 loaded in part 2 of s - 2 and stored in part 1 of s - 1
//   // (both into buffer s & 1, free from part 2 of s - 2 on, read from part 2 of s - 1 on)
//   bf16x8 st[8];
//   // prologue: K-steps 0 and 1 into the two buffers, K-step 2's first half in flight
//   for (int kk = 0; kk < 2; ++kk)
//     for (int H = 0; H < 2; ++H) {
//       w4r_load(C, rs_cur, ld, kk, H, st);
//       w4r_write(C, smem + kk * TILE_BYTES, H, st);
//     }
//   auto src = [&](int k, int d, int& kk) {   // panel and tile-local K-step of local step k + d
//     const bool nxt = k + d >= nk;
//     kk = nxt ? k + d - nk : k + d;
//     return nxt ? rs_next : rs_cur;
//   };
//   asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
//   bar();
//   bf16x8 xa[8], xb[8], ya[8], yb[8];
//   w4r_read(smem, C, 0, xa, xb);
//   f32x4 acc[8][8];
//   int m0, n0;
//   tile_of(t, ntn, m0, n0);
//   int it = 0;   // tile iteration of this workgroup
//   // One K-step, branch-free (one basic block, so the sched_group_barrier interleave applies):
//   // past the workgroup's last K-steps the loads re-read a valid panel and the stores / reads touch
//   // buffers nobody consumes any more; the first K-step after the prologue re-stores the prologue's
//   // last half (identical bytes).
//   int gs = 0;
//   auto kstep = [&](auto first_c, int k) {
//     constexpr bool first = decltype(first_c)::value;
//     char* cur = smem + (gs & 1) * TILE_BYTES;
//     char* oth = smem + ((gs & 1) ^ 1) * TILE_BYTES;
//     int kk;
//     const auto rs2 = src(k, 2, kk);
//     // ---- part 1: k-half 0 MFMAs (X) | k-half 1 reads (Y) | K-step gs + 1's second half stored
//     //      (into `oth`, read from part 2 on) | K-step gs + 2's first half loaded
//     w4r_read(cur, C, 1, ya, yb);
//     w4r_write(C, oth, 1, st);
//     w4r_load(C, rs2, ld, kk, 0, st);
//     w4r_mfma<first>(acc, xa, xb);
//     DTD_W4R_SCHED(8, 2, 1, 1, 8);
//     asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // Y in registers, the stores done
//     bar();
//     // ---- part 2: k-half 1 MFMAs (Y) | k-half 0 reads of K-step gs + 1 (X) | K-step gs + 2's
//     //      first half stored into `cur` (read out in part 1), its second half loaded
//     w4r_read(oth, C, 0, xa, xb);
//     if constexpr (BIAS && first) {   // this tile's bias -> its LDS slot (waves 0-1), read in its epilogue
//       __builtin_amdgcn_raw_ptr_buffer_load_lds(rbias, (lds_void*)(smem + LDS_BYTES + (it & 1) * 512 + (w & 1) * 256),
//                                                 4, (n0 + (w & 1) * 128) * 2 + lane * 4, 0, 0, 0);
//     }
//     w4r_write(C, cur, 0, st);
//     w4r_load(C, rs2, ld, kk, 1, st);
//     w4r_mfma<false>(acc, ya, yb);
//     DTD_W4R_SCHED(8, 2, 1, 1, 8);
//     ++gs;
//   };
//   for (int gs0 = 0; gs0 < ng; gs0 += nk) {   // one tile
//     kstep(std::true_type{}, 0);
//     for (int k = 1; k < nk; ++k) kstep(std::false_type{}, k);
//     // ---- tile done: epilogue, then the next tile
//     asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the bias LDS-DMA (waves 0-1)
//     bar();
//     w4r_epilogue<BIAS>(acc, smem + LDS_BYTES + (it & 1) * 512, g.c, g.ldc, m0, n0, C);
//     ++it;
//     t += per;
//     tile_of(t < end ? t : beg, ntn, m0, n0);
//     rs_cur = rs_next;
//     rs_next = panel(t + per < end ? t + per : t);
//   }
// }
