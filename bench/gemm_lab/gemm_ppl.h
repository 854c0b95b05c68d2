// Lab only (bench/gemm_lab): the ping-pong GEMM of ops/csrc/gemm_pp.h with
// DEDICATED LOADER WAVES.  The 8 math waves keep the two staggered groups
// (read interval / matrix interval, gemm_pp.h header) but issue no LDS-DMA at
// all; NL extra waves issue every piece of every K-tile.  Why: an LDS-DMA issue
// holds its wave 100-185 cycles inside a read burst (MI355X_MICROARCH.md,
// LDS-DMA piece issue cost), so cfg 19's read interval (16 ds_read_b128 + 6
// pieces per wave) measured ~2x the partner group's 512-cycle MFMA interval;
// with the pieces on other waves the read interval is the ds_reads alone.
//
// Loader schedule, in the math groups' barrier sequence (interval i = between
// block barriers i and i+1; group 0 reads tile k in interval 2k, group 1 in 2k+1):
//   prologue      : issue tiles 0..S-2, vmcnt until tile 0 landed, barrier 0
//   interval 2k   : issue tile k+S-1 into buffer (k-1)%S  (WAR: its last reader,
//                   group 1's read of tile k-1, drained lgkmcnt before barrier 2k)
//   interval 2k+1 : vmcnt until tile k+1 landed (RAW: group 0 reads it after
//                   barrier 2k+2, group 1 after 2k+3)
//   one extra barrier at the end (group 0 has one after its loop), then the
//   loader waves end: s_barrier waits only for the waves that have not ended,
//   so the math waves' epilogue barriers are theirs alone.
// Registers: 8 + NL waves per block -> with NL = 4, three waves per SIMD, so the
// kernel is compiled for <= 168 VGPRs (__launch_bounds__ second argument = waves per EU).
#pragma once

namespace rdb {

template <typename T, typename OutT, int BM, int BN, int GM, int GN, int STAGES, bool HAS_BIAS, int NL, int BK_ = 64,
          int OCC = 3>
__global__ void __launch_bounds__(64 * (8 + NL), OCC)
gemm_ppl_kernel(const T* __restrict__ A, int lda, const T* __restrict__ W, int ldw, OutT* __restrict__ C, int ldc,
                const T* __restrict__ bias, int M, int N, int K, float alpha, int act) {
  constexpr int NW = 8;
  typedef PPGeom<NW, BM, BN, BK_> G;
  constexpr int BK = G::BK;
  constexpr int KS = BK / 32;
  constexpr int GW = NW / 2;
  static_assert(GM * GN == GW, "group wave layout");
  constexpr int GBM = BM / 2;
  constexpr int WM = GBM / GM, WN = BN / GN;
  constexpr int TM = WM / 16, TN = WN / 16;
  // loader pieces: A pieces 0..A_PIECES-1 then W pieces; every loader wave issues LPW (surplus -> dummy slot)
  constexpr int PIECES = G::A_PIECES + G::W_PIECES;
  constexpr int LPW = (PIECES + NL - 1) / NL;
  static_assert(STAGES >= 3 && (STAGES - 2) * LPW < 64, "pipeline depth / vmcnt field");
  constexpr int STAGE_BYTES = G::W_OFF + (PIECES - G::A_PIECES + (LPW * NL != PIECES ? 1 : 0)) * 1024;
  constexpr int DUMMY_OFF = G::W_OFF + G::W_PIECES * 1024;
  typedef typename MfmaOp<T>::frag frag;
  constexpr int BIAS_OFF = STAGES * STAGE_BYTES;
  __shared__ __attribute__((aligned(16))) char smem[BIAS_OFF + (HAS_BIAS ? BN * 4 : 0)];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int tiles_n = (N + BN - 1) / BN, tiles_m = (M + BM - 1) / BM;
  const int t = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  int tile_m, tile_n;
  if (tiles_n >= 12 && tiles_m >= 8) {
    const int gsize = 4 * tiles_n;
    const int g = t / gsize, first = 4 * g;
    const int gm = tiles_m - first < 4 ? tiles_m - first : 4;
    const int r = t - g * gsize;
    tile_m = first + r % gm;
    tile_n = r / gm;
  } else {
    tile_m = t / tiles_n;
    tile_n = t - tile_m * tiles_n;
  }
  const int m0 = tile_m * BM, n0 = tile_n * BN;
  int nk = (K + BK - 1) / BK;

  auto barrier = [] {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };
  constexpr int kLgkm0 = 0xC07F;

  if (wid >= NW) {
    // ===================== loader wave =====================
    const int lw = __builtin_amdgcn_readfirstlane(wid - NW);
    const __amdgpu_buffer_rsrc_t asrc =
        make_rsrc(A, (uint32_t)((size_t)(M - 1) * lda * sizeof(T) + (size_t)K * sizeof(T)));
    const __amdgpu_buffer_rsrc_t wsrc = make_rsrc(W, (uint32_t)((size_t)(N - 1) * ldw * sizeof(T) + (size_t)K * sizeof(T)));
    uint32_t off[LPW];
    int ch[LPW];
#pragma unroll
    for (int i = 0; i < LPW; ++i) {
      const int p = lw * LPW + i;
      if (p < G::A_PIECES) {
        const int row = p * G::PR + lane / G::CPR;
        ch[i] = (lane % G::CPR) ^ G::swz(row);
        const int gm = m0 + row;
        off[i] = gm < M ? (uint32_t)((size_t)gm * lda * sizeof(T)) : kOOB;
      } else {
        const int q = p - G::A_PIECES;
        const int row = q * G::PR + lane / G::CPR;
        ch[i] = (lane % G::CPR) ^ G::swz(row);
        const int gn = n0 + row;
        off[i] = (q < G::W_PIECES && row < BN && gn < N) ? (uint32_t)((size_t)gn * ldw * sizeof(T)) : kOOB;
      }
    }
    auto stage = [&](int buf, int k0) {
      char* base = smem + buf * STAGE_BYTES;
#pragma unroll
      for (int i = 0; i < LPW; ++i) {
        const int p = lw * LPW + i;
        const int gk = k0 + ch[i] * 8;
        const uint32_t src = (gk < K && off[i] != kOOB) ? off[i] + (uint32_t)(gk * sizeof(T)) : kOOB;
        char* dst = p < G::A_PIECES ? base + p * 1024
                                    : base + (p - G::A_PIECES < G::W_PIECES ? G::W_OFF + (p - G::A_PIECES) * 1024
                                                                             : DUMMY_OFF);
        dma16(p < G::A_PIECES ? asrc : wsrc, dst, src);
      }
    };
    constexpr int kVmPro = (((STAGES - 2) * LPW) & 15) | ((((STAGES - 2) * LPW) >> 4) << 14) | 0x70 | 0xF00;
    constexpr int kVm0 = 0x70 | 0xF00;
#pragma unroll
    for (int s = 0; s < STAGES - 1; ++s)
      if (s < nk) stage(s, s * BK);
    if (nk >= STAGES - 1) __builtin_amdgcn_s_waitcnt(kVmPro);
    else __builtin_amdgcn_s_waitcnt(kVm0);
    barrier();                                           // barrier 0
    for (int kt = 0; kt < nk; ++kt) {
      const bool steady = kt + STAGES - 1 < nk;
      if (steady) stage((kt + STAGES - 1) % STAGES, (kt + STAGES - 1) * BK);   // interval 2k
      barrier();                                         // barrier 2k+1
      if (steady) __builtin_amdgcn_s_waitcnt(kVmPro);    // tile k+1 landed (S-2 tiles may stay in flight)
      else __builtin_amdgcn_s_waitcnt(kVm0);
      barrier();                                         // barrier 2k+2
    }
    barrier();                                           // group 0's extra barrier
    // the math waves' 16-bit staged epilogue runs 2 block barriers per row chunk:
    // take part in them (no reliance on ended waves leaving the barrier count)
    typedef StagedEpi16<BM, BN, STAGES * STAGE_BYTES> E16;
#pragma unroll 1
    for (int c = 0; c < BM / E16::RC; ++c) {
      __syncthreads();
      __syncthreads();
    }
    return;
  }
  static_assert(sizeof(OutT) == 2, "lab kernel: 16-bit staged epilogue only (its barrier count is mirrored above)");

  // ===================== math waves (gemm_pp.h, no DMA) =====================
  const int grp = wid / GW, gw = wid % GW;
  const int wm = gw / GN, wn = gw % GN;
  f32x4 acc[TN][TM];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int fr = lane & 15, fg = lane >> 4;
  const int arow0 = grp * GBM + wm * WM + fr;
  const int wrow0 = wn * WN + fr;
  frag af[KS][TM], wf[KS][TN];
  auto read_tile = [&](int buf) {
    const char* sa = smem + buf * STAGE_BYTES;
    const char* sw = sa + G::W_OFF;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int chunk = ks * 4 + fg;
#pragma unroll
      for (int i = 0; i < TN; ++i) wf[ks][i] = *reinterpret_cast<const frag*>(sw + G::off(wrow0 + i * 16, chunk));
#pragma unroll
      for (int j = 0; j < TM; ++j) af[ks][j] = *reinterpret_cast<const frag*>(sa + G::off(arow0 + j * 16, chunk));
    }
  };
  if constexpr (HAS_BIAS) {
    for (int q = tid; q < BN / 4; q += G::NT) {
      const __amdgpu_buffer_rsrc_t bsrc = make_rsrc(bias, (uint32_t)(N * sizeof(T)));
      const u32x2 raw = bload8(bsrc, (uint32_t)((n0 + q * 4 < N ? n0 + q * 4 : N) * sizeof(T)));
      const T* e = reinterpret_cast<const T*>(&raw);
      *reinterpret_cast<f32x4*>(smem + BIAS_OFF + q * 16) = f32x4{(float)e[0], (float)e[1], (float)e[2], (float)e[3]};
    }
    __builtin_amdgcn_s_waitcnt(0x70 | 0xF00);            // my bias loads done (no DMA on this wave)
  }
  barrier();                                             // barrier 0 (tile 0 landed)
  if (grp == 1) barrier();
  int buf = 0;
  for (int kt = 0; kt < nk; ++kt) {
    read_tile(buf);
    __builtin_amdgcn_s_waitcnt(kLgkm0);
    barrier();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int j = 0; j < TM; ++j) acc[i][j] = MfmaOp<T>::mma(wf[ks][i], af[ks][j], acc[i][j]);
    __builtin_amdgcn_s_setprio(0);
    barrier();
    buf = buf == STAGES - 1 ? 0 : buf + 1;
  }
  if (grp == 0) barrier();
  constexpr int SB = STAGES * STAGE_BYTES;
  auto go = [&](auto actf) {
    staged_epilogue<T, OutT, BM, BN, SB, G::NT, TM, TN, HAS_BIAS, false, decltype(actf), BIAS_OFF, 0, -1>(
        smem, acc, grp * GBM + wm * WM, wn * WN, m0, n0, M, N, C, ldc, bias, nullptr, 0, alpha, actf, nullptr, tile_n);
  };
  if (act == ACT_GELU) go([](float x) { return apply_act<ACT_GELU>(x); });
  else go([](float x) { return x; });
}

template <typename T, typename OutT, int BM, int BN, int GM, int GN, int STAGES, int NL, int BK = 64, int OCC = 3>
void launch_gemm_ppl(const T* A, int lda, const T* W, int ldw, OutT* C, int ldc, const T* bias, int M, int N, int K,
                     float alpha, int act, hipStream_t s) {
  const int nwg = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  if (bias)
    hipLaunchKernelGGL((gemm_ppl_kernel<T, OutT, BM, BN, GM, GN, STAGES, true, NL, BK, OCC>), dim3(nwg),
                       dim3(64 * (8 + NL)), 0, s, A, lda, W, ldw, C, ldc, bias, M, N, K, alpha, act);
  else
    hipLaunchKernelGGL((gemm_ppl_kernel<T, OutT, BM, BN, GM, GN, STAGES, false, NL, BK, OCC>), dim3(nwg),
                       dim3(64 * (8 + NL)), 0, s, A, lda, W, ldw, C, ldc, bias, M, N, K, alpha, act);
}

}  // namespace rdb
