// 256 x 256 "eight-phase" MFMA GEMM for gfx950 (cdna_hip_programming.md §5,
// "The 256² 8-phase template"): the serving GEMMs whose N fills 256-column
// tiles (BERT FFN-up N = 3072, Llama / ViT-G projections, large prefill).
//
//   C[m, n] = act(alpha * sum_k A[m, k] * W[n, k] + bias[n] + R[m, n])
//
// Geometry: 512 threads = 8 waves as 2 (M) x 4 (N); a wave owns 128 x 64 of
// the output (8 x 4 fragments of v_mfma_f32_16x16x32_bf16, 128 accumulator
// VGPRs).  BK = 64; a K-tile is staged as four 16-KiB half-tiles (A rows
// 0-127 / 128-255, W rows 0-127 / 128-255) by LDS-DMA (buffer_load ... lds,
// 16 B per lane, source-side XOR swizzle, out of range -> 0), two LDS buffers
// (128 KiB).  Each wave reads only its own A half (its 128 rows) and its W
// half (its 64 columns).
//
// Every K-tile runs as FOUR phases, one output quadrant (64 rows x 32 cols of
// the wave tile, 16 MFMAs) each, with the A / W register sub-tiles re-used
// across phases: reads per phase 12 / 4 / 8 / 0 ds_read_b128.  A phase is
//   R: fragment reads (+ DMA issue of the NEXT K-tile's half-tiles in phases
//      0 and 1, + vmcnt(0) in phase 3), lgkmcnt(0)   -- barrier --
//   M: setprio(1), 16 MFMAs, setprio(0)              -- barrier --
// and the two wave groups (M-halves) run ONE barrier apart (MI355X_MICROARCH.md
// "Two waves per SIMD"): each SIMD pairs one group's MFMA segment with the
// other group's read / DMA segment.
//
// Hazards (barriers numbered per block; group 1 is one behind group 0):
//  RAW: tile t+1 is issued in phases 4t, 4t+1 and retired by every wave's
//       vmcnt(0) in phase 4t+3, before the barrier that precedes the first
//       read of tile t+1 (group 0, phase 4t+4).
//  WAR: buffer (t+1)&1 was last read in phase 4(t-1)+2 by both groups, whose
//       lgkmcnt(0) precedes the barrier ending that read segment; the first
//       DMA into it is issued in phase 4t, at least one barrier later.
// Both groups execute the same number of s_barrier: group 1 one extra at the
// start, group 0 one extra at the end.
#pragma once
// Included by gemm_core.h (after the shared helpers and gemm_pp.h).

namespace rdb {

template <typename T, typename OutT, bool HAS_BIAS, bool HAS_RES>
__global__ void __launch_bounds__(512, 1)
gemm_8ph_kernel(const T* __restrict__ A, int lda, const T* __restrict__ W, int ldw, OutT* __restrict__ C, int ldc,
                const T* __restrict__ bias, const T* __restrict__ R, int ldr, int M, int N, int K, float alpha,
                int act) {
  constexpr int BM = 256, BN = 256, BK = 64, NT = 512;
  constexpr int HALF = 16384;                 // bytes per half-tile (128 rows x 128 B)
  constexpr int BUF = 4 * HALF;               // one K-tile
  constexpr int BIAS_OFF = 2 * BUF;
  constexpr int TM = 8, TN = 4;               // wave tile 128 x 64
  typedef typename MfmaOp<T>::frag frag;
  __shared__ __attribute__((aligned(16))) char smem[BIAS_OFF + (HAS_BIAS ? BN * 4 : 0)];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int grp = wid >> 2, wc = wid & 3;     // grp = wave row (M-half), wc = wave column
  const int wid_u = __builtin_amdgcn_readfirstlane(wid);

  const int tiles_n = (N + BN - 1) / BN, tiles_m = (M + BM - 1) / BM;
  const int t = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int tile_m = t / tiles_n, tile_n = t - tile_m * tiles_n;
  const int m0 = tile_m * BM, n0 = tile_n * BN;

  // ---- DMA addressing: wave w stages rows [16w, 16w+16) of every half-tile ----
  const __amdgpu_buffer_rsrc_t asrc = make_rsrc(A, (uint32_t)((size_t)(M - 1) * lda * sizeof(T) + (size_t)K * sizeof(T)));
  const __amdgpu_buffer_rsrc_t wsrc = make_rsrc(W, (uint32_t)((size_t)(N - 1) * ldw * sizeof(T) + (size_t)K * sizeof(T)));
  uint32_t aoff[2][2], woff[2][2];
  int ch[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int row = wid * 16 + j * 8 + (lane >> 3);       // row inside the half-tile
    ch[j] = (lane & 7) ^ ((row >> 1) & 7);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int gm = m0 + h * 128 + row, gn = n0 + h * 128 + row;
      aoff[h][j] = gm < M ? (uint32_t)((size_t)gm * lda * sizeof(T)) : kOOB;
      woff[h][j] = gn < N ? (uint32_t)((size_t)gn * ldw * sizeof(T)) : kOOB;
    }
  }
  // half h: 0 = A rows 0-127, 1 = A rows 128-255, 2 = W rows 0-127, 3 = W rows 128-255
  auto stage_half = [&](int buf, int h, int k0) {
    char* base = smem + buf * BUF + h * HALF + wid_u * 2048;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int gk = k0 + ch[j] * 8;
      const uint32_t ro = h < 2 ? aoff[h][j] : woff[h - 2][j];
      const uint32_t off = (gk < K && ro != kOOB) ? ro + (uint32_t)(gk * sizeof(T)) : kOOB;
      dma16(h < 2 ? asrc : wsrc, base + j * 1024, off);
    }
  };

  f32x4 acc[TN][TM];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fg = lane >> 4;
  frag af[2][4];        // [ks][row frag] of the current 64-row quadrant
  frag wf[2][2][2];     // [qn][ks][col frag]
  auto read_a = [&](const char* sa, int qm) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        af[ks][i] = *reinterpret_cast<const frag*>(sa + swz_off(qm * 64 + i * 16 + fr, ks * 4 + fg));
  };
  auto read_w = [&](const char* sw, int qn) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 2; ++i)
        wf[qn][ks][i] = *reinterpret_cast<const frag*>(sw + swz_off((wc & 1) * 64 + qn * 32 + i * 16 + fr, ks * 4 + fg));
  };
  auto mma = [&](int qm, int qn) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[qn * 2 + i][qm * 4 + j] = MfmaOp<T>::mma(wf[qn][ks][i], af[ks][j], acc[qn * 2 + i][qm * 4 + j]);
  };
  auto barrier = [] {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };
  constexpr int kVm0 = 0x70 | 0xF00;
  constexpr int kLgkm0 = 0xC07F;

  if constexpr (HAS_BIAS) {
    // bias -> LDS (f32) before the first DMA (an ordinary load's use would
    // otherwise drain the prologue DMA, guide §5 "Pipelining across barriers")
    for (int q = tid; q < BN / 4; q += NT) {
      const __amdgpu_buffer_rsrc_t bsrc = make_rsrc(bias, (uint32_t)(N * sizeof(T)));
      const u32x2 raw = bload8(bsrc, (uint32_t)((n0 + q * 4 < N ? n0 + q * 4 : N) * sizeof(T)));
      const T* e = reinterpret_cast<const T*>(&raw);
      *reinterpret_cast<f32x4*>(smem + BIAS_OFF + q * 16) = f32x4{(float)e[0], (float)e[1], (float)e[2], (float)e[3]};
    }
  }
  const int nk = (K + BK - 1) / BK;
  // prologue: tile 0 resident
#pragma unroll
  for (int h = 0; h < 4; ++h) stage_half(0, h, 0);
  __builtin_amdgcn_s_waitcnt(kVm0);
  barrier();
  if (grp == 1) barrier();   // stagger: group 1 one barrier behind

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const char* sa = smem + cur * BUF + grp * HALF;
    const char* sw = smem + cur * BUF + (2 + (wc >> 1)) * HALF;
    const bool more = kt + 1 < nk;
    // ---- phase 0: quadrant (0, 0) ----
    read_a(sa, 0);
    read_w(sw, 0);
    if (more) { stage_half(cur ^ 1, 0, (kt + 1) * BK); stage_half(cur ^ 1, 1, (kt + 1) * BK); }
    __builtin_amdgcn_s_waitcnt(kLgkm0);
    barrier();
    __builtin_amdgcn_s_setprio(1);
    mma(0, 0);
    __builtin_amdgcn_s_setprio(0);
    barrier();
    // ---- phase 1: quadrant (0, 1) ----
    read_w(sw, 1);
    if (more) { stage_half(cur ^ 1, 2, (kt + 1) * BK); stage_half(cur ^ 1, 3, (kt + 1) * BK); }
    __builtin_amdgcn_s_waitcnt(kLgkm0);
    barrier();
    __builtin_amdgcn_s_setprio(1);
    mma(0, 1);
    __builtin_amdgcn_s_setprio(0);
    barrier();
    // ---- phase 2: quadrant (1, 1) ----
    read_a(sa, 1);
    __builtin_amdgcn_s_waitcnt(kLgkm0);      // last read of buffer `cur` (WAR for tile kt+2)
    barrier();
    __builtin_amdgcn_s_setprio(1);
    mma(1, 1);
    __builtin_amdgcn_s_setprio(0);
    barrier();
    // ---- phase 3: quadrant (1, 0), registers only; retire tile kt+1 ----
    __builtin_amdgcn_s_waitcnt(kVm0);
    barrier();
    __builtin_amdgcn_s_setprio(1);
    mma(1, 0);
    __builtin_amdgcn_s_setprio(0);
    barrier();
  }
  if (grp == 0) barrier();
  __syncthreads();

  // ---- epilogue: LDS-staged, row-coalesced (16-bit output, N % 8 == 0, aligned) ----
  static_assert(sizeof(OutT) == 2, "8-phase GEMM stores 16-bit outputs");
  auto go = [&](auto actf) {
    staged_epilogue<T, OutT, BM, BN, 2 * BUF, NT, TM, TN, HAS_BIAS, HAS_RES, decltype(actf), BIAS_OFF>(
        smem, acc, grp * 128, wc * 64, m0, n0, M, N, C, ldc, bias, R, ldr, alpha, actf);
  };
  switch (act) {
    case ACT_GELU: go([](float x) { return apply_act<ACT_GELU>(x); }); break;
    case ACT_RELU: go([](float x) { return apply_act<ACT_RELU>(x); }); break;
    case ACT_TANH: go([](float x) { return apply_act<ACT_TANH>(x); }); break;
    case ACT_SILU: go([](float x) { return apply_act<ACT_SILU>(x); }); break;
    case ACT_GELU_TANH: go([](float x) { return apply_act<ACT_GELU_TANH>(x); }); break;
    case ACT_SIGMOID: go([](float x) { return apply_act<ACT_SIGMOID>(x); }); break;
    default: go([](float x) { return x; }); break;
  }
}

template <typename T, typename OutT>
void launch_gemm_8ph(const T* A, int lda, const T* W, int ldw, OutT* C, int ldc, const T* bias, const T* R, int ldr,
                     int M, int N, int K, float alpha, int act, hipStream_t s) {
  const int nwg = ((M + 255) / 256) * ((N + 255) / 256);
  const dim3 grid(nwg), block(512);
  if (bias && R)
    hipLaunchKernelGGL((gemm_8ph_kernel<T, OutT, true, true>), grid, block, 0, s, A, lda, W, ldw, C, ldc, bias, R, ldr,
                       M, N, K, alpha, act);
  else if (bias)
    hipLaunchKernelGGL((gemm_8ph_kernel<T, OutT, true, false>), grid, block, 0, s, A, lda, W, ldw, C, ldc, bias, R,
                       ldr, M, N, K, alpha, act);
  else if (R)
    hipLaunchKernelGGL((gemm_8ph_kernel<T, OutT, false, true>), grid, block, 0, s, A, lda, W, ldw, C, ldc, bias, R,
                       ldr, M, N, K, alpha, act);
  else
    hipLaunchKernelGGL((gemm_8ph_kernel<T, OutT, false, false>), grid, block, 0, s, A, lda, W, ldw, C, ldc, bias, R,
                       ldr, M, N, K, alpha, act);
}

}  // namespace rdb
