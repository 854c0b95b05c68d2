// Lab-only (bench/gemm_lab): the ping-pong GEMM of ops/csrc/gemm_pp.h with its
// steady-state operand staging moved from LDS-DMA to REGISTERS -- the read
// interval of tile kt issues plain buffer_load_dwordx4 for tile kt+2 into VGPRs
// and, one read interval later, ds_write_b128s them into the buffer of tile
// kt-2.  Why: the ping-pong read interval (16 ds_read_b128 + 6 LDS-DMA issues)
// measures ~2x its partner's MFMA interval, and an LDS-DMA issue holds its
// wave 100-185 cycles inside a read burst (MI355X_MICROARCH.md); a register
// load issues in a few cycles.  Dense operands, plain epilogues, 3 stages.
//
// Hazards (intervals numbered as in gemm_pp.h: group 0 reads tile kt in 2kt,
// group 1 in 2kt+1):
//   WAR: the writes of tile kt+1 (read interval kt, kt >= 1) go to the buffer of
//        tile kt-2, last read by group 1 in interval 2kt-3.
//   RAW: each wave's writes of tile kt+1 complete (lgkmcnt(0)) before the barrier
//        that ends its read interval kt; group 0 reads tile kt+1 in 2kt+2, after
//        group 1's writes (2kt+1).  Tiles 0 and 1 come from the prologue by
//        LDS-DMA, retired by the read interval of tile 0 (vmcnt).
#pragma once
#include "gemm_core.h"

namespace rdb {
namespace vs {

template <typename T, typename OutT, int NW, int BM, int BN, int GM, int GN, bool HAS_BIAS, bool HAS_RES, int BK_ = 64,
          int OCC = 2>
__global__ void __launch_bounds__(64 * NW, OCC)
ppvs_kernel(const T* __restrict__ A, int lda, const T* __restrict__ W, int ldw, OutT* __restrict__ C, int ldc,
            const T* __restrict__ bias, const T* __restrict__ R, int ldr, int M, int N, int K, float alpha, int act) {
  constexpr int STAGES = 3;
  typedef PPGeom<NW, BM, BN, BK_> G;
  constexpr int BK = G::BK;
  constexpr int KS = BK / 32;
  constexpr int GW = NW / 2;
  static_assert(GM * GN == GW, "group wave layout");
  constexpr int GBM = BM / 2;
  constexpr int WM = GBM / GM, WN = BN / GN;
  constexpr int TM = WM / 16, TN = WN / 16;
  constexpr int L = G::LOADS;
  typedef typename MfmaOp<T>::frag frag;
  constexpr int BIAS_OFF = STAGES * G::STAGE_BYTES;
  __shared__ __attribute__((aligned(16))) char smem[BIAS_OFF + (HAS_BIAS ? BN * 4 : 0)];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int grp = wid / GW, gw = wid % GW;
  const int wm = gw / GN, wn = gw % GN;
  const int wid_u = __builtin_amdgcn_readfirstlane(wid);
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

  const __amdgpu_buffer_rsrc_t asrc = make_rsrc(A, (uint32_t)((size_t)(M - 1) * lda * sizeof(T) + (size_t)K * sizeof(T)));
  const __amdgpu_buffer_rsrc_t wsrc = make_rsrc(W, (uint32_t)((size_t)(N - 1) * ldw * sizeof(T) + (size_t)K * sizeof(T)));
  uint32_t aoff[G::A_PW], woff[G::W_PW];
  int ach[G::A_PW], wch[G::W_PW];
#pragma unroll
  for (int i = 0; i < G::A_PW; ++i) {
    const int row = (wid * G::A_PW + i) * G::PR + lane / G::CPR;
    ach[i] = (lane % G::CPR) ^ G::swz(row);
    const int gm = m0 + row;
    aoff[i] = gm < M ? (uint32_t)((size_t)gm * lda * sizeof(T)) : kOOB;
  }
#pragma unroll
  for (int i = 0; i < G::W_PW; ++i) {
    const int row = (wid * G::W_PW + i) * G::PR + lane / G::CPR;
    wch[i] = (lane % G::CPR) ^ G::swz(row);
    const int gn = n0 + row;
    woff[i] = (row < BN && gn < N) ? (uint32_t)((size_t)gn * ldw * sizeof(T)) : kOOB;
  }
  auto a_src = [&](int i, int k0) -> uint32_t {
    const int gk = k0 + ach[i] * 8;
    return (gk < K && aoff[i] != kOOB) ? aoff[i] + (uint32_t)(gk * sizeof(T)) : kOOB;
  };
  auto w_src = [&](int i, int k0) -> uint32_t {
    const int gk = k0 + wch[i] * 8;
    return (gk < K && woff[i] != kOOB) ? woff[i] + (uint32_t)(gk * sizeof(T)) : kOOB;
  };
  auto a_dst = [&](char* base, int i) -> char* { return base + (wid_u * G::A_PW + i) * 1024; };
  auto w_dst = [&](char* base, int i) -> char* {
    const int piece = wid_u * G::W_PW + i;
    return base + (piece < G::W_PIECES ? G::W_OFF + piece * 1024 : G::DUMMY_OFF);
  };
  auto stage_dma = [&](int buf, int k0) {
    char* base = smem + buf * G::STAGE_BYTES;
#pragma unroll
    for (int i = 0; i < G::A_PW; ++i) dma16(asrc, a_dst(base, i), a_src(i, k0));
#pragma unroll
    for (int i = 0; i < G::W_PW; ++i) dma16(wsrc, w_dst(base, i), w_src(i, k0));
  };
  u32x4 stg[L];   // this wave's pieces of a tile, in flight between two read intervals
  auto load_regs = [&](int k0) {
#pragma unroll
    for (int i = 0; i < G::A_PW; ++i) stg[i] = __builtin_amdgcn_raw_buffer_load_b128(asrc, a_src(i, k0), 0, 0);
#pragma unroll
    for (int i = 0; i < G::W_PW; ++i) stg[G::A_PW + i] = __builtin_amdgcn_raw_buffer_load_b128(wsrc, w_src(i, k0), 0, 0);
  };
  auto write_regs = [&](int buf) {   // the DMA's layout: lane l's 16 B at piece + 16 l
    char* base = smem + buf * G::STAGE_BYTES;
#pragma unroll
    for (int i = 0; i < G::A_PW; ++i) *reinterpret_cast<u32x4*>(a_dst(base, i) + lane * 16) = stg[i];
#pragma unroll
    for (int i = 0; i < G::W_PW; ++i) *reinterpret_cast<u32x4*>(w_dst(base, i) + lane * 16) = stg[G::A_PW + i];
  };

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
    const char* sa = smem + buf * G::STAGE_BYTES;
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
  auto mfma_tile = [&]() {
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int j = 0; j < TM; ++j) acc[i][j] = MfmaOp<T>::mma(wf[ks][i], af[ks][j], acc[i][j]);
  };
  auto barrier = [] {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };
  constexpr int kVmL = (L & 15) | ((L >> 4) << 14) | 0x70 | 0xF00;
  constexpr int kVm0 = 0x70 | 0xF00;
  constexpr int kLgkm0 = 0xC07F;

  const int nk = (K + BK - 1) / BK;
  if constexpr (HAS_BIAS) {
    for (int q = tid; q < BN / 4; q += G::NT) {
      const __amdgpu_buffer_rsrc_t bsrc = make_rsrc(bias, (uint32_t)(N * sizeof(T)));
      const u32x2 raw = bload8(bsrc, (uint32_t)((n0 + q * 4 < N ? n0 + q * 4 : N) * sizeof(T)));
      const T* e = reinterpret_cast<const T*>(&raw);
      *reinterpret_cast<f32x4*>(smem + BIAS_OFF + q * 16) = f32x4{(float)e[0], (float)e[1], (float)e[2], (float)e[3]};
    }
  }
  // prologue: tiles 0 and 1 by LDS-DMA, tile 0 retired
  stage_dma(0, 0);
  if (nk > 1) stage_dma(1, BK);
  if (nk > 1) __builtin_amdgcn_s_waitcnt(kVmL);
  else __builtin_amdgcn_s_waitcnt(kVm0);
  barrier();
  if (grp == 1) barrier();

  int buf = 0;
  for (int kt = 0; kt < nk; ++kt) {
    // ---- read interval: stores of tile kt+1 (loaded one read interval ago), fragments of tile kt, loads of tile kt+2 ----
#ifndef LAB_VS_WRITE_LATE
    if (kt >= 1 && kt + 1 < nk) write_regs((kt + 1) % STAGES);
    read_tile(buf);
#else
    // stores after this interval's reads are issued: the loads get ~2 intervals to land
    read_tile(buf);
    if (kt >= 1 && kt + 1 < nk) write_regs((kt + 1) % STAGES);
#endif
    const bool more = kt + 2 < nk;
    if (more) load_regs((kt + 2) * BK);
    __builtin_amdgcn_s_waitcnt(kLgkm0);   // my reads and stores are done (WAR / RAW)
    if (kt == 0) {                        // the prologue's DMA of tile 1 landed
      if (more) __builtin_amdgcn_s_waitcnt(kVmL);
      else __builtin_amdgcn_s_waitcnt(kVm0);
    }
    barrier();
    __builtin_amdgcn_s_setprio(1);
    mfma_tile();
    __builtin_amdgcn_s_setprio(0);
    barrier();
    buf = buf == STAGES - 1 ? 0 : buf + 1;
  }
  if (grp == 0) barrier();

  static_assert(sizeof(OutT) == 2, "16-bit outputs");
  constexpr int SB = STAGES * G::STAGE_BYTES;
  const LnEpi ln{};
  auto go = [&](auto actf) {
    staged_epilogue<T, OutT, BM, BN, SB, G::NT, TM, TN, HAS_BIAS, HAS_RES, decltype(actf), BIAS_OFF, 0, -1>(
        smem, acc, grp * GBM + wm * WM, wn * WN, m0, n0, M, N, C, ldc, bias, R, ldr, alpha, actf, &ln, tile_n);
  };
  switch (act) {
    case ACT_GELU: go([](float x) { return apply_act<ACT_GELU>(x); }); break;
    default: go([](float x) { return x; }); break;
  }
}

template <typename T, typename OutT, int NW, int BM, int BN, int GM, int GN, int BK = 64, int OCC = 2>
void launch_ppvs(const T* A, int lda, const T* W, int ldw, OutT* C, int ldc, const T* bias, const T* R, int ldr, int M,
                 int N, int K, float alpha, int act, hipStream_t s) {
  const dim3 grid(((M + BM - 1) / BM) * ((N + BN - 1) / BN)), block(64 * NW);
  if (bias)
    hipLaunchKernelGGL((ppvs_kernel<T, OutT, NW, BM, BN, GM, GN, true, false, BK, OCC>), grid, block, 0, s, A, lda, W,
                       ldw, C, ldc, bias, R, ldr, M, N, K, alpha, act);
  else
    hipLaunchKernelGGL((ppvs_kernel<T, OutT, NW, BM, BN, GM, GN, false, false, BK, OCC>), grid, block, 0, s, A, lda, W,
                       ldw, C, ldc, bias, R, ldr, M, N, K, alpha, act);
}

}  // namespace vs
}  // namespace rdb
