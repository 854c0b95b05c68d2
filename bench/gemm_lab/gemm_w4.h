// Four-wave, one-block-per-CU MFMA GEMM with big per-wave tiles (gfx950).
//
//   C[m, n] = act(alpha * sum_k A[m, k] * W[n, k] + bias[n] + R[m, n])
//
// Why (profiles/gemm_side_by_side_r5.json): on MI355X the bf16 GEMM body is
// bounded by LDS traffic per MFMA, and that is set by the PER-WAVE output tile:
// a wave of a WM x WN tile reads (WM + WN) x BK x 2 B of fragments per K-step
// for WM x WN x BK x 2 FLOP.  The 8-wave ping-pong tiles give each wave 64 x 64
// (256 x 128) or 64 x 128 (256 x 256) -- 2 / 2.7 MFMAs per ds_read_b128 --
// while hipBLASLt's fastest kernels on the same shapes are 4-wave workgroups
// with 96 x 128 .. 128 x 128 per wave (MIWT6_8 / 8_8, 4 MFMAs per read): at
// 4096^3 1,547 TF/s against 1,323 for our best tile.  Here:
//
// * 4 waves (2 x 2), one workgroup per CU (__launch_bounds__(256, 1): the
//   whole 512-entry register file per lane; a 128 x 128 wave tile holds 256
//   accumulator registers, plus two fragment sets);
// * both operands by LDS-DMA (buffer_load ... lds, 16 B per lane, source-side
//   XOR swizzle, out-of-range -> 0; the PPGeom image of gemm_pp.h), STAGES LDS
//   buffers, counted vmcnt, ONE raw s_barrier per K-tile;
// * local-read prefetch: the fragments of half-step h+1 (or of the next
//   K-tile's first half) are read while the MFMAs of half-step h run, so a
//   lone wave per SIMD never waits out an LDS read with its matrix pipe idle;
// * the LDS-staged, row-coalesced fused epilogue of gemm_core.h.
//
// Pipeline per K-tile kt (S = STAGES; tile kt + S - 1 is in flight; the DMA
// pieces of tile kt + S are issued one by one BETWEEN the last half-step's MFMAs):
//   half 0 ..  KS-2 : read fragments of half h + 1 | MFMAs of half h
//   last half       : wait my DMA of tile kt + 1 (vmcnt), s_barrier (every
//                     wave is past its reads of buffer kt % S), issue tile
//                     kt + S into buffer kt % S, read tile kt + 1's first
//                     fragments | MFMAs of the last half of tile kt.
#pragma once
// Include after gemm_core.h (PPGeom, staged_epilogue, dma16, make_rsrc).

namespace rdb {

template <typename T, typename OutT, int BM, int BN, int STAGES, bool HAS_BIAS, bool HAS_RES, int BK_ = 64>
__global__ void __launch_bounds__(256, 1)
gemm_w4_kernel(const T* __restrict__ A, int lda, const T* __restrict__ W, int ldw, OutT* __restrict__ C, int ldc,
               const T* __restrict__ bias, const T* __restrict__ R, int ldr, int M, int N, int K, float alpha,
               int act) {
  constexpr int NW = 4;
  typedef PPGeom<NW, BM, BN, BK_> G;
  constexpr int BK = G::BK;
  constexpr int KS = BK / 32;                  // MFMA half-steps per K-tile
  constexpr int WM = BM / 2, WN = BN / 2;      // 2 x 2 waves
  constexpr int TM = WM / 16, TN = WN / 16;
  static_assert(WM % 16 == 0 && WN % 16 == 0, "wave tile must be whole 16x16 fragments");
  constexpr int L = G::LOADS;
  static_assert(STAGES >= 2 && (STAGES - 1) * L < 64, "pipeline depth / vmcnt field");
  static_assert(STAGES * G::STAGE_BYTES <= 160 * 1024, "LDS");
  typedef typename MfmaOp<T>::frag frag;
  constexpr int SB = STAGES * G::STAGE_BYTES;
  constexpr int BIAS_OFF = SB;                 // the tile's bias as f32, read by the epilogue
  __shared__ __attribute__((aligned(16))) char smem[SB + (HAS_BIAS ? BN * 4 : 0)];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int wid_u = __builtin_amdgcn_readfirstlane(wid);

  const int tiles_n = (N + BN - 1) / BN, tiles_m = (M + BM - 1) / BM;
  const int t = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int tile_m = t / tiles_n, tile_n = t - tile_m * tiles_n;
  const int m0 = tile_m * BM, n0 = tile_n * BN;

  const __amdgpu_buffer_rsrc_t asrc = make_rsrc(A, (uint32_t)((size_t)(M - 1) * lda * sizeof(T) + (size_t)K * sizeof(T)));
  const __amdgpu_buffer_rsrc_t wsrc = make_rsrc(W, (uint32_t)((size_t)(N - 1) * ldw * sizeof(T) + (size_t)K * sizeof(T)));
  // per DMA piece: the byte offset of this lane's 16-B chunk at k = 0 (rows
  // past M / N read as zero: kOOB stays beyond num_records for any k0 of a
  // < 2 GiB operand); the host guarantees K % BK == 0, so no K bound check
  uint32_t pbase[L];
#pragma unroll
  for (int i = 0; i < G::A_PW; ++i) {
    const int row = (wid * G::A_PW + i) * G::PR + lane / G::CPR;
    const int ch = (lane % G::CPR) ^ G::swz(row);
    const int gm = m0 + row;
    pbase[i] = gm < M ? (uint32_t)((size_t)gm * lda * sizeof(T) + ch * 16) : kOOB;
  }
#pragma unroll
  for (int i = 0; i < G::W_PW; ++i) {
    const int row = (wid * G::W_PW + i) * G::PR + lane / G::CPR;
    const int ch = (lane % G::CPR) ^ G::swz(row);
    const int gn = n0 + row;
    pbase[G::A_PW + i] = (row < BN && gn < N) ? (uint32_t)((size_t)gn * ldw * sizeof(T) + ch * 16) : kOOB;
  }
  // one DMA piece p (0 .. L-1: A pieces first, then W pieces) of the tile at k0 into buffer buf
  auto stage_piece = [&](int buf, int k0, int p) {
    char* base = smem + buf * G::STAGE_BYTES;
    const uint32_t off = pbase[p] + (uint32_t)(k0 * (int)sizeof(T));
    if (p < G::A_PW) {
      dma16(asrc, base + (wid_u * G::A_PW + p) * 1024, off);
    } else {
      const int piece = wid_u * G::W_PW + (p - G::A_PW);
      dma16(wsrc, base + (piece < G::W_PIECES ? G::W_OFF + piece * 1024 : G::DUMMY_OFF), off);
    }
  };
  auto stage = [&](int buf, int k0) {
#pragma unroll
    for (int p = 0; p < L; ++p) stage_piece(buf, k0, p);
  };

  f32x4 acc[TN][TM];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fg = lane >> 4;
  const int arow0 = wm * WM + fr, wrow0 = wn * WN + fr;
  frag fa[2][TM], fw[2][TN];    // two fragment sets: the one in the MFMAs, the one being read
  auto read_half = [&](int set, int buf, int ks) {
    const char* sa = smem + buf * G::STAGE_BYTES;
    const char* sw = sa + G::W_OFF;
    const int chunk = ks * 4 + fg;
#pragma unroll
    for (int i = 0; i < TN; ++i) fw[set][i] = *reinterpret_cast<const frag*>(sw + G::off(wrow0 + i * 16, chunk));
#pragma unroll
    for (int j = 0; j < TM; ++j) fa[set][j] = *reinterpret_cast<const frag*>(sa + G::off(arow0 + j * 16, chunk));
  };
  auto mfma_half = [&](int set) {
#pragma unroll
    for (int i = 0; i < TN; ++i)
#pragma unroll
      for (int j = 0; j < TM; ++j) acc[i][j] = MfmaOp<T>::mma(fw[set][i], fa[set][j], acc[i][j]);
  };
  // The last half-step of a K-tile: its MFMAs with the next tile's DMA pieces
  // spread between them (one piece per ~TM*TN/L MFMAs) -- an LDS-DMA issue costs
  // ~60-180 cycles of the issuing wave, so a burst of L of them in front of
  // the MFMAs would idle the matrix pipe of a one-wave-per-SIMD kernel
  constexpr int NMF = TM * TN;
  constexpr int PER = NMF / L > 0 ? NMF / L : 1;
  auto mfma_half_dma = [&](int set, bool issue, int sbuf, int sk0) {
#pragma unroll
    for (int i = 0; i < TN; ++i)
#pragma unroll
      for (int j = 0; j < TM; ++j) {
        acc[i][j] = MfmaOp<T>::mma(fw[set][i], fa[set][j], acc[i][j]);
        const int q = i * TM + j;
        if (q % PER == PER - 1 && q / PER < L) {
          if (issue) stage_piece(sbuf, sk0, q / PER);
          __builtin_amdgcn_sched_barrier(0);
        }
      }
  };
  auto barrier = [] {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };
  // s_waitcnt immediates (gfx9: vmcnt lo[3:0] hi[15:14], expcnt[6:4], lgkmcnt[11:8])
  constexpr int kVmS2 = (((STAGES - 2) * L) & 15) | ((((STAGES - 2) * L) >> 4) << 14) | 0x70 | 0xF00;
  constexpr int kVmS1 = (((STAGES - 1) * L) & 15) | ((((STAGES - 1) * L) >> 4) << 14) | 0x70 | 0xF00;
  constexpr int kVm0 = 0x70 | 0xF00;

  const int nk = (K + BK - 1) / BK;
  if constexpr (HAS_BIAS) {
    // bias -> LDS (f32) before the first DMA (an ordinary load behind an
    // in-flight LDS-DMA would make hipcc drain it); visible after the prologue barrier
    for (int q = tid; q < BN / 4; q += 256) {
      const __amdgpu_buffer_rsrc_t bsrc = make_rsrc(bias, (uint32_t)(N * sizeof(T)));
      const u32x2 raw = bload8(bsrc, (uint32_t)((n0 + q * 4 < N ? n0 + q * 4 : N) * sizeof(T)));
      const T* e = reinterpret_cast<const T*>(&raw);
      *reinterpret_cast<f32x4*>(smem + BIAS_OFF + q * 16) = f32x4{(float)e[0], (float)e[1], (float)e[2], (float)e[3]};
    }
  }
  // prologue: tiles 0 .. S-1 issued, tile 0 landed (loads retire in order)
#pragma unroll
  for (int s = 0; s < STAGES; ++s)
    if (s < nk) stage(s, s * BK);
  if (nk >= STAGES) __builtin_amdgcn_s_waitcnt(kVmS1);
  else __builtin_amdgcn_s_waitcnt(kVm0);
  barrier();
  read_half(0, 0, 0);
  static_assert(KS == 2, "the half-step schedule below is written for BK = 64 (two 32-deep MFMA steps)");
  int buf = 0;
  for (int kt = 0; kt < nk; ++kt) {
    // half 0: read half 1 (set 1) | MFMAs of half 0 (set 0)
    read_half(1, buf, 1);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
    mfma_half(0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    // half 1: tile kt + 1 made visible, its half 0 read (set 0), buffer `buf`
    // refilled with tile kt + S piece by piece | MFMAs of half 1 (set 1)
    const bool more = kt + 1 < nk;
    if (more) {
      if (kt + STAGES - 1 < nk) __builtin_amdgcn_s_waitcnt(kVmS2);   // my pieces of tile kt + 1 landed
      else __builtin_amdgcn_s_waitcnt(kVm0);
      __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): my reads of `buf` (set 1) are in
      barrier();                             // every wave's pieces visible; every wave done with `buf`
      read_half(0, buf == STAGES - 1 ? 0 : buf + 1, 0);
    }
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
    mfma_half_dma(1, more && kt + STAGES < nk, buf, (kt + STAGES) * BK);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    buf = buf == STAGES - 1 ? 0 : buf + 1;
  }
  __syncthreads();   // every wave is past its last read: the LDS is free for the epilogue

  static_assert(sizeof(OutT) == 2, "gemm_w4 stores 16-bit outputs");
  auto go = [&](auto actf) {
    staged_epilogue<T, OutT, BM, BN, SB, 256, TM, TN, HAS_BIAS, HAS_RES, decltype(actf), BIAS_OFF>(
        smem, acc, wm * WM, wn * WN, m0, n0, M, N, C, ldc, bias, R, ldr, alpha, actf);
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

template <typename T, typename OutT, int BM, int BN, int STAGES, int BK = 64>
void launch_gemm_w4(const T* A, int lda, const T* W, int ldw, OutT* C, int ldc, const T* bias, const T* R, int ldr,
                    int M, int N, int K, float alpha, int act, hipStream_t s) {
  if (K % BK) throw std::invalid_argument("gemm_w4: K must be a multiple of the K tile");
  const int nwg = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  const dim3 grid(nwg), block(256);
  if (bias && R)
    hipLaunchKernelGGL((gemm_w4_kernel<T, OutT, BM, BN, STAGES, true, true, BK>), grid, block, 0, s, A, lda, W, ldw, C,
                       ldc, bias, R, ldr, M, N, K, alpha, act);
  else if (bias)
    hipLaunchKernelGGL((gemm_w4_kernel<T, OutT, BM, BN, STAGES, true, false, BK>), grid, block, 0, s, A, lda, W, ldw, C,
                       ldc, bias, R, ldr, M, N, K, alpha, act);
  else if (R)
    hipLaunchKernelGGL((gemm_w4_kernel<T, OutT, BM, BN, STAGES, false, true, BK>), grid, block, 0, s, A, lda, W, ldw, C,
                       ldc, bias, R, ldr, M, N, K, alpha, act);
  else
    hipLaunchKernelGGL((gemm_w4_kernel<T, OutT, BM, BN, STAGES, false, false, BK>), grid, block, 0, s, A, lda, W, ldw,
                       C, ldc, bias, R, ldr, M, N, K, alpha, act);
}

}  // namespace rdb
