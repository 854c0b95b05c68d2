// Lab kernel: 4-wave, one-block-per-CU MFMA GEMM whose operands are staged
// global -> VGPR -> LDS (buffer_load_dwordx4 + ds_write_b128) instead of
// LDS-DMA, the way the vendor library's fastest gfx950 kernels do it
// (profiles/gemm_side_by_side_r5.json: 4-wave 256x256 stream-K tiles, 1,547
// TFLOP/s at 4096^3).  Why this staging: an LDS-DMA issue holds the issuing
// wave for ~60-180 cycles, which a lone wave per SIMD cannot hide (the 4-wave
// LDS-DMA kernel gemm_w4.h reached 1,053 TFLOP/s, profiles/gemm_lab_r5_w4.txt),
// while a vector load / ds_write issues in a few cycles and can be spread
// between the MFMAs.
//
//   C[m, n] = act(alpha * sum_k A[m, k] * W[n, k] + bias[n] + R[m, n])
//
// * 2 x 2 waves, per-wave WM x WN = BM/2 x BN/2 (128 x 128 at 256 x 256: 4
//   MFMAs per 16-B fragment read), accumulators in the whole register file
//   (__launch_bounds__(256, 1));
// * BK = 64, two LDS buffers, ONE block barrier per K-tile; the loads of tile
//   k+2 and the LDS writes of tile k+1 run under the MFMAs of tile k, and the
//   fragments of the next 32-deep half-step are read under the current one's
//   MFMAs (two fragment register sets);
// * LDS image = gemm_pp.h's (128-B rows, chunk ^ ((row >> 1) & 7) swizzle);
//   rows past M / N read as zero through the buffer resource's extent;
//   host-checked: K % 64 == 0;
// * the LDS-staged, row-coalesced fused epilogue of gemm_core.h.
#pragma once

namespace rdb {

template <typename T, typename OutT, int BM, int BN, bool HAS_BIAS, bool HAS_RES, bool ASM = false>
__global__ void __launch_bounds__(256, 1)
gemm_v4a_kernel(const T* __restrict__ A, int lda, const T* __restrict__ W, int ldw, OutT* __restrict__ C, int ldc,
               const T* __restrict__ bias, const T* __restrict__ R, int ldr, int M, int N, int K, float alpha,
               int act) {
  constexpr int NT = 256, BK = 64, ROWB = 128;
  constexpr int WM = BM / 2, WN = BN / 2;
  constexpr int TM = WM / 16, TN = WN / 16;
  static_assert(WM % 16 == 0 && WN % 16 == 0, "wave tile must be whole 16x16 fragments");
  constexpr int LA = BM * 8 / NT, LW = BN * 8 / NT;      // 16-B chunks per thread per tile
  static_assert((BM * 8) % NT == 0 && (BN * 8) % NT == 0, "tile rows must split over the 256 threads");
  constexpr int A_BYTES = BM * ROWB, STAGE = (BM + BN) * ROWB;
  constexpr int SB = 2 * STAGE;
  static_assert(SB + (HAS_BIAS ? BN * 4 : 0) <= 160 * 1024, "LDS");
  constexpr int BIAS_OFF = SB;
  typedef typename MfmaOp<T>::frag frag;
  __shared__ __attribute__((aligned(16))) char smem[SB + (HAS_BIAS ? BN * 4 : 0)];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  const int tiles_n = (N + BN - 1) / BN, tiles_m = (M + BM - 1) / BM;
  const int t = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int tile_m = t / tiles_n, tile_n = t - tile_m * tiles_n;
  const int m0 = tile_m * BM, n0 = tile_n * BN;

  const __amdgpu_buffer_rsrc_t asrc = make_rsrc(A, (uint32_t)((size_t)(M - 1) * lda * sizeof(T) + (size_t)K * sizeof(T)));
  const __amdgpu_buffer_rsrc_t wsrc = make_rsrc(W, (uint32_t)((size_t)(N - 1) * ldw * sizeof(T) + (size_t)K * sizeof(T)));
  // this thread's chunks: chunk c of rows r0 + 32 i (rows past M / N fall beyond the extent -> 0)
  const int c = tid & 7, r0 = tid >> 3;
  const uint32_t a_vo = (uint32_t)((m0 + r0) * lda * (int)sizeof(T) + c * 16);
  const uint32_t w_vo = (uint32_t)((n0 + r0) * ldw * (int)sizeof(T) + c * 16);
  const int a_step = 32 * lda * (int)sizeof(T), w_step = 32 * ldw * (int)sizeof(T);
  // LDS: row r0 + 32 i, chunk c -> (r0 + 32 i) * 128 + ((c ^ ((r0 >> 1) & 7)) << 4)  (the swizzle of r0 + 32 i is r0's)
  const int lds_w = r0 * ROWB + ((c ^ ((r0 >> 1) & 7)) << 4);
  u32x4 ra[LA], rw[LW];
  auto load_tile = [&](int k0) {
#pragma unroll
    for (int i = 0; i < LA; ++i)
      ra[i] = __builtin_amdgcn_raw_buffer_load_b128(asrc, a_vo + (uint32_t)(k0 * (int)sizeof(T)), i * a_step, 0);
#pragma unroll
    for (int i = 0; i < LW; ++i)
      rw[i] = __builtin_amdgcn_raw_buffer_load_b128(wsrc, w_vo + (uint32_t)(k0 * (int)sizeof(T)), i * w_step, 0);
  };
  auto store_tile = [&](int buf) {
    char* base = smem + buf * STAGE + lds_w;
#pragma unroll
    for (int i = 0; i < LA; ++i) *reinterpret_cast<u32x4*>(base + i * 32 * ROWB) = ra[i];
#pragma unroll
    for (int i = 0; i < LW; ++i) *reinterpret_cast<u32x4*>(base + A_BYTES + i * 32 * ROWB) = rw[i];
  };

  f32x4 acc[TN][TM];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int fr = lane & 15, fg = lane >> 4;
  const int arow0 = wm * WM + fr, wrow0 = wn * WN + fr;
  auto off = [](int row, int chunk) { return row * ROWB + ((chunk ^ ((row >> 1) & 7)) << 4); };
  frag fa[2][TM], fw[2][TN];
  auto read_half = [&](int set, int buf, int ks) {
    const char* sa = smem + buf * STAGE;
    const char* sw = sa + A_BYTES;
    const int chunk = ks * 4 + fg;
#pragma unroll
    for (int i = 0; i < TN; ++i) fw[set][i] = *reinterpret_cast<const frag*>(sw + off(wrow0 + i * 16, chunk));
#pragma unroll
    for (int j = 0; j < TM; ++j) fa[set][j] = *reinterpret_cast<const frag*>(sa + off(arow0 + j * 16, chunk));
  };
  auto mfma_half = [&](int set) {
#pragma unroll
    for (int i = 0; i < TN; ++i)
#pragma unroll
      for (int j = 0; j < TM; ++j) {
        if constexpr (ASM) {
          // accumulators pinned in AGPRs, updated in place (srcC == vdst)
          asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[i][j]) : "v"(fw[set][i]), "v"(fa[set][j]));
        } else {
          acc[i][j] = MfmaOp<T>::mma(fw[set][i], fa[set][j], acc[i][j]);
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
  constexpr int kLgkm0 = 0xC07F;        // lgkmcnt(0), vmcnt / expcnt at max

  if constexpr (HAS_BIAS) {
    for (int q = tid; q < BN / 4; q += NT) {
      const __amdgpu_buffer_rsrc_t bsrc = make_rsrc(bias, (uint32_t)(N * sizeof(T)));
      const u32x2 raw = bload8(bsrc, (uint32_t)((n0 + q * 4 < N ? n0 + q * 4 : N) * sizeof(T)));
      const T* e = reinterpret_cast<const T*>(&raw);
      *reinterpret_cast<f32x4*>(smem + BIAS_OFF + q * 16) = f32x4{(float)e[0], (float)e[1], (float)e[2], (float)e[3]};
    }
  }
  const int nk = K / BK;
  // prologue: tile 0 -> LDS buffer 0, tile 1 in flight into the staging registers
  load_tile(0);
  store_tile(0);
  if (nk > 1) load_tile(BK);
  __builtin_amdgcn_s_waitcnt(kLgkm0);
  barrier();
  read_half(0, 0, 0);

  // one K-tile: half 0 = (LDS writes of tile kt+1, loads of tile kt+2, reads of
  // half 1) under the MFMAs of half 0; a barrier; half 1 = reads of tile kt+1's
  // half 0 under the MFMAs of half 1
  auto step = [&](int kt, auto store_next, auto load_next) {
    const int buf = kt & 1;
    if constexpr (decltype(store_next)::value) store_tile(buf ^ 1);
    if constexpr (decltype(load_next)::value) load_tile((kt + 2) * BK);
    read_half(1, buf, 1);
    mfma_half(0);
    // interleave: per MFMA of half 0, one of the memory instructions issued above
#pragma unroll
    for (int q = 0; q < TM * TN; ++q) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                   // 1 MFMA
      __builtin_amdgcn_sched_group_barrier(0x200 | 0x020 | 0x100, 1, 0);   // 1 DS write / VMEM read / DS read
    }
    __builtin_amdgcn_s_waitcnt(kLgkm0);   // my half-1 reads of `buf` and my LDS writes of tile kt+1 are done
    barrier();
    if constexpr (decltype(store_next)::value) read_half(0, buf ^ 1, 0);
    mfma_half(1);
#pragma unroll
    for (int q = 0; q < TM * TN; ++q) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }
  };
  typedef std::integral_constant<bool, true> Y;
  typedef std::integral_constant<bool, false> Nn;
  int kt = 0;
  for (; kt + 2 < nk; ++kt) step(kt, Y{}, Y{});
  if (kt + 1 < nk) step(kt++, Y{}, Nn{});
  step(kt, Nn{}, Nn{});
  if constexpr (ASM) {
    // the compiler cannot see the inline-asm MFMAs' latency: let the last ones retire
    // before their accumulators are read
    asm volatile("s_nop 7");
    asm volatile("s_nop 7");
    asm volatile("s_nop 7");
    asm volatile("s_nop 7");
  }
  __syncthreads();   // every wave past its last fragment read: the LDS is free for the epilogue

  static_assert(sizeof(OutT) == 2, "gemm_v4 stores 16-bit outputs");
  auto go = [&](auto actf) {
    staged_epilogue<T, OutT, BM, BN, SB, NT, TM, TN, HAS_BIAS, HAS_RES, decltype(actf), BIAS_OFF>(
        smem, acc, wm * WM, wn * WN, m0, n0, M, N, C, ldc, bias, R, ldr, alpha, actf);
  };
  switch (act) {
    case ACT_GELU: go([](float x) { return apply_act<ACT_GELU>(x); }); break;
    case ACT_RELU: go([](float x) { return apply_act<ACT_RELU>(x); }); break;
    default: go([](float x) { return x; }); break;
  }
}

template <typename T, typename OutT, int BM, int BN, bool ASM = false>
void launch_gemm_v4a(const T* A, int lda, const T* W, int ldw, OutT* C, int ldc, const T* bias, const T* R, int ldr,
                    int M, int N, int K, float alpha, int act, hipStream_t s) {
  if (K % 64) throw std::invalid_argument("gemm_v4: K must be a multiple of 64");
  const int nwg = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  const dim3 grid(nwg), block(256);
  if (bias && R)
    hipLaunchKernelGGL((gemm_v4a_kernel<T, OutT, BM, BN, true, true, ASM>), grid, block, 0, s, A, lda, W, ldw, C, ldc, bias,
                       R, ldr, M, N, K, alpha, act);
  else if (bias)
    hipLaunchKernelGGL((gemm_v4a_kernel<T, OutT, BM, BN, true, false, ASM>), grid, block, 0, s, A, lda, W, ldw, C, ldc, bias,
                       R, ldr, M, N, K, alpha, act);
  else if (R)
    hipLaunchKernelGGL((gemm_v4a_kernel<T, OutT, BM, BN, false, true, ASM>), grid, block, 0, s, A, lda, W, ldw, C, ldc, bias,
                       R, ldr, M, N, K, alpha, act);
  else
    hipLaunchKernelGGL((gemm_v4a_kernel<T, OutT, BM, BN, false, false, ASM>), grid, block, 0, s, A, lda, W, ldw, C, ldc,
                       bias, R, ldr, M, N, K, alpha, act);
}

}  // namespace rdb
