// MFMA-shape lab (bench only): the ping-pong GEMM body of ops/csrc/gemm_pp.h
// with v_mfma_f32_32x32x16_bf16 fragments (32 x 32 output blocks, 16-deep
// k-steps) against the shipped v_mfma_f32_16x16x32_bf16 body, same tiles,
// same LDS-DMA pipeline, same swizzle, same staged epilogue (bias + act), on
// the BERT serving shapes; solo and two streams.
//
//   hipcc -O3 --offload-arch=gfx950 -I ray_dynamic_batching_amd/ops/csrc bench/gemm_lab/pp32_lab.hip -o labbin/pp32_lab
//
// 32 x 32 x 16 operand map (cdna_hip_programming.md §3): lane l (r = l & 31,
// h = l >> 5) holds A[row r][k = 8h + j] -- 16 contiguous bytes of a K-major
// LDS row, chunk 2 * ks + h of k-step ks -- and the accumulator, with W as the
// MFMA "A" operand, holds D[n][m]: m = l & 31, n = 8 g + 4 h + q in register
// 4 g + q.  So each 16-B fragment read serves 32 rows (vs 16), and a wave
// tile of WM x WN needs (WM + WN) / 32 reads per 16-deep step -- the same LDS
// bytes per FLOP as 16 x 16 x 32, half the MFMA instructions.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include "gemm_core.h"

using namespace rdb;

#define CK(x)                                                                                   \
  do {                                                                                          \
    hipError_t e_ = (x);                                                                        \
    if (e_ != hipSuccess) {                                                                     \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(1);                                                                                  \
    }                                                                                           \
  } while (0)

namespace rdb {

template <typename OutT, int NW, int BM, int BN, int GM, int GN, int STAGES, int BK_ = 64>
__global__ void __launch_bounds__(64 * NW, 2)
gemm_pp32_kernel(const bf16* __restrict__ A, int lda, const bf16* __restrict__ W, int ldw, OutT* __restrict__ C,
                 int ldc, const bf16* __restrict__ bias, int M, int N, int K, int act) {
  typedef PPGeom<NW, BM, BN, BK_> G;
  typedef bf16 T;
  constexpr int BK = G::BK;
  constexpr int KS = BK / 16;                // 16-deep MFMA k-steps per tile
  constexpr int GW = NW / 2;
  static_assert(GM * GN == GW, "group wave layout");
  constexpr int GBM = BM / 2;
  constexpr int WM = GBM / GM, WN = BN / GN;
  constexpr int TM = WM / 32, TN = WN / 32;
  static_assert(WM % 32 == 0 && WN % 32 == 0, "wave tile must be whole 32x32 blocks");
  constexpr int L = G::LOADS;
  static_assert(STAGES >= 3 && (STAGES - 2) * L < 64, "pipeline depth / vmcnt field");
  constexpr int BIAS_OFF = STAGES * G::STAGE_BYTES;
  __shared__ __attribute__((aligned(16))) char smem[BIAS_OFF + BN * 4];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int grp = wid / GW, gw = wid % GW;
  const int wm = gw / GN, wn = gw % GN;
  const int wid_u = __builtin_amdgcn_readfirstlane(wid);
  const int tiles_n = (N + BN - 1) / BN, tiles_m = (M + BM - 1) / BM;
  const int t = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int tile_m = t / tiles_n, tile_n = t - tile_m * tiles_n;
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
  auto wdst = [&](char* base, int i) -> char* {
    const int piece = wid_u * G::W_PW + i;
    return base + (piece < G::W_PIECES ? G::W_OFF + piece * 1024 : G::DUMMY_OFF);
  };
  auto stage = [&](int buf, int k0) {
    char* base = smem + buf * G::STAGE_BYTES;
#pragma unroll
    for (int i = 0; i < G::A_PW; ++i) {
      const int gk = k0 + ach[i] * 8;
      dma16(asrc, base + (wid_u * G::A_PW + i) * 1024, (gk < K && aoff[i] != kOOB) ? aoff[i] + (uint32_t)(gk * sizeof(T)) : kOOB);
    }
#pragma unroll
    for (int i = 0; i < G::W_PW; ++i) {
      const int gk = k0 + wch[i] * 8;
      dma16(wsrc, wdst(base, i), (gk < K && woff[i] != kOOB) ? woff[i] + (uint32_t)(gk * sizeof(T)) : kOOB);
    }
  };

  f32x16 acc[TN][TM];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  const int fr = lane & 31, fh = lane >> 5;
  const int arow0 = grp * GBM + wm * WM + fr;
  const int wrow0 = wn * WN + fr;
  bf16x8 af[KS][TM], wf[KS][TN];
  auto read_tile = [&](int buf) {
    const char* sa = smem + buf * G::STAGE_BYTES;
    const char* sw = sa + G::W_OFF;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int chunk = ks * 2 + fh;
#pragma unroll
      for (int i = 0; i < TN; ++i) wf[ks][i] = *reinterpret_cast<const bf16x8*>(sw + G::off(wrow0 + i * 32, chunk));
#pragma unroll
      for (int j = 0; j < TM; ++j) af[ks][j] = *reinterpret_cast<const bf16x8*>(sa + G::off(arow0 + j * 32, chunk));
    }
  };
  auto barrier = [] {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };
  constexpr int kVmSteady = (((STAGES - 2) * L) & 15) | ((((STAGES - 2) * L) >> 4) << 14) | 0x70 | 0xF00;
  constexpr int kVm0 = 0x70 | 0xF00;
  constexpr int kLgkm0 = 0xC07F;
  const int nk = (K + BK - 1) / BK;
  for (int q = tid; q < BN / 4; q += G::NT) {
    const __amdgpu_buffer_rsrc_t bsrc = make_rsrc(bias, (uint32_t)(N * sizeof(T)));
    const u32x2 raw = bload8(bsrc, (uint32_t)((n0 + q * 4 < N ? n0 + q * 4 : N) * sizeof(T)));
    const T* e = reinterpret_cast<const T*>(&raw);
    *reinterpret_cast<f32x4*>(smem + BIAS_OFF + q * 16) = f32x4{(float)e[0], (float)e[1], (float)e[2], (float)e[3]};
  }
#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s)
    if (s < nk) stage(s, s * BK);
  if (nk >= STAGES - 1) __builtin_amdgcn_s_waitcnt(kVmSteady);
  else __builtin_amdgcn_s_waitcnt(kVm0);
  barrier();
  if (grp == 1) barrier();
  int buf = 0;
  for (int kt = 0; kt < nk; ++kt) {
    read_tile(buf);
    const bool steady = kt + STAGES - 1 < nk;
    if (steady) stage((kt + STAGES - 1) % STAGES, (kt + STAGES - 1) * BK);
    __builtin_amdgcn_s_waitcnt(kLgkm0);
    if (steady) __builtin_amdgcn_s_waitcnt(kVmSteady);
    else __builtin_amdgcn_s_waitcnt(kVm0);
    barrier();
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int j = 0; j < TM; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(wf[ks][i], af[ks][j], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    barrier();
    buf = buf == STAGES - 1 ? 0 : buf + 1;
  }
  if (grp == 0) barrier();
  __syncthreads();

  // ---- staged 16-bit epilogue: bias + act on registers, rows parked in LDS, 16-B row stores ----
  typedef StagedEpi16<BM, BN, BIAS_OFF> E16;
  auto run = [&](auto actf) {
    u32x2 pk[TN][TM][4];
#pragma unroll
    for (int j = 0; j < TM; ++j)
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int nt = wn * WN + i * 32 + 8 * g + 4 * fh;
          f32x4 v = {acc[i][j][4 * g], acc[i][j][4 * g + 1], acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]};
          v += *reinterpret_cast<const f32x4*>(smem + BIAS_OFF + nt * 4);
          OutT o4[4] = {(OutT)actf(v[0]), (OutT)actf(v[1]), (OutT)actf(v[2]), (OutT)actf(v[3])};
          pk[i][j][g] = *reinterpret_cast<const u32x2*>(o4);
        }
    const int row_base = grp * GBM + wm * WM;
#pragma unroll 1
    for (int c = 0; c < BM / E16::RC; ++c) {
#pragma unroll
      for (int j = 0; j < TM; ++j) {
        const int rt = row_base + j * 32 + fr - c * E16::RC;
        if (rt >= 0 && rt < E16::RC) {
#pragma unroll
          for (int i = 0; i < TN; ++i)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
              const int nt = wn * WN + i * 32 + 8 * g + 4 * fh;
              *reinterpret_cast<u32x2*>(smem + rt * E16::ROWB + nt * 2) = pk[i][j][g];
            }
        }
      }
      __syncthreads();
#pragma unroll 4
      for (int idx = tid; idx < E16::RC * E16::NV; idx += G::NT) {
        const int r = idx / E16::NV, vcol = idx - r * E16::NV;
        const int m = m0 + c * E16::RC + r, n = n0 + vcol * 8;
        if (m < M && n < N)
          *reinterpret_cast<u32x4*>(C + (size_t)m * ldc + n) = *reinterpret_cast<const u32x4*>(smem + r * E16::ROWB + vcol * 16);
      }
      __syncthreads();
    }
  };
  if (act == ACT_GELU) run([](float x) { return apply_act<ACT_GELU>(x); });
  else run([](float x) { return x; });
}

}  // namespace rdb

__global__ void ref_gemm(const bf16* A, const bf16* W, const bf16* bias, float* C, int M, int N, int K, int act) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x, m = blockIdx.y;
  if (n >= N) return;
  float s = 0.f;
  for (int k = 0; k < K; ++k) s += (float)A[(size_t)m * K + k] * (float)W[(size_t)n * K + k];
  s += (float)bias[n];
  if (act == ACT_GELU) s = 0.5f * s * (1.f + erff(s * 0.70710678f));
  C[(size_t)m * N + n] = s;
}

__global__ void fill_rand(bf16* p, size_t n, uint32_t seed, float scale) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  for (; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t x = (uint32_t)i * 2654435761u ^ seed;
    x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
    p[i] = (bf16)(((float)(x & 0xFFFFFF) / 16777216.f * 2.f - 1.f) * scale);
  }
}

struct Shape { int M, N, K, act; const char* name; };
typedef std::function<void(const bf16*, const bf16*, const bf16*, bf16*, int, int, int, int, hipStream_t)> RunF;
struct Variant { std::string name; RunF run; };

template <int BM, int BN, int GM, int GN, int S, int BK>
Variant pp16(const char* nm) {
  return {nm, [](const bf16* A, const bf16* W, const bf16* b, bf16* C, int M, int N, int K, int act, hipStream_t s) {
            launch_gemm_pp<bf16, bf16, 8, BM, BN, GM, GN, S, BK, 2>(A, K, W, K, C, N, b, nullptr, 0, M, N, K, 1.f, act, s);
          }};
}
template <int BM, int BN, int GM, int GN, int S, int BK>
Variant pp32(const char* nm) {
  return {nm, [](const bf16* A, const bf16* W, const bf16* b, bf16* C, int M, int N, int K, int act, hipStream_t s) {
            const int nwg = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
            hipLaunchKernelGGL((gemm_pp32_kernel<bf16, 8, BM, BN, GM, GN, S, BK>), dim3(nwg), dim3(512), 0, s, A, K,
                               W, K, C, N, b, M, N, K, act);
          }};
}

int main(int argc, char** argv) {
  int iters = 50;
  for (int i = 1; i < argc; ++i)
    if (!strcmp(argv[i], "--iters")) iters = atoi(argv[++i]);
  std::vector<Shape> shapes = {{4096, 2304, 768, ACT_NONE, "bert.qkv"},
                               {4096, 768, 768, ACT_NONE, "bert.o"},
                               {4096, 3072, 768, ACT_GELU, "bert.ffn1+gelu"},
                               {4096, 768, 3072, ACT_NONE, "bert.ffn2"},
                               {4096, 4096, 4096, ACT_NONE, "sq4096"}};
  std::vector<Variant> vs = {
      pp16<256, 128, 2, 2, 3, 64>("mf16 pp 256x128 bk64 s3"),
      pp32<256, 128, 2, 2, 3, 64>("mf32 pp 256x128 bk64 s3"),
      pp16<256, 256, 2, 2, 4, 32>("mf16 pp 256x256 bk32 s4"),
      pp32<256, 256, 2, 2, 4, 32>("mf32 pp 256x256 bk32 s4"),
      pp32<256, 256, 1, 4, 4, 32>("mf32 pp 256x256 1x4 bk32 s4"),
      pp16<256, 192, 2, 2, 3, 32>("mf16 pp 256x192 bk32 s3"),
      pp32<256, 192, 2, 2, 3, 32>("mf32 pp 256x192 bk32 s3"),
  };
  const size_t maxA = 4096ull * 4096, maxW = 4096ull * 4096, maxC = 4096ull * 4096;
  bf16 *A, *W, *bias, *C, *C2;
  float* Cref;
  CK(hipMalloc(&A, maxA * 2));
  CK(hipMalloc(&W, maxW * 2));
  CK(hipMalloc(&bias, 4096 * 2));
  CK(hipMalloc(&C, maxC * 2));
  CK(hipMalloc(&C2, maxC * 2));
  CK(hipMalloc(&Cref, maxC * 4));
  fill_rand<<<1024, 256>>>(A, maxA, 1, 1.f);
  fill_rand<<<1024, 256>>>(W, maxW, 2, 0.05f);
  fill_rand<<<16, 256>>>(bias, 4096, 3, 1.f);
  hipStream_t s0, s1;
  CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  hipEvent_t e0, e1, e2;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventCreate(&e2));
  std::vector<uint16_t> hc(maxC);
  std::vector<float> hr(maxC);
  for (auto& sh : shapes) {
    const int M = sh.M, N = sh.N, K = sh.K;
    ref_gemm<<<dim3((N + 255) / 256, M), 256>>>(A, W, bias, Cref, M, N, K, sh.act);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(hr.data(), Cref, (size_t)M * N * 4, hipMemcpyDeviceToHost));
    const double flop = 2.0 * M * N * K;
    printf("== %s M=%d N=%d K=%d\n", sh.name, M, N, K);
    for (auto& v : vs) {
      CK(hipMemset(C, 0, (size_t)M * N * 2));
      CK(hipDeviceSynchronize());
      v.run(A, W, bias, C, M, N, K, sh.act, s0);
      CK(hipStreamSynchronize(s0));
      CK(hipGetLastError());
      CK(hipMemcpy(hc.data(), C, (size_t)M * N * 2, hipMemcpyDeviceToHost));
      double maxerr = 0;
      for (size_t i = 0; i < (size_t)M * N; ++i) {
        uint32_t u = (uint32_t)hc[i] << 16;
        float f;
        memcpy(&f, &u, 4);
        maxerr = std::max(maxerr, (double)fabsf(f - hr[i]) / (1.0 + fabsf(hr[i])));
      }
      for (int i = 0; i < 5; ++i) v.run(A, W, bias, C, M, N, K, sh.act, s0);
      float best = 1e30f;
      for (int rep = 0; rep < 3; ++rep) {   // interleaved repeats: min of 3
        CK(hipEventRecord(e0, s0));
        for (int i = 0; i < iters; ++i) v.run(A, W, bias, C, M, N, K, sh.act, s0);
        CK(hipEventRecord(e1, s0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        best = std::min(best, ms);
      }
      const double us = best * 1e3 / iters;
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0, s0));
      CK(hipStreamWaitEvent(s1, e0, 0));
      for (int i = 0; i < iters; ++i) {
        v.run(A, W, bias, C, M, N, K, sh.act, s0);
        v.run(A, W, bias, C2, M, N, K, sh.act, s1);
      }
      CK(hipEventRecord(e2, s1));
      CK(hipStreamWaitEvent(s0, e2, 0));
      CK(hipEventRecord(e1, s0));
      CK(hipEventSynchronize(e1));
      float ms2;
      CK(hipEventElapsedTime(&ms2, e0, e1));
      const double us2 = ms2 * 1e3 / iters / 2;
      printf("  %-30s %8.2f us %7.1f TF/s  err %.2e%s | 2-stream %8.2f us/gemm %7.1f TF/s\n", v.name.c_str(), us,
             flop / us * 1e-6, maxerr, maxerr > 2e-2 ? "  <-- WRONG" : "", us2, flop / us2 * 1e-6);
      fflush(stdout);
    }
  }
  return 0;
}
