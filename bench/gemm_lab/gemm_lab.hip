// Standalone GEMM lab (bench only, not part of the library): times the
// ping-pong GEMM (ops/csrc/gemm_pp.h) against the production tile kernel
// (ops/csrc/gemm_core.h) on the serving shapes, and checks every result
// against a plain fp32 reference GEMM on the GPU.
//
//   hipcc -O3 --offload-arch=gfx950 -I ray_dynamic_batching_amd/ops/csrc bench/gemm_lab/gemm_lab.hip -o bench/gemm_lab/gemm_lab
//   ./bench/gemm_lab/gemm_lab [--iters 50] [--concurrent]
//
// --concurrent also times each kernel as TWO streams running the same GEMM
// side by side (the serving engine's 2-compute-stream regime).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <algorithm>
#include <functional>
#include <string>
#include <vector>

#include "gemm_core.h"
#include "gemm_8ph.h"   // lab-only 8-phase schedule (not in the library)

using namespace rdb;

#define CK(x)                                                                                   \
  do {                                                                                          \
    hipError_t e_ = (x);                                                                        \
    if (e_ != hipSuccess) {                                                                     \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(1);                                                                                  \
    }                                                                                           \
  } while (0)

__global__ void ref_gemm(const bf16* A, const bf16* W, const bf16* bias, float* C, int M, int N, int K) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x, m = blockIdx.y;
  if (n >= N) return;
  float s = 0.f;
  for (int k = 0; k < K; ++k) s += (float)A[(size_t)m * K + k] * (float)W[(size_t)n * K + k];
  C[(size_t)m * N + n] = s + (bias ? (float)bias[n] : 0.f);
}

__global__ void fill_rand(bf16* p, size_t n, uint32_t seed, float scale) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  for (; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t x = (uint32_t)i * 2654435761u ^ seed;
    x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
    p[i] = (bf16)(((float)(x & 0xFFFFFF) / 16777216.f * 2.f - 1.f) * scale);
  }
}

struct Shape { int M, N, K; const char* name; };
struct Variant { std::string name; std::function<void(const bf16*, const bf16*, const bf16*, bf16*, int, int, int, hipStream_t)> run; };

template <int NW, int BM, int BN, int GM, int GN, int S, int BK = 64, int OCC = 2, int ACT = ACT_NONE>
Variant pp(const char* nm) {
  return {nm, [](const bf16* A, const bf16* W, const bf16* b, bf16* C, int M, int N, int K, hipStream_t s) {
            launch_gemm_pp<bf16, bf16, NW, BM, BN, GM, GN, S, BK, OCC>(A, K, W, K, C, N, b, nullptr, 0, M, N, K, 1.f,
                                                                   ACT, s);
          }};
}
Variant e8(const char* nm) {
  return {nm, [](const bf16* A, const bf16* W, const bf16* b, bf16* C, int M, int N, int K, hipStream_t s) {
            launch_gemm_8ph<bf16, bf16>(A, K, W, K, C, N, b, nullptr, 0, M, N, K, 1.f, ACT_NONE, s);
          }};
}
// one production-kernel tile, instantiated alone (core() instantiates the whole tile table)
template <int BM, int BN, int WGM, int NW>
Variant core1(const char* nm) {
  return {nm, [](const bf16* A, const bf16* W, const bf16* b, bf16* C, int M, int N, int K, hipStream_t s) {
            DenseParams p{A, K, M, K};
            launch_one<bf16, bf16, DenseLoader, true, false, BM, BN, WGM, NW>(p, W, K, C, N, b, nullptr, 0, M, N, K,
                                                                               1.f, ACT_NONE, s);
          }};
}
// one production-kernel tile with DEEP (one block per CU, launch bounds for 512 VGPRs): the 4-wave
// 256x256 tile with 128x128 per wave halves the LDS bytes per MFMA of the 64x64-per-wave tiles
template <int BM, int BN, int WGM, int NW>
Variant core1d(const char* nm) {
  return {nm, [](const bf16* A, const bf16* W, const bf16* b, bf16* C, int M, int N, int K, hipStream_t s) {
            DenseParams p{A, K, M, K};
            launch_one<bf16, bf16, DenseLoader, true, false, BM, BN, WGM, NW, 0, 1>(p, W, K, C, N, b, nullptr, 0, M, N,
                                                                                    K, 1.f, ACT_NONE, s);
          }};
}
#if !defined(LAB_SET_GELU) && !defined(LAB_SET_FFN2) && !defined(LAB_FAST) && !defined(LAB_SET_BIG)   // the whole tile table: minutes of compile time
Variant core(int cfg) {
  char nm[64];
  snprintf(nm, sizeof nm, "core cfg%d %dx%d/%dw", cfg, kTileBM[cfg], kTileBN[cfg], 4 * kTileNW[cfg] / 4);
  return {nm, [cfg](const bf16* A, const bf16* W, const bf16* b, bf16* C, int M, int N, int K, hipStream_t s) {
            DenseParams p{A, K, M, K};
            launch_mfma_gemm<bf16, bf16, DenseLoader>(p, W, K, C, N, b, nullptr, 0, M, N, K, 1.f, ACT_NONE, s, cfg);
          }};
}
#endif

int main(int argc, char** argv) {
  int iters = 50;
  bool conc = false;
  std::string only;
  for (int i = 1; i < argc; ++i) {
    if (!strcmp(argv[i], "--iters")) iters = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--concurrent")) conc = true;
    else if (!strcmp(argv[i], "--only")) only = argv[++i];
  }
  std::vector<Shape> shapes = {{4096, 2304, 768, "bert.qkv"},
                               {4096, 768, 768, "bert.o"},
                               {4096, 3072, 768, "bert.ffn1"},
                               {4096, 768, 3072, "bert.ffn2"},
                               {4096, 4096, 4096, "sq4096"}};
  std::vector<Variant> vs = {
#if defined(LAB_SET_FFN2)
      // FFN-down (N = 768) on wider tiles: fewer L2 bytes per FLOP, fewer blocks
      pp<8, 256, 128, 2, 2, 3, 64>("pp8 256x128 bk64 s3"),
      pp<8, 256, 192, 2, 2, 4, 32>("pp8 256x192 2x2 bk32 s4"),
      pp<8, 256, 192, 1, 4, 4, 32>("pp8 256x192 1x4 bk32 s4"),
      pp<8, 256, 192, 2, 2, 3, 32>("pp8 256x192 2x2 bk32 s3"),
      pp<8, 256, 256, 2, 2, 4, 32>("pp8 256x256 bk32 s4"),
#elif defined(LAB_SET_GELU)
      // epilogue cost: the FFN-up tile with and without its GELU
      pp<8, 256, 256, 2, 2, 4, 32, 2, ACT_NONE>("pp8 256x256 bk32 s4 none"),
      pp<8, 256, 256, 2, 2, 4, 32, 2, ACT_GELU>("pp8 256x256 bk32 s4 gelu"),
      pp<8, 256, 256, 2, 2, 4, 32, 2, ACT_GELU_TANH>("pp8 256x256 bk32 s4 gelu_tanh"),
      pp<8, 256, 128, 2, 2, 3, 64, 2, ACT_NONE>("pp8 256x128 bk64 s3 none"),
      pp<8, 256, 128, 2, 2, 3, 64, 2, ACT_GELU>("pp8 256x128 bk64 s3 gelu"),
      // two co-resident blocks per CU: one block's GELU epilogue beside the other's MFMAs
      pp<8, 128, 256, 1, 4, 3, 32, 4, ACT_GELU>("pp8 128x256 bk32 s3 occ4 gelu"),
      pp<8, 256, 128, 2, 2, 3, 32, 4, ACT_GELU>("pp8 256x128 bk32 s3 occ4 gelu"),
      pp<8, 256, 256, 2, 2, 4, 32, 2, ACT_SILU>("pp8 256x256 bk32 s4 silu"),
#elif defined(LAB_SET_OCC)
      // occupancy: one 8-wave block per CU (OCC 2) vs two co-resident blocks (OCC 4, LDS <= 80 KiB)
      pp<8, 256, 128, 2, 2, 3, 64, 2>("pp8 256x128 bk64 s3"),
      pp<8, 256, 128, 2, 2, 3, 32, 4>("pp8 256x128 bk32 s3 occ4"),
      pp<8, 256, 128, 2, 2, 4, 32, 2>("pp8 256x128 bk32 s4"),
      pp<8, 128, 128, 2, 2, 4, 32, 4>("pp8 128x128 bk32 s4 occ4"),
      pp<8, 128, 256, 1, 4, 3, 32, 4>("pp8 128x256 bk32 s3 occ4"),
      pp<8, 256, 256, 2, 2, 4, 32, 2>("pp8 256x256 bk32 s4"),
      pp<4, 128, 128, 1, 2, 4, 32, 2>("pp4 128x128 bk32 s4"),
      pp<4, 128, 128, 1, 2, 3, 32, 3>("pp4 128x128 bk32 s3 occ3"),
      core(10), core(9),
#elif defined(LAB_SET_BIG)
      // per-wave tile size vs LDS bytes per MFMA (round 6): 128x128 per wave on 4 waves
      core1d<256, 256, 2, 4>("core 256x256 4w (128x128/wave) deep"),
      core1d<256, 128, 2, 4>("core 256x128 4w (128x64/wave) deep"),
      core1d<128, 256, 2, 4>("core 128x256 4w (64x128/wave) deep"),
      pp<8, 256, 128, 2, 2, 3>("pp8 256x128 2x2 s3"),
      pp<8, 256, 256, 2, 2, 4, 32>("pp8 256x256 bk32 s4"),
#elif defined(LAB_FAST)
      LAB_FAST
#else
      pp<8, 256, 128, 2, 2, 3>("pp8 256x128 2x2 s3"),
      pp<8, 128, 256, 1, 4, 3>("pp8 128x256 1x4 s3"),
      pp<8, 256, 144, 4, 1, 3>("pp8 256x144 4x1 s3"),
      pp<8, 128, 128, 2, 2, 3>("pp8 128x128 2x2 s3"),
      pp<8, 128, 96, 2, 2, 3>("pp8 128x96 2x2 s3"),
      pp<8, 256, 48, 4, 1, 3>("pp8 256x48 4x1 s3"),
      pp<8, 128, 192, 2, 2, 3>("pp8 128x192 2x2 s3"),
      pp<4, 128, 64, 1, 2, 3>("pp4 128x64 1x2 s3"),
      pp<4, 64, 128, 1, 2, 3>("pp4 64x128 1x2 s3"),
      core(8), core(12), core(9), core(17), core(15), core(13), core(0), core(4),
#endif
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
#ifdef RDB_PP_STAMPS
  // every pp launch writes its stamps: the buffer must exist before the first one
  constexpr int kStampBlocks = 65536;
  unsigned long long* stamp_buf = nullptr;
  CK(hipMalloc(&stamp_buf, kStampBlocks * 64));
  CK(hipMemcpyToSymbol(HIP_SYMBOL(rdb_pp_stamps), &stamp_buf, sizeof(stamp_buf)));
#endif
  hipStream_t s0, s1;
  CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<uint16_t> hc(maxC);
  std::vector<float> hr(maxC);
  for (auto& sh : shapes) {
    const int M = sh.M, N = sh.N, K = sh.K;
    ref_gemm<<<dim3((N + 255) / 256, M), 256>>>(A, W, bias, Cref, M, N, K);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(hr.data(), Cref, (size_t)M * N * 4, hipMemcpyDeviceToHost));
    const double flop = 2.0 * M * N * K;
    printf("== %s M=%d N=%d K=%d\n", sh.name, M, N, K);
    for (auto& v : vs) {
      if (!only.empty() && v.name.find(only) == std::string::npos) continue;
      CK(hipMemset(C, 0, (size_t)M * N * 2));
      CK(hipDeviceSynchronize());   // hipMemset runs on the null stream: order it before the s0 launch
      v.run(A, W, bias, C, M, N, K, s0);
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
      for (int i = 0; i < 5; ++i) v.run(A, W, bias, C, M, N, K, s0);
      CK(hipEventRecord(e0, s0));
      for (int i = 0; i < iters; ++i) v.run(A, W, bias, C, M, N, K, s0);
      CK(hipEventRecord(e1, s0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double us = ms * 1e3 / iters;
      printf("  %-26s %8.2f us %7.1f TF/s  err %.2e%s", v.name.c_str(), us, flop / us * 1e-6, maxerr,
             maxerr > 2e-2 ? "  <-- WRONG" : "");
#ifdef RDB_PP_STAMPS
      if (v.name.rfind("pp", 0) == 0) {
        const int nb = kStampBlocks;
        unsigned long long* dst = stamp_buf;
        CK(hipMemset(dst, 0, nb * 64));
        v.run(A, W, bias, C, M, N, K, s0);
        CK(hipStreamSynchronize(s0));
        std::vector<unsigned long long> h(nb * 8);
        CK(hipMemcpy(h.data(), dst, nb * 64, hipMemcpyDeviceToHost));
        std::vector<double> pro, loop, epi, start;
        unsigned long long t0 = ~0ull, t1 = 0, r0 = ~0ull, r1 = 0;
        for (int b = 0; b < nb; ++b) {
          unsigned long long* q = &h[b * 8];
          if (!q[0]) continue;
          pro.push_back((double)(q[1] - q[0]));
          loop.push_back((double)(q[2] - q[1]));
          epi.push_back((double)(q[3] - q[2]));
          start.push_back((double)q[0]);
          t0 = std::min(t0, q[0]);
          t1 = std::max(t1, q[3]);
          r1 = std::max(r1, q[5]);
        }
        auto med = [](std::vector<double> x) { std::sort(x.begin(), x.end()); return x[x.size() / 2]; };
        auto mx = [](std::vector<double> x) { return *std::max_element(x.begin(), x.end()); };
        for (auto& x : start) x -= (double)t0;
        printf("\n      stamps: %zu blocks, span %llu cyc | prologue med %.0f max %.0f | loop med %.0f max %.0f | "
               "epilogue med %.0f max %.0f | start skew max %.0f",
               pro.size(), t1 - t0, med(pro), mx(pro), med(loop), mx(loop), med(epi), mx(epi), mx(start));
      }
#endif
      if (conc) {
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0, s0));
        CK(hipStreamWaitEvent(s1, e0, 0));
        for (int i = 0; i < iters; ++i) {
          v.run(A, W, bias, C, M, N, K, s0);
          v.run(A, W, bias, C2, M, N, K, s1);
        }
        hipEvent_t e2;
        CK(hipEventCreate(&e2));
        CK(hipEventRecord(e2, s1));
        CK(hipStreamWaitEvent(s0, e2, 0));
        CK(hipEventRecord(e1, s0));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        CK(hipEventDestroy(e2));
        const double us2 = ms * 1e3 / iters / 2;
        printf("   | 2-stream %8.2f us/gemm %7.1f TF/s", us2, flop / us2 * 1e-6);
      }
      printf("\n");
    }
  }
  return 0;
}
