// Lab for the 4-wave VGPR-staged GEMM (bench/gemm_lab/gemm_v4.h) against the
// shipped ping-pong tiles on the BERT shapes and 4096^3; every result is
// checked against an fp32 reference GEMM on the GPU.  Timing: hipGraph-free
// back-to-back launches on one stream (median of 5 runs of --iters launches),
// plus --concurrent: the same GEMM on two streams side by side.
//
//   hipcc -O3 --offload-arch=gfx950 -I ray_dynamic_batching_amd/ops/csrc bench/gemm_lab/v4_lab.hip -o labbin/v4_lab
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
#include "gemm_v4a.h"

using namespace rdb;

#define CK(x)                                                                                   \
  do {                                                                                          \
    hipError_t e_ = (x);                                                                        \
    if (e_ != hipSuccess) {                                                                     \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(1);                                                                                  \
    }                                                                                           \
  } while (0)

__global__ void ref_gemm(const bf16* A, const bf16* W, const bf16* bias, const bf16* R, float* C, int M, int N, int K) {
  const int n = blockIdx.x * blockDim.x + threadIdx.x, m = blockIdx.y;
  if (n >= N) return;
  float s = 0.f;
  for (int k = 0; k < K; ++k) s += (float)A[(size_t)m * K + k] * (float)W[(size_t)n * K + k];
  C[(size_t)m * N + n] = s + (bias ? (float)bias[n] : 0.f) + (R ? (float)R[(size_t)m * N + n] : 0.f);
}

__global__ void fill_rand(bf16* p, size_t n, uint32_t seed, float scale) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  for (; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t x = (uint32_t)i * 2654435761u ^ seed;
    x ^= x >> 13; x *= 0x5bd1e995u; x ^= x >> 15;
    p[i] = (bf16)(((float)(x & 0xFFFFFF) / 16777216.f * 2.f - 1.f) * scale);
  }
}

struct Shape { int M, N, K; bool res; const char* name; };
typedef std::function<void(const bf16*, const bf16*, const bf16*, const bf16*, bf16*, int, int, int, hipStream_t)> Fn;
struct Variant { std::string name; Fn run; };

template <int BM, int BN, bool ASM = false>
Variant v4(const char* nm) {
  return {nm, [](const bf16* A, const bf16* W, const bf16* b, const bf16* R, bf16* C, int M, int N, int K, hipStream_t s) {
            launch_gemm_v4a<bf16, bf16, BM, BN, ASM>(A, K, W, K, C, N, b, R, N, M, N, K, 1.f, ACT_NONE, s);
          }};
}
template <int NW, int BM, int BN, int GM, int GN, int S, int BK = 64, int OCC = 2>
Variant pp(const char* nm) {
  return {nm, [](const bf16* A, const bf16* W, const bf16* b, const bf16* R, bf16* C, int M, int N, int K, hipStream_t s) {
            launch_gemm_pp<bf16, bf16, NW, BM, BN, GM, GN, S, BK, OCC>(A, K, W, K, C, N, b, R, N, M, N, K, 1.f,
                                                                   ACT_NONE, s);
          }};
}

int main(int argc, char** argv) {
  int iters = 50;
  bool conc = false;
  for (int i = 1; i < argc; ++i) {
    if (!strcmp(argv[i], "--iters") && i + 1 < argc) iters = atoi(argv[++i]);
    if (!strcmp(argv[i], "--concurrent")) conc = true;
  }
  std::vector<Shape> shapes = {{4096, 4096, 4096, false, "sq4096"},
                               {4096, 3072, 768, false, "ffn_up"},
                               {4096, 768, 3072, true, "ffn_down"},
                               {4096, 2304, 768, false, "qkv"},
                               {4096, 768, 768, true, "oproj"}};
  std::vector<Variant> vs = {
      pp<8, 256, 256, 2, 2, 4, 32>("pp 256x256 bk32 s4 (cfg22)"),
      pp<8, 256, 128, 2, 2, 3>("pp 256x128 (cfg19)"),
      pp<8, 256, 128, 2, 2, 3, 32, 4>("pp 256x128 bk32 occ2 (cfg23)"),
      pp<8, 256, 192, 2, 2, 4, 32>("pp 256x192 bk32 s4 (cfg25)"),
      v4<256, 256, true>("v4a 256x256 agpr-asm"),
      v4<256, 192, true>("v4a 256x192 agpr-asm"),
      v4<256, 128, true>("v4a 256x128 agpr-asm"),
      v4<128, 96, false>("v4 128x96 (vgpr-form)"),
  };
  size_t maxA = 0, maxW = 0, maxC = 0;
  for (auto& s : shapes) {
    maxA = std::max(maxA, (size_t)s.M * s.K);
    maxW = std::max(maxW, (size_t)s.N * s.K);
    maxC = std::max(maxC, (size_t)s.M * s.N);
  }
  bf16 *A, *Wt, *bias, *R, *C, *C2;
  float* Cref;
  CK(hipMalloc(&A, maxA * 2));
  CK(hipMalloc(&Wt, maxW * 2));
  CK(hipMalloc(&bias, 8192 * 2));
  CK(hipMalloc(&R, maxC * 2));
  CK(hipMalloc(&C, maxC * 2));
  CK(hipMalloc(&C2, maxC * 2));
  CK(hipMalloc(&Cref, maxC * 4));
  fill_rand<<<1024, 256>>>(A, maxA, 1, 1.f);
  fill_rand<<<1024, 256>>>(Wt, maxW, 2, 0.05f);
  fill_rand<<<64, 256>>>(bias, 8192, 3, 0.1f);
  fill_rand<<<1024, 256>>>(R, maxC, 4, 1.f);
  hipStream_t s0, s1;
  CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  hipEvent_t e0, e1, e2;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventCreate(&e2));
  for (auto& sh : shapes) {
    const int M = sh.M, N = sh.N, K = sh.K;
    const bf16* Rp = sh.res ? R : nullptr;
    ref_gemm<<<dim3((N + 255) / 256, M), 256>>>(A, Wt, bias, Rp, Cref, M, N, K);
    CK(hipDeviceSynchronize());
    std::vector<float> hr((size_t)M * N);
    CK(hipMemcpy(hr.data(), Cref, (size_t)M * N * 4, hipMemcpyDeviceToHost));
    const double flop = 2.0 * M * N * K;
    for (auto& v : vs) {
      CK(hipMemset(C, 0, (size_t)M * N * 2));
      v.run(A, Wt, bias, Rp, C, M, N, K, s0);
      CK(hipStreamSynchronize(s0));
      std::vector<bf16> hc((size_t)M * N);
      CK(hipMemcpy(hc.data(), C, (size_t)M * N * 2, hipMemcpyDeviceToHost));
      double maxerr = 0, maxref = 0;
      for (size_t i = 0; i < hc.size(); ++i) {
        maxerr = std::max(maxerr, (double)std::fabs((float)hc[i] - hr[i]));
        maxref = std::max(maxref, (double)std::fabs(hr[i]));
      }
      const bool ok = maxerr <= 0.02 * maxref + 0.05;
      std::vector<float> ts;
      for (int r = 0; r < 5; ++r) {
        CK(hipEventRecord(e0, s0));
        for (int i = 0; i < iters; ++i) v.run(A, Wt, bias, Rp, C, M, N, K, s0);
        CK(hipEventRecord(e1, s0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ts.push_back(ms * 1e3f / iters);
      }
      std::sort(ts.begin(), ts.end());
      const float us = ts[2];
      float us2 = 0;
      if (conc) {
        std::vector<float> t2;
        for (int r = 0; r < 5; ++r) {
          CK(hipDeviceSynchronize());
          CK(hipEventRecord(e0, s0));
          CK(hipStreamWaitEvent(s1, e0, 0));
          for (int i = 0; i < iters; ++i) {
            v.run(A, Wt, bias, Rp, C, M, N, K, s0);
            v.run(A, Wt, bias, Rp, C2, M, N, K, s1);
          }
          CK(hipEventRecord(e2, s1));
          CK(hipStreamWaitEvent(s0, e2, 0));
          CK(hipEventRecord(e1, s0));
          CK(hipEventSynchronize(e1));
          float ms;
          CK(hipEventElapsedTime(&ms, e0, e1));
          t2.push_back(ms * 1e3f / (2 * iters));
        }
        std::sort(t2.begin(), t2.end());
        us2 = t2[2];
      }
      printf("%-9s %-30s %8.2f us %7.1f TF/s", sh.name, v.name.c_str(), us, flop / us / 1e6);
      if (conc) printf("  2-stream %7.2f us/GEMM %7.1f TF/s", us2, flop / us2 / 1e6);
      printf("  maxerr %.4f%s\n", maxerr, ok ? "" : "  <-- WRONG");
      fflush(stdout);
    }
  }
  return 0;
}
