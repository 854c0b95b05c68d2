// Stream-K GEMM lab (bench only): times gemm_sk_kernel (ops/csrc/gemm_sk.h)
// against the shipped ping-pong tiles on the BERT serving shapes, with the
// epilogues they run in the model (bias, + residual), and checks every result
// -- the first launch AND the last of the timed loop (the workspace state
// words must reset between launches) -- against an fp32 reference GEMM.
//
//   hipcc -O3 --offload-arch=gfx950 -I ray_dynamic_batching_amd/ops/csrc bench/gemm_lab/sk_lab.hip -o labbin/sk_lab
//   ./labbin/sk_lab [--iters 50] [--concurrent] [--only substr]
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
#include "gemm_sk.h"

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
typedef std::function<void(const bf16*, const bf16*, const bf16*, const bf16*, bf16*, int, int, int, void*, hipStream_t)> RunF;
struct Variant { std::string name; RunF run; size_t ws_bytes; };

template <int BM, int BN, int GM, int GN, int S, int BK>
Variant pp(const char* nm) {
  return {nm, [](const bf16* A, const bf16* W, const bf16* b, const bf16* R, bf16* C, int M, int N, int K, void*, hipStream_t s) {
            launch_gemm_pp<bf16, bf16, 8, BM, BN, GM, GN, S, BK, 2>(A, K, W, K, C, N, b, R, R ? N : 0, M, N, K, 1.f, ACT_NONE, s);
          }, 0};
}
template <int BM, int BN, int GM, int GN, int S, int BK>
Variant sk(const char* nm, int grid) {
  return {nm, [grid](const bf16* A, const bf16* W, const bf16* b, const bf16* R, bf16* C, int M, int N, int K, void* ws,
                     hipStream_t s) {
            launch_gemm_sk<bf16, bf16, 8, BM, BN, GM, GN, S, BK>(A, K, W, K, C, N, b, R, R ? N : 0, M, N, K, 1.f, ACT_NONE, ws,
                                                                 grid, s);
          }, gemm_sk_workspace_bytes<BM, BN>(grid)};
}
Variant core10(const char* nm) {
  return {nm, [](const bf16* A, const bf16* W, const bf16* b, const bf16* R, bf16* C, int M, int N, int K, void*, hipStream_t s) {
            DenseParams p{A, K, M, K};
            if (R) launch_one<bf16, bf16, DenseLoader, true, true, 128, 96, 2, 4>(p, W, K, C, N, b, R, N, M, N, K, 1.f, ACT_NONE, s);
            else launch_one<bf16, bf16, DenseLoader, true, false, 128, 96, 2, 4>(p, W, K, C, N, b, nullptr, 0, M, N, K, 1.f, ACT_NONE, s);
          }, 0};
}

static double check(const std::vector<uint16_t>& hc, const std::vector<float>& hr, size_t n) {
  double maxerr = 0;
  for (size_t i = 0; i < n; ++i) {
    uint32_t u = (uint32_t)hc[i] << 16;
    float f;
    memcpy(&f, &u, 4);
    maxerr = std::max(maxerr, (double)fabsf(f - hr[i]) / (1.0 + fabsf(hr[i])));
  }
  return maxerr;
}

int main(int argc, char** argv) {
  int iters = 50;
  bool conc = false;
  std::string only;
  for (int i = 1; i < argc; ++i) {
    if (!strcmp(argv[i], "--iters")) iters = atoi(argv[++i]);
    else if (!strcmp(argv[i], "--concurrent")) conc = true;
    else if (!strcmp(argv[i], "--only")) only = argv[++i];
  }
  std::vector<Shape> shapes = {{4096, 768, 3072, true, "bert.ffn2+res"},
                               {4096, 768, 768, true, "bert.o+res"},
                               {4096, 2304, 768, false, "bert.qkv"},
                               {4096, 3072, 768, false, "bert.ffn1"},
                               {1000, 768, 3072, true, "ffn2 M=1000 (ragged)"}};
  std::vector<Variant> vs = {
      pp<256, 128, 2, 2, 3, 64>("pp 256x128 bk64 s3 (shipped ffn2)"),
      core10("core 128x96/4w (shipped o)"),
      sk<256, 128, 2, 2, 3, 64>("sk 256x128 bk64 s3 G256", 256),
      sk<256, 128, 2, 2, 3, 64>("sk 256x128 bk64 s3 G192", 192),
      sk<256, 128, 2, 2, 3, 64>("sk 256x128 bk64 s3 G128", 128),
      sk<128, 128, 2, 2, 4, 64>("sk 128x128 bk64 s4 G256", 256),
      sk<128, 128, 2, 2, 4, 64>("sk 128x128 bk64 s4 G192", 192),
      sk<256, 128, 2, 2, 4, 32>("sk 256x128 bk32 s4 G256", 256),
  };
  const size_t maxA = 4096ull * 4096, maxW = 4096ull * 4096, maxC = 4096ull * 4096;
  bf16 *A, *W, *bias, *R, *C, *C2;
  float* Cref;
  CK(hipMalloc(&A, maxA * 2));
  CK(hipMalloc(&W, maxW * 2));
  CK(hipMalloc(&bias, 4096 * 2));
  CK(hipMalloc(&R, maxC * 2));
  CK(hipMalloc(&C, maxC * 2));
  CK(hipMalloc(&C2, maxC * 2));
  CK(hipMalloc(&Cref, maxC * 4));
  size_t wsb = 0;
  for (auto& v : vs) wsb = std::max(wsb, v.ws_bytes);
  void *ws0 = nullptr, *ws1 = nullptr;
  CK(hipMalloc(&ws0, wsb + 4096));
  CK(hipMalloc(&ws1, wsb + 4096));
  CK(hipMemset(ws0, 0, wsb + 4096));
  CK(hipMemset(ws1, 0, wsb + 4096));
  fill_rand<<<1024, 256>>>(A, maxA, 1, 1.f);
  fill_rand<<<1024, 256>>>(W, maxW, 2, 0.05f);
  fill_rand<<<16, 256>>>(bias, 4096, 3, 1.f);
  fill_rand<<<1024, 256>>>(R, maxC, 4, 1.f);
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
    const bf16* Rp = sh.res ? R : nullptr;
    ref_gemm<<<dim3((N + 255) / 256, M), 256>>>(A, W, bias, Rp, Cref, M, N, K);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(hr.data(), Cref, (size_t)M * N * 4, hipMemcpyDeviceToHost));
    const double flop = 2.0 * M * N * K;
    printf("== %s M=%d N=%d K=%d\n", sh.name, M, N, K);
    for (auto& v : vs) {
      if (!only.empty() && v.name.find(only) == std::string::npos) continue;
      CK(hipMemset(C, 0, (size_t)M * N * 2));
      CK(hipDeviceSynchronize());   // hipMemset runs on the null stream: order it before the s0 launch
      v.run(A, W, bias, Rp, C, M, N, K, ws0, s0);
      CK(hipStreamSynchronize(s0));
      CK(hipGetLastError());
      CK(hipMemcpy(hc.data(), C, (size_t)M * N * 2, hipMemcpyDeviceToHost));
      const double err1 = check(hc, hr, (size_t)M * N);
      for (int i = 0; i < 5; ++i) v.run(A, W, bias, Rp, C, M, N, K, ws0, s0);
      CK(hipEventRecord(e0, s0));
      for (int i = 0; i < iters; ++i) v.run(A, W, bias, Rp, C, M, N, K, ws0, s0);
      CK(hipEventRecord(e1, s0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double us = ms * 1e3 / iters;
      CK(hipMemcpy(hc.data(), C, (size_t)M * N * 2, hipMemcpyDeviceToHost));
      const double err2 = check(hc, hr, (size_t)M * N);
      int werr = 0;

      printf("  %-36s %8.2f us %7.1f TF/s  err %.2e / %.2e%s%s", v.name.c_str(), us, flop / us * 1e-6, err1, err2,
             (err1 > 2e-2 || err2 > 2e-2) ? "  <-- WRONG" : "", werr ? "  <-- WAIT TIMEOUT" : "");
      if (conc) {
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0, s0));
        CK(hipStreamWaitEvent(s1, e0, 0));
        for (int i = 0; i < iters; ++i) {
          v.run(A, W, bias, Rp, C, M, N, K, ws0, s0);
          v.run(A, W, bias, Rp, C2, M, N, K, ws1, s1);
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
        CK(hipMemcpy(hc.data(), C2, (size_t)M * N * 2, hipMemcpyDeviceToHost));
        const double err3 = check(hc, hr, (size_t)M * N);
        printf("   | 2-stream %8.2f us/gemm %7.1f TF/s err %.2e%s", us2, flop / us2 * 1e-6, err3,
               err3 > 2e-2 ? " <-- WRONG" : "");
      }
      (void)werr;
      printf("\n");
      fflush(stdout);
    }
  }
  return 0;
}
