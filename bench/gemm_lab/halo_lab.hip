// Diagnostic harness for the resident-weight halo conv (conv_halo.hip built with
// RDB_HALO_STAMPS): times variant v on a ResNet-50 bs32 3x3 layer, then prints
// the mean per-wave cycles of the loop segments (vmcnt wait, barrier, patch
// issue, MFMA taps, epilogue) and the kernel span.  Never part of the real build.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I../../ray_dynamic_batching_amd/ops/csrc \
//         -DRDB_HALO_STAMPS halo_lab.hip -o halo_lab && ./halo_lab 6 32 56 64 64
// (without -DRDB_HALO_STAMPS: the real kernels, timing only -- for counter runs)
#include "conv_halo.hip"
#include <cstdio>
#include <cstdlib>
#include <vector>

using namespace rdb;

int main(int argc, char** argv) {
  const int v = argc > 1 ? atoi(argv[1]) : 6, N = argc > 2 ? atoi(argv[2]) : 32, H = argc > 3 ? atoi(argv[3]) : 56;
  const int C = argc > 4 ? atoi(argv[4]) : 64, K = argc > 5 ? atoi(argv[5]) : 64;
  const size_t nx = (size_t)N * H * H * C, nw = (size_t)K * 9 * C, ny = (size_t)N * H * H * K;
  std::vector<f16> hx(nx), hw(nw), hb(K);
  for (size_t i = 0; i < nx; ++i) hx[i] = (f16)((rand() % 200 - 100) / 100.f);
  for (size_t i = 0; i < nw; ++i) hw[i] = (f16)((rand() % 200 - 100) / 3000.f);
  for (int i = 0; i < K; ++i) hb[i] = (f16)0.1f;
  f16 *x, *w, *b, *y;
  RDB_HIP_CHECK(hipMalloc(&x, nx * 2));
  RDB_HIP_CHECK(hipMalloc(&w, nw * 2));
  RDB_HIP_CHECK(hipMalloc(&b, K * 2));
  RDB_HIP_CHECK(hipMalloc(&y, ny * 2));
  RDB_HIP_CHECK(hipMemcpy(x, hx.data(), nx * 2, hipMemcpyHostToDevice));
  RDB_HIP_CHECK(hipMemcpy(w, hw.data(), nw * 2, hipMemcpyHostToDevice));
  RDB_HIP_CHECK(hipMemcpy(b, hb.data(), K * 2, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  RDB_HIP_CHECK(hipEventCreate(&e0));
  RDB_HIP_CHECK(hipEventCreate(&e1));
  for (int i = 0; i < 5; ++i) conv3x3_halo(v, x, w, y, b, nullptr, N, H, H, C, K, ACT_RELU, 0);
  RDB_HIP_CHECK(hipDeviceSynchronize());
  const int iters = 20;
  RDB_HIP_CHECK(hipEventRecord(e0, 0));
  for (int i = 0; i < iters; ++i) conv3x3_halo(v, x, w, y, b, nullptr, N, H, H, C, K, ACT_RELU, 0);
  RDB_HIP_CHECK(hipEventRecord(e1, 0));
  RDB_HIP_CHECK(hipEventSynchronize(e1));
  float ms = 0.f;
  RDB_HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
  static unsigned long long st[4096][8];
#ifdef RDB_HALO_STAMPS
  RDB_HIP_CHECK(hipMemcpyFromSymbol(st, HIP_SYMBOL(rdb_halo_stamps), sizeof(st)));
#endif
  double sum[8] = {0};
  int nw_ = 0;
  unsigned long long tmin = ~0ull, tmax = 0;
  for (int i = 0; i < 4096; ++i) {
    if (st[i][6] == 0) continue;
    ++nw_;
    for (int k = 0; k < 7; ++k) sum[k] += (double)st[i][k];
    tmin = st[i][7] < tmin ? st[i][7] : tmin;
    tmax = st[i][7] + st[i][0] > tmax ? st[i][7] + st[i][0] : tmax;
  }
  printf("{\"variant\": %d, \"shape\": [%d, %d, %d, %d, %d], \"us_per_launch\": %.2f, \"waves\": %d, "
         "\"units_per_wave\": %.1f, \"cycles_per_wave\": {\"loop_total\": %.0f, \"wait\": %.0f, \"barrier_or_bias\": %.0f, "
         "\"issue_or_setup\": %.0f, \"compute\": %.0f, \"epilogue\": %.0f}, \"last_launch_span_cycles\": %llu}\n",
         v, N, H, H, C, K, ms * 1e3 / iters, nw_, sum[6] / nw_, sum[0] / nw_, sum[1] / nw_, sum[2] / nw_, sum[3] / nw_,
         sum[4] / nw_, sum[5] / nw_, tmax - tmin);
  return 0;
}
