// Small memory-bound CNN glue kernels (ShuffleNetV2 /
// EfficientNetV2 rows):
//   * shuffle_remap - ShuffleNetV2's concat(x1, branch) + channel_shuffle(g=2)
//                     + the NEXT unit's channel split, fused into one index
//                     remap pass: logical out channel j comes from
//                     (j odd ? B : A)[j / 2]; written either as one full
//                     tensor or directly as the two halves the next unit
//                     consumes.  Physical channel counts are padded to a
//                     multiple of 8 (zero-filled) so every conv stays on the
//                     16-byte / MFMA-aligned path.
//   * se_scale      - EfficientNet squeeze-excitation: y = x * s[n, c] with
//                     8 channels (16 B) per lane.
#include "common.h"
#include <stdexcept>

namespace rdb {

__global__ void __launch_bounds__(256)
shuffle_remap_kernel(const f16* __restrict__ A, int ldA, const f16* __restrict__ B, int ldB, int Ch,
                     long pixels, f16* __restrict__ O1, int ld1, f16* __restrict__ O2, int ld2, int split) {
  // one thread per (pixel, physical output channel)
  const int w1 = ld1, w2 = split ? ld2 : 0;
  const long per_pix = w1 + w2;
  const long total = pixels * per_pix;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const long pix = e / per_pix;
    const int c = (int)(e - pix * per_pix);
    int j;       // logical channel of the shuffled concat
    f16* dst;
    if (c < w1) {
      j = c;
      dst = O1 + pix * ld1 + c;
      if (split ? (c >= Ch) : (c >= 2 * Ch)) { *dst = (f16)0.f; continue; }
    } else {
      const int c2 = c - w1;
      dst = O2 + pix * ld2 + c2;
      if (c2 >= Ch) { *dst = (f16)0.f; continue; }
      j = Ch + c2;
    }
    const f16 v = (j & 1) ? B[pix * ldB + (j >> 1)] : A[pix * ldA + (j >> 1)];
    *dst = v;
  }
}

void shuffle_remap(uintptr_t A, int ldA, uintptr_t B, int ldB, int Ch, long pixels, uintptr_t O1, int ld1,
                   uintptr_t O2, int ld2, int split, uintptr_t stream) {
  if (Ch <= 0 || pixels <= 0) return;
  if (ldA < Ch || ldB < Ch || (split ? (ld1 < Ch || ld2 < Ch) : ld1 < 2 * Ch))
    throw std::invalid_argument("shuffle_remap: leading dimensions too small");
  const long total = pixels * (ld1 + (split ? ld2 : 0));
  const int blocks = (int)std::min<long>((total + 255) / 256, 16384);
  hipLaunchKernelGGL(shuffle_remap_kernel, dim3(blocks), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     (const f16*)A, ldA, (const f16*)B, ldB, Ch, pixels, (f16*)O1, ld1, (f16*)O2, ld2, split);
  RDB_HIP_CHECK(hipGetLastError());
}

__global__ void __launch_bounds__(256)
se_scale_kernel(const f16* __restrict__ x, const f16* __restrict__ s, f16* __restrict__ y, int N, long HW,
                int C) {
  const int cg = C >> 3;
  const long total = (long)N * HW * cg;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const int c8 = (int)(e % cg);
    const long pix = e / cg;
    const int n = (int)(pix / HW);
    const f16x8 xv = *reinterpret_cast<const f16x8*>(x + pix * C + c8 * 8);
    const f16x8 sv = *reinterpret_cast<const f16x8*>(s + (long)n * C + c8 * 8);
    f16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (f16)((float)xv[j] * (float)sv[j]);
    *reinterpret_cast<f16x8*>(y + pix * C + c8 * 8) = o;
  }
}

void se_scale(uintptr_t x, uintptr_t s, uintptr_t y, int N, long HW, int C, uintptr_t stream) {
  if (C % 8 != 0) throw std::invalid_argument("se_scale: C must be a multiple of 8");
  if ((x | s | y) & 15) throw std::invalid_argument("se_scale: 16-byte alignment required");
  const long total = (long)N * HW * (C / 8);
  if (total <= 0) return;
  const int blocks = (int)std::min<long>((total + 255) / 256, 16384);
  hipLaunchKernelGGL(se_scale_kernel, dim3(blocks), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     (const f16*)x, (const f16*)s, (f16*)y, N, HW, C);
  RDB_HIP_CHECK(hipGetLastError());
}

}  // namespace rdb
