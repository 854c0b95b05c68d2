// ResNet stem in ONE kernel: uint8 image -> normalise -> 2x2 space-to-depth ->
// 4x4 / stride-1 conv (the 7x7 / stride-2 conv of the image, BN folded, see
// ops.stem_weight_s2d) -> bias + ReLU -> 3x3 / stride-2 max-pool, writing only
// the pooled f16 NHWC tensor.
//
// Unfused, the stem wrote its 112x112x64 activation (51 MB at bs32) for the
// max-pool to read back, and the space-to-depth image made another round trip:
// image_to_s2d 11 us + conv 54 us + maxpool 16.5 us per bs32 forward
// (profiles/trace_table_resnet50_forward_r4.txt).
//
// One workgroup (4 waves) = one image x an 8x8 tile of pooled outputs x all 64
// channels:
//   * the 17x17 stem pixels under its pooling windows (rows / cols 2*i0-1 ..
//     2*i0+15, a 1-pixel halo recomputed by the neighbour) need 20x20 space-to-
//     depth pixels: built in LDS straight from the image bytes (zero outside);
//   * the weights [64][256] (k = (bi*4 + bj)*16 + c) are staged in LDS once;
//   * MFMA 16x16x32 f16 with the im2col matrix read implicitly from the LDS
//     patch: a lane's 8-element k group is 8 channels of one tap = one 16-B LDS
//     read (row pitches padded to 48 B / 528 B: the 16 lanes of a fragment hit
//     distinct banks);
//   * bias + ReLU (positions outside the image are stored as 0: ReLU outputs
//     are >= 0 and every window holds a valid pixel, so 0 never wins the max),
//     parked as f16 in LDS over the dead patch / weights, then pooled.
#include "common.h"
#include <stdexcept>

namespace rdb {

namespace {
constexpr int kPT = 8;                     // pooled tile (kPT x kPT)
constexpr int kSR = 2 * kPT + 1;           // stem rows / cols per tile (17)
constexpr int kSM = kSR * kSR;             // stem pixels per tile (289)
constexpr int kMT = (kSM + 15) / 16;       // 16-row MFMA tiles (19)
constexpr int kXR = kSR + 3;               // space-to-depth rows / cols per tile (20)
constexpr int kXS = 24;                    // halfs per space-to-depth pixel in LDS (16 + pad)
constexpr int kWS = 264;                   // halfs per weight row in LDS (256 + pad)
constexpr int kOS = 72;                    // halfs per stem pixel in the output park (64 + pad)
constexpr int kXBytes = kXR * kXR * kXS * 2;          // 19,200
constexpr int kWBytes = 64 * kWS * 2;                 // 33,792
constexpr int kOBytes = kSM * kOS * 2;                // 41,616
constexpr int kLds = (kXBytes + kWBytes) > kOBytes ? (kXBytes + kWBytes) : kOBytes;
}  // namespace

__global__ void __launch_bounds__(256, 2)
stem_s2d_pool_kernel(const uint8_t* __restrict__ img, int H, int W, const f16* __restrict__ w,
                     const f16* __restrict__ bias, f16* __restrict__ out, float m0, float m1, float m2,
                     float s0, float s1, float s2, u32x4* __restrict__ zero, int zero_n) {
  __shared__ __attribute__((aligned(16))) char smem[kLds];
  f16* xp = reinterpret_cast<f16*>(smem);
  f16* wl = reinterpret_cast<f16*>(smem + kXBytes);
  f16* op = reinterpret_cast<f16*>(smem);   // after the MFMA phase (aliases xp / wl)

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int P = H >> 1, Q = W >> 1;         // stem output (= space-to-depth) size
  const int i0 = blockIdx.y * kPT, j0 = blockIdx.x * kPT, n = blockIdx.z;
  {
    // side job: zero a split-K counter header for the rest of the forward
    const int nthr = gridDim.x * gridDim.y * gridDim.z * 256;
    for (int z = ((blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x) * 256 + tid; z < zero_n; z += nthr)
      zero[z] = u32x4{0u, 0u, 0u, 0u};
  }

  // ---- weights -> LDS (2048 16-B chunks) ----
#pragma unroll
  for (int it = 0; it < 8; ++it) {
    const int e = it * 256 + tid;
    const int row = e >> 5, ch = e & 31;
    *reinterpret_cast<f16x8*>(wl + row * kWS + ch * 8) = *reinterpret_cast<const f16x8*>(w + row * 256 + ch * 8);
  }
  // ---- image bytes -> normalised space-to-depth patch in LDS ----
  const float a[3] = {1.f / (255.f * s0), 1.f / (255.f * s1), 1.f / (255.f * s2)};
  const float b[3] = {-m0 / s0, -m1 / s1, -m2 / s2};
  const uint8_t* im = img + (size_t)n * H * W * 3;
  for (int e = tid; e < kXR * kXR; e += 256) {
    const int rr = e / kXR, cc = e - rr * kXR;
    const int si = 2 * i0 - 3 + rr, sj = 2 * j0 - 3 + cc;
    f16x8 lo = {0, 0, 0, 0, 0, 0, 0, 0}, hi = {0, 0, 0, 0, 0, 0, 0, 0};
    if ((unsigned)si < (unsigned)P && (unsigned)sj < (unsigned)Q) {
#pragma unroll
      for (int dy = 0; dy < 2; ++dy) {
        // 6 bytes = pixels (2si+dy, 2sj) and (2si+dy, 2sj+1), RGB; 2-byte aligned
        const uint16_t* r16 = reinterpret_cast<const uint16_t*>(im + ((size_t)(2 * si + dy) * W + 2 * sj) * 3);
        const uint32_t u0 = r16[0], u1 = r16[1], u2 = r16[2];
        const uint32_t bytes[6] = {u0 & 255u, u0 >> 8, u1 & 255u, u1 >> 8, u2 & 255u, u2 >> 8};
#pragma unroll
        for (int t = 0; t < 6; ++t) {
          const int ch = dy * 6 + t;          // (dy*2 + dx)*3 + c with (dx, c) = (t / 3, t % 3)
          const f16 v = (f16)((float)bytes[t] * a[t % 3] + b[t % 3]);
          if (ch < 8) lo[ch] = v; else hi[ch - 8] = v;
        }
      }
    }
    f16* d = xp + e * kXS;
    *reinterpret_cast<f16x8*>(d) = lo;
    *reinterpret_cast<f16x8*>(d + 8) = hi;
  }
  __syncthreads();

  // ---- MFMA: wave w owns the 16-row tiles w, w+4, ... (<= 5) x all 4 column tiles ----
  const int fr = lane & 15, fg = lane >> 4;
  f32x4 acc[5][4];
  int pix[5];
#pragma unroll
  for (int t = 0; t < 5; ++t) {
    const int m = min((wid + 4 * t) * 16 + fr, kSM - 1);
    const int r = m / kSR, c = m - r * kSR;
    pix[t] = (r * kXR + c) * kXS;
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) acc[t][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int ks = 0; ks < 8; ++ks) {
    const int k = ks * 32 + fg * 8;                  // this lane's 8 k: one tap, 8 channels
    const int tap = k >> 4, c0 = k & 15;
    const int toff = ((tap >> 2) * kXR + (tap & 3)) * kXS + c0;
    f16x8 bf[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) bf[nt] = *reinterpret_cast<const f16x8*>(wl + (nt * 16 + fr) * kWS + k);
#pragma unroll
    for (int t = 0; t < 5; ++t) {
      if (wid + 4 * t < kMT) {                       // wave-uniform
        const f16x8 af = *reinterpret_cast<const f16x8*>(xp + pix[t] + toff);
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) acc[t][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bf[nt], af, acc[t][nt], 0, 0, 0);
      }
    }
  }
  __syncthreads();                                   // patch / weights dead: park the stem tile over them

  // ---- bias + ReLU -> f16 stem tile in LDS (lane: stem pixel m, channels n .. n+3) ----
  float bv[4][4];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt)
#pragma unroll
    for (int q = 0; q < 4; ++q) bv[nt][q] = (float)bias[nt * 16 + fg * 4 + q];
#pragma unroll
  for (int t = 0; t < 5; ++t) {
    const int m = (wid + 4 * t) * 16 + fr;
    if (wid + 4 * t < kMT && m < kSM) {
      const int r = m / kSR, c = m - r * kSR;
      const int p = 2 * i0 - 1 + r, q = 2 * j0 - 1 + c;
      const bool valid = (unsigned)p < (unsigned)P && (unsigned)q < (unsigned)Q;
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        f16x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = (f16)(valid ? fmaxf(acc[t][nt][e] + bv[nt][e], 0.f) : 0.f);
        *reinterpret_cast<f16x4*>(op + m * kOS + nt * 16 + fg * 4) = v;
      }
    }
  }
  __syncthreads();

  // ---- 3x3 / stride-2 max-pool of the tile: 8 x 8 pixels x 8 chunks of 8 channels ----
  const int Po = P >> 1, Qo = Q >> 1;
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int e = it * 256 + tid;
    const int px = e >> 3, c8 = e & 7;
    const int pi = px >> 3, pj = px & 7;
    f16x8 mx = *reinterpret_cast<const f16x8*>(op + ((2 * pi) * kSR + 2 * pj) * kOS + c8 * 8);
#pragma unroll
    for (int dy = 0; dy < 3; ++dy)
#pragma unroll
      for (int dx = 0; dx < 3; ++dx) {
        const f16x8 v = *reinterpret_cast<const f16x8*>(op + ((2 * pi + dy) * kSR + 2 * pj + dx) * kOS + c8 * 8);
#pragma unroll
        for (int q = 0; q < 8; ++q) mx[q] = v[q] > mx[q] ? v[q] : mx[q];
      }
    *reinterpret_cast<f16x8*>(out + (((size_t)n * Po + i0 + pi) * Qo + j0 + pj) * 64 + c8 * 8) = mx;
  }
}

void stem_s2d_pool(uintptr_t img, int N, int H, int W, uintptr_t w, uintptr_t bias, uintptr_t out, uintptr_t zero,
                   long zero_bytes, uintptr_t stream) {
  if (N <= 0) return;
  if (H % 32 != 0 || W % 32 != 0)
    throw std::invalid_argument("stem_s2d_pool: H and W must be multiples of 32 (8x8 pooled tiles)");
  if ((img & 1) || (w & 15) || (out & 15) || (zero & 15) || (zero_bytes & 15))
    throw std::invalid_argument("stem_s2d_pool: alignment (image 2 B, weights / out / zero 16 B)");
  const dim3 grid(W / 32, H / 32, N);
  const long zn = zero ? zero_bytes / 16 : 0;
  hipLaunchKernelGGL(stem_s2d_pool_kernel, grid, dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     (const uint8_t*)img, H, W, (const f16*)w, (const f16*)bias, (f16*)out, 0.485f, 0.456f, 0.406f,
                     0.229f, 0.224f, 0.225f, (u32x4*)zero, (int)zn);
  RDB_HIP_CHECK(hipGetLastError());
}

}  // namespace rdb
