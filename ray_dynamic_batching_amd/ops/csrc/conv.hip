// NHWC convolution family for gfx950 (ResNet-50 / ShuffleNet / EfficientNet
// forward):
//   * conv2d_nhwc  - implicit-GEMM conv on MFMA (f16): the im2col matrix is
//                    gathered tile-by-tile into LDS by Im2colLoader (never
//                    materialised); BN is folded into (W, bias) at load time and
//                    bias + residual + ReLU/SiLU are fused into the epilogue.
//   * dwconv_nhwc  - depthwise conv (memory-bound; 8 channels per lane, 16-B loads)
//   * maxpool_nhwc / avgpool_nhwc (global average pool feeding the FC GEMM)
#include "gemm_core.h"
#include <stdexcept>

namespace rdb {

// ---- ping-pong implicit-GEMM convolutions (force_cfg = kConvPPFlag | v | splits << 8) ----
// The 8-wave two-group ping-pong kernel (gemm_pp.h) with the im2col A operand:
// the per-wave tiles (64 x 64 / 64 x 32) read half the LDS bytes per MFMA of the
// 4-wave 64 x 128 / 128 x 64 im2col tiles, and split-K keeps the small-M layers
// (ResNet stages 3 / 4: M = 6272 / 1568 at batch 32) on >= ~200 blocks.
constexpr int kConvPPFlag = 1 << 17;
// force_cfg = kConvHaloFlag | v: the halo-tile 3x3 kernel (conv_halo.hip)
constexpr int kConvHaloFlag = 1 << 18;
void conv3x3_halo(int v, const void* x, const void* w, void* y, const void* bias, const void* res, int N, int H, int W,
                  int C, int K, int stride, int act, hipStream_t s, int splits, void* ws, size_t ws_bytes);
constexpr int kNumConvPP = 5;
//                                  0    1    2    3    4
constexpr int kConvPPBM[kNumConvPP] = {256, 128, 256, 256, 128};
constexpr int kConvPPBN[kNumConvPP] = {128, 256, 128, 64, 128};
constexpr int kConvPPBK[kNumConvPP] = {64, 64, 32, 64, 32};

static size_t conv_pp_splitk_bytes(int M, int N, int v, int splits) {
  const size_t tiles = (size_t)((M + kConvPPBM[v] - 1) / kConvPPBM[v]) * ((N + kConvPPBN[v] - 1) / kConvPPBN[v]);
  return kSplitKHeader + tiles * splits * kConvPPBM[v] * kConvPPBN[v] * sizeof(float);
}

template <int BM, int BN, int GM, int GN, int STAGES, int BK, int OCC>
static void launch_conv_pp(const ConvParams& p, const f16* w, f16* y, const f16* bias, const f16* res, int N, int act,
                           hipStream_t s, int splits, void* ws, size_t ws_bytes) {
  const int M = p.M, K = p.K;
  if (p.C % BK != 0) throw std::invalid_argument("conv2d_nhwc: ping-pong conv tiles need C % BK == 0");
  if (bias == nullptr || act == ACT_SWIGLU || !gemm_pp_ok(N, N, N, y, bias, res, act))
    throw std::invalid_argument("conv2d_nhwc: ping-pong conv tiles need a bias, N % 8 == 0, 16-B aligned y / residual");
  const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  LnEpi ln{};
  int eff = 1;
  if (splits > 1 && ws != nullptr) {
    const int nk = K / BK;
    const int kper = (nk + splits - 1) / splits;
    eff = (nk + kper - 1) / kper;
    const size_t need = kSplitKHeader + (size_t)tiles * eff * BM * BN * sizeof(float);
    if (eff >= 2 && tiles <= kSplitKMaxTiles && need <= ws_bytes && need - kSplitKHeader <= (size_t(1) << 31)) {
      ln.sk_cnt = static_cast<int*>(ws);
      ln.sk_part = reinterpret_cast<float*>(static_cast<char*>(ws) + kSplitKHeader);
      ln.sk_kper = kper;
    } else {
      eff = 1;
    }
  }
  const ConvGeom cv{p.H, p.W, p.C, p.S, p.stride, p.pad, p.P, p.Q, (uint32_t)((size_t)p.N * p.H * p.W * p.C * sizeof(f16))};
  const f16* x = static_cast<const f16*>(p.x);
  const dim3 grid(tiles, eff), block(512);
  if (res)
    hipLaunchKernelGGL((gemm_pp_kernel<f16, f16, 8, BM, BN, GM, GN, STAGES, true, true, BK, OCC, 0, true>), grid, block, 0,
                       s, x, 0, w, K, y, N, bias, res, N, M, N, K, 1.f, act, ln, cv);
  else
    hipLaunchKernelGGL((gemm_pp_kernel<f16, f16, 8, BM, BN, GM, GN, STAGES, true, false, BK, OCC, 0, true>), grid, block, 0,
                       s, x, 0, w, K, y, N, bias, res, N, M, N, K, 1.f, act, ln, cv);
}

static void conv_pp(int v, const ConvParams& p, const f16* w, f16* y, const f16* bias, const f16* res, int N, int act,
                    hipStream_t s, int splits, void* ws, size_t ws_bytes) {
  switch (v) {
    case 0: launch_conv_pp<256, 128, 2, 2, 3, 64, 2>(p, w, y, bias, res, N, act, s, splits, ws, ws_bytes); return;
    case 1: launch_conv_pp<128, 256, 1, 4, 3, 64, 2>(p, w, y, bias, res, N, act, s, splits, ws, ws_bytes); return;
    case 2: launch_conv_pp<256, 128, 2, 2, 3, 32, 4>(p, w, y, bias, res, N, act, s, splits, ws, ws_bytes); return;
    case 3: launch_conv_pp<256, 64, 2, 2, 3, 64, 2>(p, w, y, bias, res, N, act, s, splits, ws, ws_bytes); return;
    case 4: launch_conv_pp<128, 128, 1, 4, 4, 32, 4>(p, w, y, bias, res, N, act, s, splits, ws, ws_bytes); return;
    default: throw std::invalid_argument("conv2d_nhwc: unknown ping-pong conv tile");
  }
}

// force_cfg = tile | (splits << 8) [| kDeepFlag]: splits > 1 runs split-K on the workspace
// `ws` (ws_bytes; zeroed counter header, see splitk_bytes) when it fits, else unsplit.
// force_cfg = kConvPPFlag | v | (splits << 8): ping-pong conv tile v (R x S convs
// and strided 1 x 1 -- the im2col operand; C % BK == 0, bias required).
void conv2d_nhwc(uintptr_t x, uintptr_t w, uintptr_t bias, uintptr_t res, uintptr_t y, int N, int H,
                 int W, int C, int K, int R, int S, int stride, int pad, int P, int Q, int act,
                 uintptr_t stream, int force_cfg, uintptr_t ws, size_t ws_bytes) {
  if (C % 8 != 0) throw std::invalid_argument("conv2d_nhwc: C must be a multiple of 8 (pad channels)");
  if ((x | w) & 15) throw std::invalid_argument("conv2d_nhwc: x/w must be 16-byte aligned");
  if (P > (H + 2 * pad - R) / stride + 1 || Q > (W + 2 * pad - S) / stride + 1)
    throw std::invalid_argument("conv2d_nhwc: P / Q larger than the padded output");
  const int M = N * P * Q, Kg = R * S * C;
  if (M <= 0 || K <= 0) return;
  if (force_cfg >= 0 && (force_cfg & kConvHaloFlag)) {
    if (R != 3 || S != 3 || (stride != 1 && stride != 2) || pad != 1 || P != (H - 1) / stride + 1 ||
        Q != (W - 1) / stride + 1)
      throw std::invalid_argument("conv2d_nhwc: halo conv tiles are 3x3, stride 1 or 2, pad 1, full output");
    conv3x3_halo(force_cfg & 255, reinterpret_cast<const void*>(x), reinterpret_cast<const void*>(w),
                 reinterpret_cast<void*>(y), reinterpret_cast<const void*>(bias), reinterpret_cast<const void*>(res), N,
                 H, W, C, K, stride, act, reinterpret_cast<hipStream_t>(stream), (force_cfg >> 8) & 15,
                 reinterpret_cast<void*>(ws), ws_bytes);
    return;
  }
  if (force_cfg >= 0 && (force_cfg & kConvPPFlag)) {
    ConvParams p{reinterpret_cast<const void*>(x), N, H, W, C, R, S, stride, pad, P, Q, M, Kg};
    conv_pp(force_cfg & 255, p, (const f16*)w, (f16*)y, (const f16*)bias, (const f16*)res, K, act,
            reinterpret_cast<hipStream_t>(stream), (force_cfg >> 8) & 15, reinterpret_cast<void*>(ws), ws_bytes);
    RDB_HIP_CHECK(hipGetLastError());
    return;
  }
  const int tile = force_cfg < 0 ? -1 : (force_cfg & 255);
  const int splits = force_cfg < 0 ? 1 : ((force_cfg >> 8) & 15);
  const int cfg = force_cfg < 0 ? -1 : (tile | (force_cfg & kDeepFlag));
  const LnEpi sk = splitk_epi(M, K, Kg, tile, splits, reinterpret_cast<void*>(ws), ws_bytes);
  ConvParams p{reinterpret_cast<const void*>(x), N, H, W, C, R, S, stride, pad, P, Q, M, Kg};
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (R == 1 && S == 1 && stride == 1 && pad == 0) {
    // 1x1 stride-1 conv is a plain GEMM over the NHWC pixels.
    DenseParams d{reinterpret_cast<const void*>(x), C, M, C};
    launch_mfma_gemm<f16, f16, DenseLoader>(d, (const f16*)w, Kg, (f16*)y, K, (const f16*)bias,
                                            (const f16*)res, K, M, K, Kg, 1.f, act, s, cfg, sk);
  } else {
    launch_mfma_gemm<f16, f16, Im2colLoader>(p, (const f16*)w, Kg, (f16*)y, K, (const f16*)bias,
                                             (const f16*)res, K, M, K, Kg, 1.f, act, s, cfg, sk);
  }
  RDB_HIP_CHECK(hipGetLastError());
}

size_t conv_splitk_bytes(int M, int N, int cfg, int splits) {
  if (cfg & kConvHaloFlag) return 0;
  if (cfg & kConvPPFlag) return conv_pp_splitk_bytes(M, N, cfg & 255, splits);
  return splitk_bytes(M, N, cfg & 255, splits);
}

// Depthwise RxR conv, NHWC f16, weights [R][R][C] (channel-contiguous), bias [C].
// One thread = 8 channels of one output pixel.
__global__ void __launch_bounds__(256)
dwconv_kernel(const f16* __restrict__ x, const f16* __restrict__ w, const f16* __restrict__ b,
              f16* __restrict__ y, int N, int H, int W, int C, int R, int stride, int pad, int P, int Q,
              int act) {
  const int cg = C >> 3;
  const long total = (long)N * P * Q * cg;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const int c8 = e % cg;
    const long pix = e / cg;
    const int q = pix % Q;
    const int p = (pix / Q) % P;
    const int n = pix / ((long)P * Q);
    float acc[8];
    const f16x8 bv = *reinterpret_cast<const f16x8*>(b + c8 * 8);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = (float)bv[j];
    for (int r = 0; r < R; ++r) {
      const int h = p * stride - pad + r;
      if ((unsigned)h >= (unsigned)H) continue;
      for (int s = 0; s < R; ++s) {
        const int ww = q * stride - pad + s;
        if ((unsigned)ww >= (unsigned)W) continue;
        const f16x8 xv = *reinterpret_cast<const f16x8*>(x + (((size_t)n * H + h) * W + ww) * C + c8 * 8);
        const f16x8 wv = *reinterpret_cast<const f16x8*>(w + ((size_t)r * R + s) * C + c8 * 8);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += (float)xv[j] * (float)wv[j];
      }
    }
    f16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (f16)act_rt(act, acc[j]);
    *reinterpret_cast<f16x8*>(y + (size_t)pix * C + c8 * 8) = o;
  }
}

void dwconv_nhwc(uintptr_t x, uintptr_t w, uintptr_t bias, uintptr_t y, int N, int H, int W, int C,
                 int R, int stride, int pad, int P, int Q, int act, uintptr_t stream) {
  if (C % 8 != 0) throw std::invalid_argument("dwconv_nhwc: C must be a multiple of 8");
  const long total = (long)N * P * Q * (C / 8);
  if (total <= 0) return;
  int blocks = (int)std::min<long>((total + 255) / 256, 8192);
  hipLaunchKernelGGL(dwconv_kernel, dim3(blocks), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     (const f16*)x, (const f16*)w, (const f16*)bias, (f16*)y, N, H, W, C, R, stride, pad,
                     P, Q, act);
  RDB_HIP_CHECK(hipGetLastError());
}

__global__ void __launch_bounds__(256)
maxpool_kernel(const f16* __restrict__ x, f16* __restrict__ y, int N, int H, int W, int C, int k,
               int stride, int pad, int P, int Q) {
  const int cg = C >> 3;
  const long total = (long)N * P * Q * cg;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const int c8 = e % cg;
    const long pix = e / cg;
    const int q = pix % Q;
    const int p = (pix / Q) % P;
    const int n = pix / ((long)P * Q);
    float m[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) m[j] = -INFINITY;
    for (int r = 0; r < k; ++r) {
      const int h = p * stride - pad + r;
      if ((unsigned)h >= (unsigned)H) continue;
      for (int s = 0; s < k; ++s) {
        const int ww = q * stride - pad + s;
        if ((unsigned)ww >= (unsigned)W) continue;
        const f16x8 xv = *reinterpret_cast<const f16x8*>(x + (((size_t)n * H + h) * W + ww) * C + c8 * 8);
#pragma unroll
        for (int j = 0; j < 8; ++j) m[j] = fmaxf(m[j], (float)xv[j]);
      }
    }
    f16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (f16)m[j];
    *reinterpret_cast<f16x8*>(y + (size_t)pix * C + c8 * 8) = o;
  }
}

void maxpool_nhwc(uintptr_t x, uintptr_t y, int N, int H, int W, int C, int k, int stride, int pad,
                  int P, int Q, uintptr_t stream) {
  if (C % 8 != 0) throw std::invalid_argument("maxpool_nhwc: C must be a multiple of 8");
  const long total = (long)N * P * Q * (C / 8);
  if (total <= 0) return;
  int blocks = (int)std::min<long>((total + 255) / 256, 8192);
  hipLaunchKernelGGL(maxpool_kernel, dim3(blocks), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     (const f16*)x, (f16*)y, N, H, W, C, k, stride, pad, P, Q);
  RDB_HIP_CHECK(hipGetLastError());
}

// Global average pool [N, HW, C] -> [N, C]: a block owns (n, 256 channels) --
// 32 lanes x 8 channels per row slice, 8 slices of the HW positions -- and the
// slices meet in LDS.  (One block per image with one thread per 8 channels left
// 32 blocks for 256 CUs: 15.7 us at ResNet-50 bs32, profiles/pmc_resnet50_forward_r3.json.)
__global__ void __launch_bounds__(256)
avgpool_kernel(const f16* __restrict__ x, f16* __restrict__ y, int N, int HW, int C) {
  constexpr int CG = 32, SL = 8;
  __shared__ float part[SL][CG * 8 + 4];
  const int n = blockIdx.y;
  const int cl = threadIdx.x % CG, sl = threadIdx.x / CG;
  const int c8 = blockIdx.x * CG + cl;
  const bool on = c8 * 8 < C;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (on) {
    const f16* base = x + (size_t)n * HW * C + c8 * 8;
    int i = sl;
#pragma unroll 1
    for (; i + SL < HW; i += 2 * SL) {     // two independent 16-B loads in flight
      const f16x8 a = *reinterpret_cast<const f16x8*>(base + (size_t)i * C);
      const f16x8 b = *reinterpret_cast<const f16x8*>(base + (size_t)(i + SL) * C);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += (float)a[j] + (float)b[j];
    }
    if (i < HW) {
      const f16x8 a = *reinterpret_cast<const f16x8*>(base + (size_t)i * C);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += (float)a[j];
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) part[sl][cl * 8 + j] = acc[j];
  __syncthreads();
  // 256 threads finish 256 channels: thread t sums channel t over the slices
  const int ch = blockIdx.x * CG * 8 + threadIdx.x;
  if (ch < C) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < SL; ++k) s += part[k][threadIdx.x];
    y[(size_t)n * C + ch] = (f16)(s / HW);
  }
}

void avgpool_nhwc(uintptr_t x, uintptr_t y, int N, int HW, int C, uintptr_t stream) {
  if (C % 8 != 0) throw std::invalid_argument("avgpool_nhwc: C must be a multiple of 8");
  if (N <= 0 || HW <= 0) return;
  dim3 grid((C + 255) / 256, N);
  hipLaunchKernelGGL(avgpool_kernel, grid, dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     (const f16*)x, (f16*)y, N, HW, C);
  RDB_HIP_CHECK(hipGetLastError());
}

}  // namespace rdb
