// Core MFMA GEMM main loop shared by the dense GEMM (gemm.hip) and the
// implicit-GEMM NHWC convolution (conv.hip).  Only the A-operand loader differs:
// DenseLoader reads a row-major [M, K] matrix, Im2colLoader gathers the
// [N*P*Q, R*S*C] im2col matrix on the fly from an NHWC activation tensor (it is
// never materialised).
//
//   C[m, n] = act(alpha * sum_k A[m, k] * W[n, k] + bias[n] + R[m, n])
//
// Design (cdna_hip_programming.md §5):
//  * 256 threads = 4 waves in a 2x2 grid; each wave owns (BM/2)x(BN/2).
//  * v_mfma_f32_16x16x32_{bf16,f16} with SWAPPED operands (W fragment as the
//    MFMA A operand): the accumulator then holds 4 consecutive n for one m per
//    lane, so the fused epilogue stores 8 contiguous bytes per lane.
//  * BK = 64, two LDS buffers, register-staged prefetch of tile k+1 issued
//    before the MFMAs of tile k (async-STAGE split, T14), one barrier per K-step.
//  * LDS rows are 128 B; the 16-B chunk index is XOR-swizzled with (row>>1)&7 so
//    each 16-lane group of ds_read_b128 hits 16 distinct bank quads (T2).
//  * XCD-aware bijective block remap: the N-tiles of one M-panel share an L2 (T1).
#pragma once
#include "common.h"

namespace rdb {

template <typename T> struct MfmaOp;
template <> struct MfmaOp<bf16> {
  typedef bf16x8 frag;
  static __device__ __forceinline__ f32x4 mma(frag a, frag b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
};
template <> struct MfmaOp<f16> {
  typedef f16x8 frag;
  static __device__ __forceinline__ f32x4 mma(frag a, frag b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
  }
};

__device__ __forceinline__ int swz_off(int row, int chunk) {
  return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4);
}

template <typename OutT>
__device__ __forceinline__ void store4(OutT* p, float a, float b, float c, float d);
template <>
__device__ __forceinline__ void store4<bf16>(bf16* p, float a, float b, float c, float d) {
  bf16x4 v = {(bf16)a, (bf16)b, (bf16)c, (bf16)d};
  *reinterpret_cast<bf16x4*>(p) = v;
}
template <>
__device__ __forceinline__ void store4<f16>(f16* p, float a, float b, float c, float d) {
  f16x4 v = {(f16)a, (f16)b, (f16)c, (f16)d};
  *reinterpret_cast<f16x4*>(p) = v;
}
template <>
__device__ __forceinline__ void store4<float>(float* p, float a, float b, float c, float d) {
  *reinterpret_cast<f32x4*>(p) = f32x4{a, b, c, d};
}

__device__ __forceinline__ float act_rt(int act, float x) {
  switch (act) {
    case ACT_GELU: return apply_act<ACT_GELU>(x);
    case ACT_RELU: return apply_act<ACT_RELU>(x);
    case ACT_TANH: return apply_act<ACT_TANH>(x);
    case ACT_SILU: return apply_act<ACT_SILU>(x);
    case ACT_GELU_TANH: return apply_act<ACT_GELU_TANH>(x);
    default: return x;
  }
}

// ---- A-operand loaders ------------------------------------------------------
struct DenseParams {
  const void* A;
  int lda, M, K;
};
template <typename T, int NCH>
struct DenseLoader {
  typedef DenseParams Params;
  const T* rowp[NCH];
  bool ok[NCH];
  int K;
  __device__ __forceinline__ void init(const Params& p, int tid, int m0) {
    K = p.K;
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int row = (tid + 256 * i) >> 3;
      const int gm = m0 + row;
      ok[i] = gm < p.M;
      rowp[i] = reinterpret_cast<const T*>(p.A) + (size_t)(ok[i] ? gm : 0) * p.lda;
    }
  }
  __device__ __forceinline__ u32x4 load(int i, int gk) const {
    if (ok[i] && gk < K) return *reinterpret_cast<const u32x4*>(rowp[i] + gk);
    return u32x4{0, 0, 0, 0};
  }
};

struct ConvParams {
  const void* x;  // NHWC
  int N, H, W, C, R, S, stride, pad, P, Q;
  int M, K;       // M = N*P*Q, K = R*S*C
};
template <typename T, int NCH>
struct Im2colLoader {
  typedef ConvParams Params;
  const T* img[NCH];
  int h0[NCH], w0[NCH];
  bool ok[NCH];
  int K, C, S, H, W;
  __device__ __forceinline__ void init(const Params& p, int tid, int m0) {
    K = p.K; C = p.C; S = p.S; H = p.H; W = p.W;
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int row = (tid + 256 * i) >> 3;
      int gm = m0 + row;
      ok[i] = gm < p.M;
      gm = ok[i] ? gm : 0;
      const int pq = p.P * p.Q;
      const int n = gm / pq;
      const int rem = gm - n * pq;
      const int pp = rem / p.Q, qq = rem - (rem / p.Q) * p.Q;
      h0[i] = pp * p.stride - p.pad;
      w0[i] = qq * p.stride - p.pad;
      img[i] = reinterpret_cast<const T*>(p.x) + (size_t)n * p.H * p.W * p.C;
    }
  }
  __device__ __forceinline__ u32x4 load(int i, int gk) const {
    if (!ok[i] || gk >= K) return u32x4{0, 0, 0, 0};
    const int rs = gk / C;
    const int cc = gk - rs * C;
    const int r = rs / S, s = rs - (rs / S) * S;
    const int h = h0[i] + r, w = w0[i] + s;
    if ((unsigned)h >= (unsigned)H || (unsigned)w >= (unsigned)W) return u32x4{0, 0, 0, 0};
    return *reinterpret_cast<const u32x4*>(img[i] + ((size_t)h * W + w) * C + cc);
  }
};

// ---- the kernel ---------------------------------------------------------------
template <typename T, typename OutT, int BM, int BN, template <typename, int> class LoaderT>
__global__ void __launch_bounds__(256, 2)
mfma_gemm_kernel(typename LoaderT<T, BM * 8 / 256>::Params ap, const T* __restrict__ W, int ldw,
                 OutT* __restrict__ C, int ldc, const T* __restrict__ bias,
                 const T* __restrict__ R, int ldr, int M, int N, int K, float alpha, int act) {
  constexpr int BK = 64;
  constexpr int WM = BM / 2, WN = BN / 2;
  constexpr int TM = WM / 16, TN = WN / 16;
  constexpr int A_CH = BM * 8 / 256;  // 16-B chunks per thread per A tile
  constexpr int W_CH = BN * 8 / 256;
  constexpr int kStage = (BM + BN) * BK * 2;  // bytes per LDS stage (A tile, then W tile)
  typedef typename MfmaOp<T>::frag frag;

  __shared__ __attribute__((aligned(16))) char smem[2 * kStage];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;

  const int tiles_n = (N + BN - 1) / BN;
  const int tiles_m = (M + BM - 1) / BM;
  const int nwg = tiles_m * tiles_n;
  const int t = xcd_remap(blockIdx.x, nwg);
  const int tile_m = t / tiles_n, tile_n = t - tile_m * tiles_n;
  const int m0 = tile_m * BM, n0 = tile_n * BN;

  LoaderT<T, A_CH> la;
  la.init(ap, tid, m0);
  const int cA = tid & 7;

  const T* wrow[W_CH];
  bool wok[W_CH];
#pragma unroll
  for (int i = 0; i < W_CH; ++i) {
    const int gn = n0 + ((tid + 256 * i) >> 3);
    wok[i] = gn < N;
    wrow[i] = W + (size_t)(wok[i] ? gn : 0) * ldw;
  }

  u32x4 ra[A_CH], rw[W_CH];
  auto gload = [&](int k0) {
    const int gk = k0 + cA * 8;
#pragma unroll
    for (int i = 0; i < A_CH; ++i) ra[i] = la.load(i, gk);
#pragma unroll
    for (int i = 0; i < W_CH; ++i)
      rw[i] = (wok[i] && gk < K) ? *reinterpret_cast<const u32x4*>(wrow[i] + gk) : u32x4{0, 0, 0, 0};
  };
  auto lstore = [&](int buf) {
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      const int row = (tid + 256 * i) >> 3;
      *reinterpret_cast<u32x4*>(smem + buf * kStage + swz_off(row, cA)) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < W_CH; ++i) {
      const int row = (tid + 256 * i) >> 3;
      *reinterpret_cast<u32x4*>(smem + buf * kStage + BM * BK * 2 + swz_off(row, cA)) = rw[i];
    }
  };

  f32x4 acc[TN][TM];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (K + BK - 1) / BK;
  gload(0);
  lstore(0);
  __syncthreads();

  const int fr = lane & 15, fg = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) gload((kt + 1) * BK);
    const char* sa = smem + cur * kStage;
    const char* sw = sa + BM * BK * 2;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      frag wf[TN], af[TM];
      const int chunk = ks * 4 + fg;
#pragma unroll
      for (int i = 0; i < TN; ++i)
        wf[i] = *reinterpret_cast<const frag*>(sw + swz_off(wn * WN + i * 16 + fr, chunk));
#pragma unroll
      for (int j = 0; j < TM; ++j)
        af[j] = *reinterpret_cast<const frag*>(sa + swz_off(wm * WM + j * 16 + fr, chunk));
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int j = 0; j < TM; ++j) acc[i][j] = MfmaOp<T>::mma(wf[i], af[j], acc[i][j]);
    }
    if (kt + 1 < nk) lstore(cur ^ 1);
    __syncthreads();
  }

  // ---- fused epilogue: lane holds C[m][n..n+3] ----
#pragma unroll
  for (int j = 0; j < TM; ++j) {
    const int m = m0 + wm * WM + j * 16 + fr;
    if (m >= M) continue;
#pragma unroll
    for (int i = 0; i < TN; ++i) {
      const int n = n0 + wn * WN + i * 16 + fg * 4;
      if (n >= N) continue;
      if (act == ACT_SWIGLU) {  // W rows interleaved (gate_j, up_j) -> out column n/2
        float g0 = alpha * acc[i][j][0], u0 = alpha * acc[i][j][1];
        float g1 = alpha * acc[i][j][2], u1 = alpha * acc[i][j][3];
        if (bias != nullptr) {
          g0 += (float)bias[n]; u0 += (float)bias[n + 1];
          g1 += (float)bias[n + 2]; u1 += (float)bias[n + 3];
        }
        float r0 = apply_act<ACT_SILU>(g0) * u0, r1 = apply_act<ACT_SILU>(g1) * u1;
        if (R != nullptr) {
          r0 += (float)R[(size_t)m * ldr + (n >> 1)];
          r1 += (float)R[(size_t)m * ldr + (n >> 1) + 1];
        }
        OutT* cp = C + (size_t)m * ldc + (n >> 1);
        cp[0] = (OutT)r0;
        cp[1] = (OutT)r1;
        continue;
      }
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float x = alpha * acc[i][j][e];
        if (bias != nullptr && n + e < N) x += (float)bias[n + e];
        if (R != nullptr && n + e < N) x += (float)R[(size_t)m * ldr + n + e];
        v[e] = act_rt(act, x);
      }
      OutT* cp = C + (size_t)m * ldc + n;
      if (n + 3 < N && ((ldc & 3) == 0)) {
        store4<OutT>(cp, v[0], v[1], v[2], v[3]);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (n + e < N) cp[e] = (OutT)v[e];
      }
    }
  }
}

// Tile selection: the largest tile that still puts >= 256 workgroups on the
// 256 CUs (fewer leaves CUs idle), else 64x64.
inline int pick_tile_cfg(int M, int N) {
  auto nwg = [&](int bm, int bn) { return ((M + bm - 1) / bm) * ((N + bn - 1) / bn); };
  if (nwg(128, 128) >= 256) return 0;
  if (nwg(64, 128) >= 256) return 1;
  if (nwg(128, 64) >= 256) return 2;
  return 3;
}

template <typename T, typename OutT, template <typename, int> class LoaderT, typename P>
void launch_mfma_gemm(const P& ap, const T* W, int ldw, OutT* C, int ldc, const T* bias, const T* R,
                      int ldr, int M, int N, int K, float alpha, int act, hipStream_t s, int cfg) {
  if (cfg < 0) cfg = pick_tile_cfg(M, N);
  auto nwg = [&](int bm, int bn) { return ((M + bm - 1) / bm) * ((N + bn - 1) / bn); };
  dim3 blk(256);
  switch (cfg) {
    case 0:
      hipLaunchKernelGGL((mfma_gemm_kernel<T, OutT, 128, 128, LoaderT>), dim3(nwg(128, 128)), blk, 0, s,
                         ap, W, ldw, C, ldc, bias, R, ldr, M, N, K, alpha, act);
      break;
    case 1:
      hipLaunchKernelGGL((mfma_gemm_kernel<T, OutT, 64, 128, LoaderT>), dim3(nwg(64, 128)), blk, 0, s,
                         ap, W, ldw, C, ldc, bias, R, ldr, M, N, K, alpha, act);
      break;
    case 2:
      hipLaunchKernelGGL((mfma_gemm_kernel<T, OutT, 128, 64, LoaderT>), dim3(nwg(128, 64)), blk, 0, s,
                         ap, W, ldw, C, ldc, bias, R, ldr, M, N, K, alpha, act);
      break;
    default:
      hipLaunchKernelGGL((mfma_gemm_kernel<T, OutT, 64, 64, LoaderT>), dim3(nwg(64, 64)), blk, 0, s,
                         ap, W, ldw, C, ldc, bias, R, ldr, M, N, K, alpha, act);
      break;
  }
}

}  // namespace rdb
