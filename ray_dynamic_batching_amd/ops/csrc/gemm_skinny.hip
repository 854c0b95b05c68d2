// Skinny-M GEMM (M <= 64): the batch-row GEMMs of a serving forward -- BERT's
// pooler / classifier and its CLS-only last layer, the Llama LM head on the
// last token of each prompt, a CNN's FC at small batch.  At M <= 64 the tiled
// kernel (gemm_core.h) runs N/BN blocks that each walk the whole K with a
// mostly-empty M tile: 12 blocks for 32 x 768 x 3072.  This kernel is the
// guide's weight-streaming form instead (cdna_hip_programming.md §5, "GEMV /
// M <= 16 decode weights" row): operands go straight to VGPRs, no LDS staging.
//
//   C[m, n] = act(alpha * sum_k A[m, k] * W[n, k] + bias[n] + R[m, n])
//
//  * one block = 8 waves = one 16-column slice of W; wave w walks the K range
//    [w*K/8, (w+1)*K/8), so W is streamed from HBM exactly once, 8 K-streams
//    deep per CU; A (<= 64 x K, a few hundred KB) stays L2-resident and is
//    re-read by every block;
//  * v_mfma_f32_16x16x32 with SWAPPED operands (W fragment as MFMA-A): each
//    lane ends with 4 consecutive n of one m, the same epilogue layout as the
//    tiled kernel; A fragments of the up-to-4 M tiles share one W fragment;
//  * the 8 partial accumulators meet in LDS (fixed order, deterministic) and
//    wave 0 applies the fused epilogue.
#include "common.h"
#include <stdexcept>

namespace rdb {

constexpr int kSkWaves = 8;

template <typename T> struct SkMfma;
template <> struct SkMfma<bf16> {
  typedef bf16x8 frag;
  static __device__ __forceinline__ f32x4 mma(frag a, frag b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
};
template <> struct SkMfma<f16> {
  typedef f16x8 frag;
  static __device__ __forceinline__ f32x4 mma(frag a, frag b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
  }
};

template <typename OutT> __device__ __forceinline__ void sk_store(OutT* p, const float (&y)[4], int valid);
template <> __device__ __forceinline__ void sk_store<float>(float* p, const float (&y)[4], int valid) {
  if (valid == 4) { *reinterpret_cast<f32x4*>(p) = f32x4{y[0], y[1], y[2], y[3]}; return; }
  for (int e = 0; e < valid; ++e) p[e] = y[e];
}
template <> __device__ __forceinline__ void sk_store<bf16>(bf16* p, const float (&y)[4], int valid) {
  if (valid == 4) { *reinterpret_cast<bf16x4*>(p) = bf16x4{(bf16)y[0], (bf16)y[1], (bf16)y[2], (bf16)y[3]}; return; }
  for (int e = 0; e < valid; ++e) p[e] = (bf16)y[e];
}
template <> __device__ __forceinline__ void sk_store<f16>(f16* p, const float (&y)[4], int valid) {
  if (valid == 4) { *reinterpret_cast<f16x4*>(p) = f16x4{(f16)y[0], (f16)y[1], (f16)y[2], (f16)y[3]}; return; }
  for (int e = 0; e < valid; ++e) p[e] = (f16)y[e];
}

__device__ __forceinline__ float sk_act(int act, float x) {
  switch (act) {
    case ACT_GELU: return apply_act<ACT_GELU>(x);
    case ACT_RELU: return apply_act<ACT_RELU>(x);
    case ACT_TANH: return apply_act<ACT_TANH>(x);
    case ACT_SILU: return apply_act<ACT_SILU>(x);
    case ACT_GELU_TANH: return apply_act<ACT_GELU_TANH>(x);
    case ACT_SIGMOID: return apply_act<ACT_SIGMOID>(x);
    default: return x;
  }
}

// MT = number of 16-row M tiles (M <= 16 * MT); U = K-steps (of 32) whose
// loads a wave issues together before their MFMAs.  The launcher picks U >=
// the wave's step count whenever the registers allow, so all of a wave's W / A
// loads are in flight at once: one memory latency per wave instead of one per
// step (at K = 768 a wave owns 3 steps, at K = 3072 12).  The epilogue's bias
// and residual are fetched before the main loop, under it.
template <typename T, typename OutT, int MT, int U>
__global__ void __launch_bounds__(kSkWaves * 64)
skinny_gemm_kernel(const T* __restrict__ A, int lda, const T* __restrict__ W, int ldw, OutT* __restrict__ C, int ldc,
                   const T* __restrict__ bias, const T* __restrict__ R, int ldr, int M, int N, int K, float alpha,
                   int act) {
  typedef typename SkMfma<T>::frag frag;
  __shared__ f32x4 red[kSkWaves][MT][64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int n0 = blockIdx.x * 16;
  const int fr = lane & 15, fg = lane >> 4;

  // epilogue operands of the finishing waves (wave t < MT finishes M tile t)
  const int m_ep = wid * 16 + fr, n_ep = n0 + fg * 4;
  const int valid = N - n_ep < 4 ? N - n_ep : 4;
  float bv[4] = {0.f, 0.f, 0.f, 0.f}, rv[4] = {0.f, 0.f, 0.f, 0.f};
  if (wid < MT && m_ep < M && n_ep < N) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if (e < valid) {
        if (bias) bv[e] = (float)bias[n_ep + e];
        if (R) rv[e] = (float)R[(size_t)m_ep * ldr + n_ep + e];
      }
    }
  }

  // this wave's K range, in whole 32-deep steps
  const int steps = K / 32;
  const int per = (steps + kSkWaves - 1) / kSkWaves;
  const int s0 = wid * per, s1 = min(steps, s0 + per);

  // W row (n) of this lane, clamped (rows past N compute garbage that is never stored)
  const int wn = min(n0 + fr, N - 1);
  const T* wrow = W + (size_t)wn * ldw + fg * 8;
  const T* arow[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) arow[t] = A + (size_t)min(t * 16 + fr, M - 1) * lda + fg * 8;

  f32x4 acc[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};

  for (int s = s0; s < s1; s += U) {
    frag wf[U], af[U][MT];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (s + u < s1) {                       // wave-uniform
        wf[u] = *reinterpret_cast<const frag*>(wrow + (s + u) * 32);
#pragma unroll
        for (int t = 0; t < MT; ++t) af[u][t] = *reinterpret_cast<const frag*>(arow[t] + (s + u) * 32);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (s + u < s1)
#pragma unroll
        for (int t = 0; t < MT; ++t) acc[t] = SkMfma<T>::mma(wf[u], af[u][t], acc[t]);
  }

#pragma unroll
  for (int t = 0; t < MT; ++t) red[wid][t][lane] = acc[t];
  __syncthreads();
  if (wid >= MT) return;
  // wave t finishes M tile t: lane holds C[m = t*16 + fr][n0 + fg*4 .. +3]
  const int t = wid;
  f32x4 v = red[0][t][lane];
#pragma unroll
  for (int w = 1; w < kSkWaves; ++w) v += red[w][t][lane];
  if (m_ep >= M || n_ep >= N) return;
  float y[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) y[e] = sk_act(act, alpha * v[e] + bv[e] + rv[e]);
  sk_store<OutT>(C + (size_t)m_ep * ldc + n_ep, y, (valid == 4 && (ldc & 3) == 0) ? 4 : valid);
}

template <typename T, typename OutT, int MT>
static void launch_sk_mt(const T* A, int lda, const T* W, int ldw, OutT* C, int ldc, const T* bias, const T* R,
                         int ldr, int M, int N, int K, float alpha, int act, hipStream_t s) {
  const dim3 grid((N + 15) / 16), block(kSkWaves * 64);
  const int per = (K / 32 + kSkWaves - 1) / kSkWaves;
  // all of a wave's steps in flight at once while (MT + 1) * U frags fit ~200 VGPRs
  constexpr int UMAX = (MT + 1) * 16 * 4 <= 200 ? 16 : 8;
#define RDB_SKU(U_) hipLaunchKernelGGL((skinny_gemm_kernel<T, OutT, MT, U_>), grid, block, 0, s, A, lda, W, ldw, C, \
                                       ldc, bias, R, ldr, M, N, K, alpha, act)
  if (per <= 4) RDB_SKU(4);
  else if (per <= 8 || UMAX == 8) RDB_SKU(8);
  else RDB_SKU(UMAX);
#undef RDB_SKU
}

template <typename T, typename OutT>
static void launch_sk(const T* A, int lda, const T* W, int ldw, OutT* C, int ldc, const T* bias, const T* R, int ldr,
                      int M, int N, int K, float alpha, int act, hipStream_t s) {
  const int mt = (M + 15) / 16;
  if (mt == 1) launch_sk_mt<T, OutT, 1>(A, lda, W, ldw, C, ldc, bias, R, ldr, M, N, K, alpha, act, s);
  else if (mt == 2) launch_sk_mt<T, OutT, 2>(A, lda, W, ldw, C, ldc, bias, R, ldr, M, N, K, alpha, act, s);
  else if (mt == 3) launch_sk_mt<T, OutT, 3>(A, lda, W, ldw, C, ldc, bias, R, ldr, M, N, K, alpha, act, s);
  else launch_sk_mt<T, OutT, 4>(A, lda, W, ldw, C, ldc, bias, R, ldr, M, N, K, alpha, act, s);
}

bool skinny_gemm_ok(int M, int N, int K, int lda, int ldw, int act, uintptr_t A, uintptr_t W) {
  return M >= 1 && M <= 64 && N >= 1 && K % 32 == 0 && lda % 8 == 0 && ldw % 8 == 0 && act != ACT_SWIGLU &&
         ((A | W) & 15) == 0;
}

// dtype codes: 0 bf16, 1 f16, 2 f32 (output only)
void skinny_gemm(int in_dtype, int out_dtype, uintptr_t A, int lda, uintptr_t W, int ldw, uintptr_t C, int ldc,
                 uintptr_t bias, uintptr_t R, int ldr, int M, int N, int K, float alpha, int act, hipStream_t s) {
  if (in_dtype == 0) {
    auto a = reinterpret_cast<const bf16*>(A);
    auto w = reinterpret_cast<const bf16*>(W);
    auto b = reinterpret_cast<const bf16*>(bias);
    auto r = reinterpret_cast<const bf16*>(R);
    if (out_dtype == 0) launch_sk<bf16, bf16>(a, lda, w, ldw, reinterpret_cast<bf16*>(C), ldc, b, r, ldr, M, N, K, alpha, act, s);
    else if (out_dtype == 2) launch_sk<bf16, float>(a, lda, w, ldw, reinterpret_cast<float*>(C), ldc, b, r, ldr, M, N, K, alpha, act, s);
    else throw std::invalid_argument("skinny_gemm: bad output dtype");
  } else if (in_dtype == 1) {
    auto a = reinterpret_cast<const f16*>(A);
    auto w = reinterpret_cast<const f16*>(W);
    auto b = reinterpret_cast<const f16*>(bias);
    auto r = reinterpret_cast<const f16*>(R);
    if (out_dtype == 1) launch_sk<f16, f16>(a, lda, w, ldw, reinterpret_cast<f16*>(C), ldc, b, r, ldr, M, N, K, alpha, act, s);
    else if (out_dtype == 2) launch_sk<f16, float>(a, lda, w, ldw, reinterpret_cast<float*>(C), ldc, b, r, ldr, M, N, K, alpha, act, s);
    else throw std::invalid_argument("skinny_gemm: bad output dtype");
  } else {
    throw std::invalid_argument("skinny_gemm: bf16 / f16 inputs only");
  }
}

}  // namespace rdb
