// Dense MFMA GEMM with fused epilogue (gfx950).  Kernel body: gemm_core.h.
//
//   C[m, n] = act(alpha * sum_k A[m, k] * W[n, k] + bias[n] + R[m, n])
//
// A is [M, K] (row stride lda), W is [N, K] (nn.Linear layout, row stride ldw).
// The op behind every projection of the batched forward pass (SURVEY.md §2.7:
// BERT QKV / out / FFN GEMMs with bias/GELU/residual epilogues, pooler tanh,
// ResNet FC, Llama SwiGLU gate/up pair).
#include "gemm_core.h"
#include <stdexcept>

namespace rdb {

void gemm_tn_bf16(const DenseParams& p, uintptr_t W, int ldw, uintptr_t C, int ldc, uintptr_t bias, uintptr_t R,
                  int ldr, int M, int N, int K, float alpha, int act, hipStream_t s, int cfg, int out_dtype,
                  const LnEpi& sk);
void gemm_tn_f16(const DenseParams& p, uintptr_t W, int ldw, uintptr_t C, int ldc, uintptr_t bias, uintptr_t R,
                 int ldr, int M, int N, int K, float alpha, int act, hipStream_t s, int cfg, int out_dtype,
                 const LnEpi& sk);

bool skinny_gemm_ok(int M, int N, int K, int lda, int ldw, int act, uintptr_t A, uintptr_t W);
void skinny_gemm(int in_dtype, int out_dtype, uintptr_t A, int lda, uintptr_t W, int ldw, uintptr_t C, int ldc,
                 uintptr_t bias, uintptr_t R, int ldr, int M, int N, int K, float alpha, int act, hipStream_t s);
constexpr int kForceTiled = 99;  // force_cfg value that bypasses the skinny-M kernel (tests)

void gemm_tn_sk(int in_dtype, int out_dtype, uintptr_t A, int lda, uintptr_t W, int ldw, uintptr_t C,
                int ldc, uintptr_t bias, uintptr_t R, int ldr, int M, int N, int K, float alpha,
                int act, uintptr_t stream, int force_cfg, uintptr_t ws, size_t ws_bytes);

// dtype codes shared with the Python side: 0 = bf16, 1 = f16, 2 = f32
void gemm_tn(int in_dtype, int out_dtype, uintptr_t A, int lda, uintptr_t W, int ldw, uintptr_t C,
             int ldc, uintptr_t bias, uintptr_t R, int ldr, int M, int N, int K, float alpha,
             int act, uintptr_t stream, int force_cfg) {
  gemm_tn_sk(in_dtype, out_dtype, A, lda, W, ldw, C, ldc, bias, R, ldr, M, N, K, alpha, act, stream, force_cfg, 0, 0);
}

// force_cfg = tile | (splits << 8) [| kDeepFlag]: splits > 1 runs split-K (4-wave tiles, 16-bit output, no
// SwiGLU) on the workspace ``ws`` (zeroed counter header; see splitk_bytes) when it fits, else unsplit
void gemm_tn_sk(int in_dtype, int out_dtype, uintptr_t A, int lda, uintptr_t W, int ldw, uintptr_t C,
                int ldc, uintptr_t bias, uintptr_t R, int ldr, int M, int N, int K, float alpha,
                int act, uintptr_t stream, int force_cfg, uintptr_t ws, size_t ws_bytes) {
  if (K % 8 != 0) throw std::invalid_argument("gemm_tn: K must be a multiple of 8");
  if (lda % 8 != 0 || ldw % 8 != 0) throw std::invalid_argument("gemm_tn: lda/ldw must be multiples of 8");
  if ((A | W) & 15) throw std::invalid_argument("gemm_tn: A/W must be 16-byte aligned");
  if (act == ACT_SWIGLU && N % 4 != 0) throw std::invalid_argument("gemm_tn: SWIGLU needs N % 4 == 0");
  if (M <= 0 || N <= 0 || K <= 0) return;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (force_cfg != kForceTiled && skinny_gemm_ok(M, N, K, lda, ldw, act, A, W)) {
    skinny_gemm(in_dtype, out_dtype, A, lda, W, ldw, C, ldc, bias, R, ldr, M, N, K, alpha, act, s);
    RDB_HIP_CHECK(hipGetLastError());
    return;
  }
  if (force_cfg == kForceTiled) force_cfg = -1;
  LnEpi sk{};
  if (force_cfg >= 0) {
    const int splits = (force_cfg >> 8) & 15;
    if (splits > 1 && out_dtype != 2 && act != ACT_SWIGLU)
      sk = splitk_epi(M, N, K, force_cfg & 255, splits, reinterpret_cast<void*>(ws), ws_bytes);
    force_cfg &= 255 | kDeepFlag;
  }
  DenseParams p{reinterpret_cast<const void*>(A), lda, M, K};
  if (in_dtype == 0) {
    gemm_tn_bf16(p, W, ldw, C, ldc, bias, R, ldr, M, N, K, alpha, act, s, force_cfg, out_dtype, sk);
  } else if (in_dtype == 1) {
    gemm_tn_f16(p, W, ldw, C, ldc, bias, R, ldr, M, N, K, alpha, act, s, force_cfg, out_dtype, sk);
  } else {
    throw std::invalid_argument("gemm_tn: unsupported input dtype");
  }
  RDB_HIP_CHECK(hipGetLastError());
}

}  // namespace rdb
