// bf16 instantiations of the dense MFMA GEMM (split from gemm.hip so the
// kernel variants compile in parallel).
#include "gemm_core.h"
#include <stdexcept>

namespace rdb {

// f32-output instantiations live in gemm_bf16_f32.hip (a separate translation
// unit: the template instantiations dominate the build, two TUs compile in parallel)
void gemm_tn_bf16_f32out(const DenseParams& p, uintptr_t W, int ldw, uintptr_t C, int ldc, uintptr_t bias, uintptr_t R,
                        int ldr, int M, int N, int K, float alpha, int act, hipStream_t s, int cfg);

void gemm_tn_bf16(const DenseParams& p, uintptr_t W, int ldw, uintptr_t C, int ldc, uintptr_t bias, uintptr_t R,
          int ldr, int M, int N, int K, float alpha, int act, hipStream_t s, int cfg, int out_dtype,
          const LnEpi& sk) {
  auto w = reinterpret_cast<const bf16*>(W);
  auto b = reinterpret_cast<const bf16*>(bias);
  auto r = reinterpret_cast<const bf16*>(R);
  if (out_dtype == 0)
    launch_mfma_gemm<bf16, bf16, DenseLoader>(p, w, ldw, reinterpret_cast<bf16*>(C), ldc, b, r, ldr, M, N, K, alpha, act, s, cfg,
                                         sk);
  else if (out_dtype == 2)
    gemm_tn_bf16_f32out(p, W, ldw, C, ldc, bias, R, ldr, M, N, K, alpha, act, s, cfg & 255);
  else
    throw std::invalid_argument("gemm_tn: output dtype must match the input dtype or be f32");
}

}  // namespace rdb
