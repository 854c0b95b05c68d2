// f16 instantiations of the dense MFMA GEMM (split from gemm.hip so the
// kernel variants compile in parallel).
#include "gemm_core.h"
#include <stdexcept>

namespace rdb {

void gemm_tn_f16(const DenseParams& p, uintptr_t W, int ldw, uintptr_t C, int ldc, uintptr_t bias, uintptr_t R,
          int ldr, int M, int N, int K, float alpha, int act, hipStream_t s, int cfg, int out_dtype) {
  auto w = reinterpret_cast<const f16*>(W);
  auto b = reinterpret_cast<const f16*>(bias);
  auto r = reinterpret_cast<const f16*>(R);
  if (out_dtype == 1)
    launch_mfma_gemm<f16, f16, DenseLoader>(p, w, ldw, reinterpret_cast<f16*>(C), ldc, b, r, ldr, M, N, K, alpha, act, s, cfg);
  else if (out_dtype == 2)
    launch_mfma_gemm<f16, float, DenseLoader>(p, w, ldw, reinterpret_cast<float*>(C), ldc, b, r, ldr, M, N, K, alpha, act, s, cfg);
  else
    throw std::invalid_argument("gemm_tn: output dtype must match the input dtype or be f32");
}

}  // namespace rdb
