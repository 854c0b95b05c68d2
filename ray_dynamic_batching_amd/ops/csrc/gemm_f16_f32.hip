// f16 -> f32-output instantiations of the dense MFMA GEMM (split from
// gemm_f16.hip so the two halves of the template instantiations compile in parallel).
#include "gemm_core.h"

namespace rdb {

void gemm_tn_f16_f32out(const DenseParams& p, uintptr_t W, int ldw, uintptr_t C, int ldc, uintptr_t bias, uintptr_t R,
                        int ldr, int M, int N, int K, float alpha, int act, hipStream_t s, int cfg) {
  launch_mfma_gemm<f16, float, DenseLoader>(p, reinterpret_cast<const f16*>(W), ldw, reinterpret_cast<float*>(C), ldc,
                                            reinterpret_cast<const f16*>(bias), reinterpret_cast<const f16*>(R), ldr,
                                            M, N, K, alpha, act, s, cfg);
}

}  // namespace rdb
