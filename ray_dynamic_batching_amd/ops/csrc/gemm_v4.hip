// Dense GEMM on the 4-wave VGPR-staged tiles (gemm_v4.h): tile cfgs 26..28 of
// gemm_core.h (26 = 128 x 96, 27 = 128 x 128, 28 = 256 x 192), bf16 / f16 in and
// out, bias / residual / activation epilogues.  Own translation unit: it is
// compiled with VGPR-form MFMA accumulators (_build.py SRC_FLAGS).
// Experimental build only (RDB_EXPERIMENTAL_KERNELS, common.h): the tiles tied the
// shipped ping-pong choice in the two-stream BERT engine (profiles/ab_r5_v4_bert.json)
// and no shipped table uses them, so the default library does not carry them.
#include "gemm_core.h"
#if RDB_EXPERIMENTAL
#include "gemm_v4.h"
#endif
#include <stdexcept>

namespace rdb {

#if RDB_EXPERIMENTAL

template <typename T>
static void v4_dispatch(int cfg, const T* A, int lda, const T* W, int ldw, T* C, int ldc, const T* bias, const T* R,
                        int ldr, int M, int N, int K, float alpha, int act, hipStream_t s) {
  switch (cfg) {
    case 26: launch_gemm_v4<T, T, 128, 96>(A, lda, W, ldw, C, ldc, bias, R, ldr, M, N, K, alpha, act, s); return;
    case 27: launch_gemm_v4<T, T, 128, 128>(A, lda, W, ldw, C, ldc, bias, R, ldr, M, N, K, alpha, act, s); return;
    case 28: launch_gemm_v4<T, T, 256, 192>(A, lda, W, ldw, C, ldc, bias, R, ldr, M, N, K, alpha, act, s); return;
    default: throw std::invalid_argument("gemm_v4: tile cfg must be 26..28");
  }
}

void launch_gemm_v4_cfg(int cfg, int dtype, const void* A, int lda, const void* W, int ldw, void* C, int ldc,
                        const void* bias, const void* R, int ldr, int M, int N, int K, float alpha, int act,
                        hipStream_t s) {
  // the staged epilogue here is the plain one: SwiGLU pairing lives in the ping-pong / 4-wave kernels
  if (act == ACT_SWIGLU) throw std::invalid_argument("gemm_v4: no SwiGLU epilogue on tile cfgs 26..28");
  if (K % 64 != 0) throw std::invalid_argument("gemm_v4: K must be a multiple of 64");
  if (dtype == 0)
    v4_dispatch<bf16>(cfg, static_cast<const bf16*>(A), lda, static_cast<const bf16*>(W), ldw, static_cast<bf16*>(C),
                      ldc, static_cast<const bf16*>(bias), static_cast<const bf16*>(R), ldr, M, N, K, alpha, act, s);
  else
    v4_dispatch<f16>(cfg, static_cast<const f16*>(A), lda, static_cast<const f16*>(W), ldw, static_cast<f16*>(C), ldc,
                     static_cast<const f16*>(bias), static_cast<const f16*>(R), ldr, M, N, K, alpha, act, s);
}
#else
void launch_gemm_v4_cfg(int, int, const void*, int, const void*, int, void*, int, const void*, const void*, int, int,
                        int, int, float, int, hipStream_t) {
  RDB_EXPERIMENTAL_MISSING("gemm_v4 tiles 26..28");
}
#endif

}  // namespace rdb
