// Stream-K GEMM entry point (gemm_sk.h): bf16 in / bf16 out, bias, residual,
// activation; the 256 x 128 ping-pong tile at BK = 64 (3 stages) or the
// 128 x 128 tile at BK = 64 (4 stages).  Own translation unit: the header is
// not pulled into gemm_core.h's users.
#include "gemm_core.h"
#if RDB_EXPERIMENTAL
#include "gemm_sk.h"
#endif
#include <stdexcept>
#include <string>

namespace rdb {

#if RDB_EXPERIMENTAL
size_t gemm_sk_workspace_size(int tile, int grid) {
  return tile == 1 ? gemm_sk_workspace_bytes<128, 128>(grid) : gemm_sk_workspace_bytes<256, 128>(grid);
}

void gemm_sk_bf16(uintptr_t A, int lda, uintptr_t W, int ldw, uintptr_t C, int ldc, uintptr_t bias, uintptr_t R,
                  int ldr, int M, int N, int K, float alpha, int act, uintptr_t workspace, int grid, int tile,
                  uintptr_t stream) {
  if (N % 8 || ldc % 8 || (R && ldr % 8) || ((C | R) & 15) || act == ACT_SWIGLU)
    throw std::invalid_argument("gemm_sk: needs N % 8 == 0, 16-B aligned C / residual, no SwiGLU");
  auto s = reinterpret_cast<hipStream_t>(stream);
  const bf16* a = reinterpret_cast<const bf16*>(A);
  const bf16* w = reinterpret_cast<const bf16*>(W);
  bf16* c = reinterpret_cast<bf16*>(C);
  const bf16* b = reinterpret_cast<const bf16*>(bias);
  const bf16* r = reinterpret_cast<const bf16*>(R);
  void* ws = reinterpret_cast<void*>(workspace);
  if (tile == 1)
    launch_gemm_sk<bf16, bf16, 8, 128, 128, 2, 2, 4, 64>(a, lda, w, ldw, c, ldc, b, r, ldr, M, N, K, alpha, act, ws,
                                                         grid, s);
  else
    launch_gemm_sk<bf16, bf16, 8, 256, 128, 2, 2, 3, 64>(a, lda, w, ldw, c, ldc, b, r, ldr, M, N, K, alpha, act, ws,
                                                         grid, s);
  RDB_HIP_CHECK(hipGetLastError());
}
#else
size_t gemm_sk_workspace_size(int, int) { RDB_EXPERIMENTAL_MISSING("gemm_sk"); }
void gemm_sk_bf16(uintptr_t, int, uintptr_t, int, uintptr_t, int, uintptr_t, uintptr_t, int, int, int, int, float, int,
                  uintptr_t, int, int, uintptr_t) {
  RDB_EXPERIMENTAL_MISSING("gemm_sk");
}
#endif

}  // namespace rdb
