// gemm_lab variant set: ping-pong tiles with LDS-DMA staging (pp) vs register staging (vs, gemm_ppvs.h).
//   hipcc -O3 --offload-arch=gfx950 -I ray_dynamic_batching_amd/ops/csrc -include bench/gemm_lab/lab_vs.h \
//     bench/gemm_lab/gemm_lab.hip -o labbin/lab_vs
#include "../../bench/gemm_lab/gemm_ppvs.h"
#define LAB_VS(NM, BM, BN, GM, GN, BK, OCC)                                                                           \
  Variant{NM, [](const bf16* A, const bf16* W, const bf16* b, bf16* C, int M, int N, int K, hipStream_t s) {          \
            rdb::vs::launch_ppvs<bf16, bf16, 8, BM, BN, GM, GN, BK, OCC>(A, K, W, K, C, N, b, nullptr, 0, M, N, K, 1.f, \
                                                                          ACT_NONE, s);                                \
          }}
#define LAB_FAST                                                                                                   \
  pp<8, 256, 128, 2, 2, 3, 64>("pp cfg19 256x128 bk64"), LAB_VS("vs 256x128 bk64", 256, 128, 2, 2, 64, 2),         \
  pp<8, 128, 256, 1, 4, 3, 64>("pp cfg21 128x256 bk64"), LAB_VS("vs 128x256 bk64", 128, 256, 1, 4, 64, 2),         \
  pp<8, 256, 256, 2, 2, 4, 32>("pp cfg22 256x256 bk32 s4"), LAB_VS("vs 256x256 bk32", 256, 256, 2, 2, 32, 2),     \
  pp<8, 256, 128, 2, 2, 3, 32, 4>("pp cfg23 256x128 bk32 o4"), LAB_VS("vs 256x128 bk32 o4", 256, 128, 2, 2, 32, 4),
