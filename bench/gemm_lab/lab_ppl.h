// gemm_lab variant set: shipped ping-pong tiles vs the loader-wave ping-pong (gemm_ppl.h).
//   hipcc -O3 --offload-arch=gfx950 -I ray_dynamic_batching_amd/ops/csrc -include bench/gemm_lab/lab_ppl.h \
//     bench/gemm_lab/gemm_lab.hip -o labbin/lab_ppl
#include "gemm_core.h"
#include "../../bench/gemm_lab/gemm_ppl.h"
template <int BM, int BN, int GM, int GN, int S, int NL, int BK = 64, int OCC = 3>
struct PplV {
  static void run(const rdb::bf16* A, const rdb::bf16* W, const rdb::bf16* b, rdb::bf16* C, int M, int N, int K,
                  hipStream_t s) {
    rdb::launch_gemm_ppl<rdb::bf16, rdb::bf16, BM, BN, GM, GN, S, NL, BK, OCC>(A, K, W, K, C, N, b, M, N, K, 1.f,
                                                                             rdb::ACT_NONE, s);
  }
};
#define LAB_FAST                                                                                                  \
  pp<8, 256, 128, 2, 2, 3, 64>("cfg19 256x128 bk64 s3"), pp<8, 256, 128, 2, 2, 3, 32, 4>("cfg23 256x128 bk32 o4"), \
  pp<8, 256, 256, 2, 2, 4, 32>("cfg22 256x256 bk32 s4"),                                                          \
  Variant{"ppl 256x128 bk64 s3 L4", PplV<256, 128, 2, 2, 3, 4>::run},                                             \
  Variant{"ppl 256x128 bk64 s3 L2", PplV<256, 128, 2, 2, 3, 2, 64, 3>::run},                                      \
  Variant{"ppl 256x128 bk64 s3 L8", PplV<256, 128, 2, 2, 3, 8, 64, 4>::run},                                      \
  Variant{"ppl 256x256 bk32 s4 L4", PplV<256, 256, 2, 2, 4, 4, 32, 3>::run},
