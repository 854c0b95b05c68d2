// gemm_lab variant set: prefetch depth (LDS stages) of the ping-pong tiles.
//   hipcc -O3 --offload-arch=gfx950 -I ray_dynamic_batching_amd/ops/csrc -include bench/gemm_lab/lab_stages.h \
//     bench/gemm_lab/gemm_lab.hip -o bench/gemm_lab/lab_stages
#define LAB_FAST                                                                              \
  pp<8, 256, 128, 2, 2, 3, 64>("pp8 256x128 bk64 s3"), pp<8, 256, 128, 2, 2, 4, 32>("pp8 256x128 bk32 s4"), \
  pp<8, 256, 128, 2, 2, 5, 32>("pp8 256x128 bk32 s5"), pp<8, 256, 128, 2, 2, 6, 32>("pp8 256x128 bk32 s6"), \
  pp<8, 256, 192, 2, 2, 4, 32>("pp8 256x192 bk32 s4"), pp<8, 256, 192, 2, 2, 5, 32>("pp8 256x192 bk32 s5"), \
  pp<8, 256, 256, 2, 2, 4, 32>("pp8 256x256 bk32 s4"),
