// gemm_lab variant set: the shipped ping-pong tiles, built with -D RDB_PP_LATE_PCT=<0|34|50|67> to A/B
// how many of a wave's LDS-DMA pieces per K-tile are issued in the matrix interval (gemm_pp.h).
//   hipcc -O3 --offload-arch=gfx950 -I ray_dynamic_batching_amd/ops/csrc -include bench/gemm_lab/lab_late.h \
//     -D RDB_PP_LATE_PCT=50 bench/gemm_lab/gemm_lab.hip -o labbin/lab_late50
#define LAB_FAST                                                                                                  \
  pp<8, 256, 128, 2, 2, 3, 64>("cfg19 256x128 bk64 s3"), pp<8, 128, 256, 1, 4, 3, 64>("cfg21 128x256 bk64 s3"),     \
  pp<8, 256, 128, 2, 2, 3, 32, 4>("cfg23 256x128 bk32 s3 o4"), pp<8, 256, 192, 2, 2, 4, 32>("cfg25 256x192 bk32 s4"), \
  pp<8, 256, 256, 2, 2, 4, 32>("cfg22 256x256 bk32 s4"),
