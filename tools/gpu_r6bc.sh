#!/bin/bash
# r6b measurements, then the r6c GEMM lab (last: a new kernel)
bash tools/gpu_r6b.sh && bash tools/gpu_r6c.sh
