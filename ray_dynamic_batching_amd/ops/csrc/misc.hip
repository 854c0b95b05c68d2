// Small fused kernels for the serving path on gfx950:
//   * softmax_topk   - classification head: row softmax fused with top-k
//                      (ResNet-50 Serve workload: softmax + argmax)
//   * rope           - in-place rotary embedding on the packed QKV buffer (Llama)
//   * gather_rows    - batch formation on the device: copies request payloads
//                      straight out of host-mapped (pinned shm) ring slots into
//                      the padded device input, zero-filling pad rows.  This is
//                      the H2D step of the replica engine, run on a side stream.
//   * image_to_nhwc  - uint8 HWC images -> normalised f16 NHWC model input.
#include "common.h"
#include <algorithm>
#include <stdexcept>

namespace rdb {

// One wave per row, one row per 64-thread workgroup (so a 32-row batch runs on
// 32 CUs, not 8), C <= 4096, k <= 16.  Each lane holds NV float4 of the row
// (16-B loads when C % 4 == 0 and the rows are 16-B aligned, else element
// loads): C = 1000 is 4 float4 per lane instead of the 64 scalar registers a
// fixed 4096-wide layout scans per top-k pass.
template <int NV, bool VEC>
__global__ void __launch_bounds__(64)
softmax_topk_kernel(const float* __restrict__ x, int rows, int C, int k, float* __restrict__ probs,
                    int* __restrict__ idx) {
  const int lane = threadIdx.x;
  const int row = blockIdx.x;
  const float* xr = x + (size_t)row * C;
  // element e of this lane: column 4 * (lane + 64 * (e / 4)) + e % 4
  float v[NV * 4];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c0 = 4 * (lane + 64 * i);
    if constexpr (VEC) {
      f32x4 q = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
      if (c0 < C) q = *reinterpret_cast<const f32x4*>(xr + c0);   // C % 4 == 0: whole vector in range
#pragma unroll
      for (int e = 0; e < 4; ++e) v[4 * i + e] = q[e];
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) v[4 * i + e] = c0 + e < C ? xr[c0 + e] : -INFINITY;
    }
  }
  float mx = -INFINITY;
#pragma unroll
  for (int e = 0; e < NV * 4; ++e) mx = fmaxf(mx, v[e]);
  mx = wave_max(mx);
  float s = 0.f;
#pragma unroll
  for (int e = 0; e < NV * 4; ++e) s += __expf(v[e] - mx);   // exp(-inf) = 0 for the padding
  s = wave_sum(s);
  const float inv = 1.f / s;
  for (int t = 0; t < k; ++t) {
    float best = -INFINITY;
    int bi = 0x7fffffff;
#pragma unroll
    for (int e = 0; e < NV * 4; ++e) {
      const int c = 4 * (lane + 64 * (e >> 2)) + (e & 3);
      if (v[e] > best) { best = v[e]; bi = c; }   // ascending c per lane: the first max wins ties
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ob = __shfl_xor(best, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      if (ob > best || (ob == best && oi < bi)) { best = ob; bi = oi; }
    }
    if (lane == 0) {
      if (idx != nullptr) {
        probs[(size_t)row * k + t] = __expf(best - mx) * inv;
        idx[(size_t)row * k + t] = bi < C ? bi : -1;
      } else {   // packed serving output: row = [k probabilities | k class ids as f32]
        probs[(size_t)row * 2 * k + t] = __expf(best - mx) * inv;
        probs[(size_t)row * 2 * k + k + t] = (float)(bi < C ? bi : -1);
      }
    }
#pragma unroll
    for (int e = 0; e < NV * 4; ++e)
      if (4 * (lane + 64 * (e >> 2)) + (e & 3) == bi) v[e] = -INFINITY;   // remove the winner
  }
}

template <int NV>
static void launch_softmax_topk(const float* x, int rows, int C, int k, float* probs, int* idx, hipStream_t st) {
  const bool vec = (C & 3) == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0;
  if (vec)
    hipLaunchKernelGGL((softmax_topk_kernel<NV, true>), dim3(rows), dim3(64), 0, st, x, rows, C, k, probs, idx);
  else
    hipLaunchKernelGGL((softmax_topk_kernel<NV, false>), dim3(rows), dim3(64), 0, st, x, rows, C, k, probs, idx);
}

void softmax_topk(uintptr_t x, int rows, int C, int k, uintptr_t probs, uintptr_t idx, uintptr_t stream) {
  if (C > 4096 || k < 1 || k > 16 || k > C) throw std::invalid_argument("softmax_topk: need C <= 4096, 1 <= k <= min(16, C)");
  if (rows <= 0) return;
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const float* xp = (const float*)x;
  float* pp = (float*)probs;
  int* ip = (int*)idx;
  const int nv = (C + 255) / 256;   // float4 per lane
  if (nv <= 1) launch_softmax_topk<1>(xp, rows, C, k, pp, ip, st);
  else if (nv <= 2) launch_softmax_topk<2>(xp, rows, C, k, pp, ip, st);
  else if (nv <= 4) launch_softmax_topk<4>(xp, rows, C, k, pp, ip, st);
  else if (nv <= 8) launch_softmax_topk<8>(xp, rows, C, k, pp, ip, st);
  else launch_softmax_topk<16>(xp, rows, C, k, pp, ip, st);
  RDB_HIP_CHECK(hipGetLastError());
}

// Rotary embedding (HF "rotate_half" convention) on Q and K heads of the packed
// [T, ld] projection output.  cos/sin tables are [max_pos, D/2] f32 built on the
// host (Appendix B: precomputed trig tables).  One thread per (token, head, i<D/2).
__global__ void rope_kernel(bf16* __restrict__ qkv, int ld, int q_off, int k_off, int H, int Hkv,
                            int D, int S, const float* __restrict__ cos_t,
                            const float* __restrict__ sin_t, int T, int pos_offset) {
  const int half = D >> 1;
  const long total = (long)T * (H + Hkv) * half;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const int i = e % half;
    const long r = e / half;
    const int hh = r % (H + Hkv);
    const int t = r / (H + Hkv);
    const int pos = t % S + pos_offset;
    bf16* base = qkv + (size_t)t * ld + (hh < H ? q_off + hh * D : k_off + (hh - H) * D);
    const float c = cos_t[pos * half + i], s = sin_t[pos * half + i];
    const float x1 = (float)base[i], x2 = (float)base[i + half];
    base[i] = (bf16)(x1 * c - x2 * s);
    base[i + half] = (bf16)(x2 * c + x1 * s);
  }
}

void rope(uintptr_t qkv, int ld, int q_off, int k_off, int H, int Hkv, int D, int S, uintptr_t cos_t,
          uintptr_t sin_t, int T, int pos_offset, uintptr_t stream) {
  if (T <= 0) return;
  const long total = (long)T * (H + Hkv) * (D / 2);
  int blocks = (int)((total + 255) / 256);
  blocks = blocks > 4096 ? 4096 : blocks;
  hipLaunchKernelGGL(rope_kernel, dim3(blocks), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     (bf16*)qkv, ld, q_off, k_off, H, Hkv, D, S, (const float*)cos_t,
                     (const float*)sin_t, T, pos_offset);
  RDB_HIP_CHECK(hipGetLastError());
}

// dst[r, :] = src_ptrs[r][0:row_bytes) for r < n, zeros for n <= r < rows.
// src_ptrs lives in pinned host memory and the payloads in hipHostRegister'ed
// (device-mapped) shared memory, so this one kernel replaces n hipMemcpyAsync's.
__global__ void __launch_bounds__(256)
gather_rows_kernel(const uint64_t* __restrict__ src_ptrs, int n, int rows, int row_bytes,
                   char* __restrict__ dst) {
  const int r = blockIdx.x;
  char* d = dst + (size_t)r * row_bytes;
  const int nvec = row_bytes >> 4;
  if (r < n) {
    const char* s = reinterpret_cast<const char*>(src_ptrs[r]);
    for (int i = threadIdx.x; i < nvec; i += blockDim.x)
      reinterpret_cast<u32x4*>(d)[i] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(s) + i);
    for (int i = (nvec << 4) + threadIdx.x; i < row_bytes; i += blockDim.x) d[i] = s[i];
  } else {
    for (int i = threadIdx.x; i < nvec; i += blockDim.x) reinterpret_cast<u32x4*>(d)[i] = u32x4{0, 0, 0, 0};
    for (int i = (nvec << 4) + threadIdx.x; i < row_bytes; i += blockDim.x) d[i] = 0;
  }
}

void gather_rows(uintptr_t src_ptrs, int n, int rows, int row_bytes, uintptr_t dst, uintptr_t stream) {
  if (rows <= 0) return;
  if (row_bytes % 16 != 0) throw std::invalid_argument("gather_rows: row_bytes must be a multiple of 16");
  hipLaunchKernelGGL(gather_rows_kernel, dim3(rows), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     (const uint64_t*)src_ptrs, n, rows, row_bytes, (char*)dst);
  RDB_HIP_CHECK(hipGetLastError());
}

// uint8 HWC (RGB) -> f16 NHWC normalised with per-channel mean/std, C padded to Cp
// (Cp = 4 keeps the first conv's channel dim 8-byte aligned; pad channels are 0).
__global__ void image_to_nhwc_kernel(const uint8_t* __restrict__ src, int N, int HW, int Cp,
                                     float m0, float m1, float m2, float s0, float s1, float s2,
                                     f16* __restrict__ dst) {
  const long total = (long)N * HW;
  for (long p = blockIdx.x * (long)blockDim.x + threadIdx.x; p < total; p += (long)gridDim.x * blockDim.x) {
    const uint8_t* s = src + p * 3;
    f16* d = dst + p * Cp;
    d[0] = (f16)((s[0] * (1.f / 255.f) - m0) / s0);
    d[1] = (f16)((s[1] * (1.f / 255.f) - m1) / s1);
    d[2] = (f16)((s[2] * (1.f / 255.f) - m2) / s2);
    for (int c = 3; c < Cp; ++c) d[c] = (f16)0.f;
  }
}

void image_to_nhwc(uintptr_t src, int N, int HW, int Cp, uintptr_t dst, uintptr_t stream) {
  if (N <= 0) return;
  const long total = (long)N * HW;
  int blocks = (int)((total + 255) / 256);
  blocks = blocks > 8192 ? 8192 : blocks;
  hipLaunchKernelGGL(image_to_nhwc_kernel, dim3(blocks), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     (const uint8_t*)src, N, HW, Cp, 0.485f, 0.456f, 0.406f, 0.229f, 0.224f, 0.225f,
                     (f16*)dst);
  RDB_HIP_CHECK(hipGetLastError());
}

// uint8 HWC (RGB) -> normalised f16 SPACE-TO-DEPTH [N, H/2, W/2, 16]: channel
// (dy*2 + dx)*3 + c of output pixel (i, j) is input pixel (2i+dy, 2j+dx) channel c,
// channels 12..15 are zero.  A 7x7 stride-2 stem conv on the image is then a 4x4
// stride-1 conv on this tensor (ResNet50.stem_w_s2d): 256 reduction elements per
// output instead of 7*7*8 = 392 with the channel-padded layout.  Optionally
// zeroes `zero_bytes` at `zero` (the forward's split-K counters) on the side.
__global__ void image_to_s2d_kernel(const uint8_t* __restrict__ src, int N, int H, int W,
                                    float m0, float m1, float m2, float s0, float s1, float s2,
                                    f16* __restrict__ dst, u32x4* __restrict__ zero, int zero_n) {
  // side job: zero a split-K counter header for the forward this kernel starts
  {
    const long z = blockIdx.x * (long)blockDim.x + threadIdx.x;
    if (z < zero_n) zero[z] = u32x4{0u, 0u, 0u, 0u};
  }
  const int P = H >> 1, Q2 = W >> 2;          // a thread makes output pixels (i, 2j) and (i, 2j + 1)
  const long total = (long)N * P * Q2;
  const float a[3] = {1.f / (255.f * s0), 1.f / (255.f * s1), 1.f / (255.f * s2)};
  const float b[3] = {-m0 / s0, -m1 / s1, -m2 / s2};
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const int j = e % Q2;
    const long ni = e / Q2;
    const int i = ni % P;
    const int n = ni / P;
    // 12 input bytes per row (4 pixels x RGB), three aligned dword loads (W % 4 == 0)
    uint32_t raw[2][3];
#pragma unroll
    for (int dy = 0; dy < 2; ++dy) {
      const uint32_t* r = reinterpret_cast<const uint32_t*>(src + (((size_t)n * H + 2 * i + dy) * W + 4 * j) * 3);
#pragma unroll
      for (int t = 0; t < 3; ++t) raw[dy][t] = r[t];
    }
    f16x8 o[4];   // pixel 2j: o[0], o[1]; pixel 2j + 1: o[2], o[3]
#pragma unroll
    for (int px = 0; px < 2; ++px) {
#pragma unroll
      for (int dy = 0; dy < 2; ++dy) {
#pragma unroll
        for (int t = 0; t < 6; ++t) {           // (dx, c) = (t / 3, t % 3): byte 6 px + t of the row
          const int byte = 6 * px + t;
          const float u = (float)((raw[dy][byte >> 2] >> (8 * (byte & 3))) & 0xffu);
          const int ch = dy * 6 + t;
          o[2 * px + (ch >> 3)][ch & 7] = (f16)(u * a[t % 3] + b[t % 3]);
        }
      }
#pragma unroll
      for (int c = 4; c < 8; ++c) o[2 * px + 1][c] = (f16)0.f;
    }
    f16x8* d = reinterpret_cast<f16x8*>(dst + (size_t)(ni * (W >> 1) + 2 * j) * 16);
#pragma unroll
    for (int q = 0; q < 4; ++q) d[q] = o[q];
  }
}

void image_to_s2d(uintptr_t src, int N, int H, int W, uintptr_t dst, uintptr_t zero, long zero_bytes,
                  uintptr_t stream) {
  if (N <= 0) return;
  if ((H & 1) || (W & 3)) throw std::invalid_argument("image_to_s2d: H must be even and W a multiple of 4");
  if ((src & 3) || (dst & 15) || (zero & 15) || (zero_bytes & 15))
    throw std::invalid_argument("image_to_s2d: src 4-byte, dst / zero 16-byte aligned; zero_bytes % 16 == 0");
  const long total = (long)N * (H / 2) * (W / 4);
  const long zn = zero ? zero_bytes / 16 : 0;
  long blocks = (std::max(total, zn) + 255) / 256;
  blocks = blocks > 8192 ? std::max<long>(8192, (zn + 255) / 256) : blocks;
  hipLaunchKernelGGL(image_to_s2d_kernel, dim3((unsigned)blocks), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     (const uint8_t*)src, N, H, W, 0.485f, 0.456f, 0.406f, 0.229f, 0.224f, 0.225f, (f16*)dst,
                     (u32x4*)zero, (int)zn);
  RDB_HIP_CHECK(hipGetLastError());
}

// Per-sequence valid length = number of non-pad token ids (BERT key-padding
// mask for the attention kernel): one wave per sequence, one launch.
__global__ void __launch_bounds__(64) seq_lens_kernel(const int* __restrict__ ids, int S, int pad, int* __restrict__ lens) {
  const int b = blockIdx.x;
  int c = 0;
  for (int t = threadIdx.x; t < S; t += 64) c += ids[(size_t)b * S + t] != pad;
  const float tot = wave_sum((float)c);
  if (threadIdx.x == 0) lens[b] = max(1, (int)tot);
}

void seq_lens(uintptr_t ids, int B, int S, int pad, uintptr_t lens, uintptr_t stream) {
  if (B <= 0) return;
  hipLaunchKernelGGL(seq_lens_kernel, dim3(B), dim3(64), 0, reinterpret_cast<hipStream_t>(stream),
                     reinterpret_cast<const int*>(ids), S, pad, reinterpret_cast<int*>(lens));
  RDB_HIP_CHECK(hipGetLastError());
}

}  // namespace rdb
