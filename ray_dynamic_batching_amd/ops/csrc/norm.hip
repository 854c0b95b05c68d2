// Row normalisation kernels for gfx950: LayerNorm (+ fused residual add),
// RMSNorm (+ fused residual add) and the BERT embedding gather fused with its
// LayerNorm.  Memory-bound ops: one wave per row, 8-byte (4 x 16-bit) vector
// loads per lane (cdna_hip_programming.md Guideline 13), the row is kept in
// registers between the statistics pass and the output pass, so each element
// is read from HBM exactly once.
#include "common.h"
#include <cstdlib>
#include <stdexcept>

namespace rdb {

constexpr int kMaxVec = 32;  // 32 x 4 elements x 64 lanes = rows up to 8192
// NV = D / 256 is a template parameter so the row lives in exactly NV*4 VGPRs.

template <typename T>
__device__ __forceinline__ void load4(const T* p, float* o) {
  typedef T v4 __attribute__((ext_vector_type(4)));
  v4 v = *reinterpret_cast<const v4*>(p);
  o[0] = (float)v[0]; o[1] = (float)v[1]; o[2] = (float)v[2]; o[3] = (float)v[3];
}
template <typename T>
__device__ __forceinline__ void st4(T* p, const float* o) {
  typedef T v4 __attribute__((ext_vector_type(4)));
  v4 v = {(T)o[0], (T)o[1], (T)o[2], (T)o[3]};
  *reinterpret_cast<v4*>(p) = v;
}

// MODE 0 = LayerNorm, 1 = RMSNorm.
template <typename T, int MODE, int NV>
__global__ void __launch_bounds__(256)
norm_kernel(const T* __restrict__ x, const T* __restrict__ res, T* __restrict__ res_out,
            const T* __restrict__ gamma, const T* __restrict__ beta, T* __restrict__ y,
            int rows, int D, int ldx, float eps) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const T* xr = x + (size_t)row * ldx;  // x may be a row-strided view (e.g. the [CLS] rows)
  float v[NV][4];
  float gv[NV][4], bv[NV][4];
  // gamma/beta are issued with the row loads so their latency overlaps the
  // reductions instead of following them
  // rows need not be a multiple of 256: lanes past D (last vector only) hold
  // zeros, are excluded from the variance and are not stored
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = i * 256 + lane * 4;
    if (c < D) {
      load4(xr + c, v[i]);
      load4(gamma + c, gv[i]);
      if (MODE == 0) load4(beta + c, bv[i]);
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) v[i][e] = gv[i][e] = bv[i][e] = 0.f;
    }
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    {
      const int c = i * 256 + lane * 4;
      if (res != nullptr && c < D) {
        float r[4];
        load4(res + (size_t)row * D + c, r);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[i][e] += r[e];
        if (res_out != nullptr) st4(res_out + (size_t)row * D + c, v[i]);
      }
      if (MODE == 0) s += v[i][0] + v[i][1] + v[i][2] + v[i][3];
      else s += v[i][0] * v[i][0] + v[i][1] * v[i][1] + v[i][2] * v[i][2] + v[i][3] * v[i][3];
    }
  }
  s = wave_sum(s);
  float mean = 0.f, rstd;
  if (MODE == 0) {
    mean = s / D;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      if (i * 256 + lane * 4 >= D) continue;
#pragma unroll
      for (int e = 0; e < 4; ++e) { const float d = v[i][e] - mean; q += d * d; }
    }
    q = wave_sum(q);
    rstd = rsqrtf(q / D + eps);
  } else {
    rstd = rsqrtf(s / D + eps);
  }
  T* yr = y + (size_t)row * D;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    {
      const int c = i * 256 + lane * 4;
      float o[4];
      if (MODE == 0) {
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = (v[i][e] - mean) * rstd * gv[i][e] + bv[i][e];
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = v[i][e] * rstd * gv[i][e];
      }
      if (c < D) st4(yr + c, o);
    }
  }
}

// Half-wave-per-row form for rows of 256 * NV16 elements with 16-B aligned
// operands (the transformer hidden sizes: 768 = 3 x 256, 1024, 4096): 32 lanes
// own a row, each lane NV16 16-B vectors (8 elements), so every load / store
// instruction moves 512 B of ONE row and a wave keeps two rows in flight; the
// row reductions stay inside the half wave (xor 1..16: DPP / swizzle, no
// cross-half ds_bpermute).  Two passes (mean, then centered variance) over the
// register-resident row.  Measured against norm_kernel: bench/launch_floor.py.
template <typename T>
__device__ __forceinline__ void load8(const T* p, float* o) {
  const u32x4 raw = *reinterpret_cast<const u32x4*>(p);
  const T* e = reinterpret_cast<const T*>(&raw);
#pragma unroll
  for (int q = 0; q < 8; ++q) o[q] = (float)e[q];
}
template <typename T>
__device__ __forceinline__ void st8(T* p, const float* o) {
  T v[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) v[q] = (T)o[q];
  *reinterpret_cast<u32x4*>(p) = *reinterpret_cast<const u32x4*>(v);
}
__device__ __forceinline__ float half_sum(float v) {
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <typename T, int MODE, int NV16>
__global__ void __launch_bounds__(256)
norm16_kernel(const T* __restrict__ x, const T* __restrict__ res, T* __restrict__ res_out,
              const T* __restrict__ gamma, const T* __restrict__ beta, T* __restrict__ y, int rows, int ldx,
              float eps) {
  constexpr int D = 256 * NV16;
  const int hl = threadIdx.x & 31;
  // grid-stride over 8-row groups: a capped grid (RDB_LN_BLOCKS) leaves CUs to a
  // concurrently running kernel of another stream instead of flooding the dispatcher
  const int rpb = blockDim.x >> 5;             // rows per block (half-wave per row)
  for (int row = blockIdx.x * rpb + (threadIdx.x >> 5); row < rows; row += gridDim.x * rpb) {
  const T* xr = x + (size_t)row * ldx;
  float v[NV16][8];
#pragma unroll
  for (int i = 0; i < NV16; ++i) load8(xr + i * 256 + hl * 8, v[i]);
  if (res != nullptr) {
#pragma unroll
    for (int i = 0; i < NV16; ++i) {
      float r[8];
      load8(res + (size_t)row * D + i * 256 + hl * 8, r);
#pragma unroll
      for (int q = 0; q < 8; ++q) v[i][q] += r[q];
      if (res_out != nullptr) st8(res_out + (size_t)row * D + i * 256 + hl * 8, v[i]);
    }
  }
  float mean = 0.f, rstd;
  if constexpr (MODE == 0) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NV16; ++i)
#pragma unroll
      for (int q = 0; q < 8; ++q) s += v[i][q];
    mean = half_sum(s) * (1.0f / D);
    float qs = 0.f;
#pragma unroll
    for (int i = 0; i < NV16; ++i)
#pragma unroll
      for (int q = 0; q < 8; ++q) { const float d = v[i][q] - mean; qs += d * d; }
    rstd = rsqrtf(half_sum(qs) * (1.0f / D) + eps);
  } else {
    float qs = 0.f;
#pragma unroll
    for (int i = 0; i < NV16; ++i)
#pragma unroll
      for (int q = 0; q < 8; ++q) qs += v[i][q] * v[i][q];
    rstd = rsqrtf(half_sum(qs) * (1.0f / D) + eps);
  }
  T* yr = y + (size_t)row * D;
#pragma unroll
  for (int i = 0; i < NV16; ++i) {
    const int c = i * 256 + hl * 8;
    float g[8], b[8], o[8];
    load8(gamma + c, g);
    if constexpr (MODE == 0) load8(beta + c, b);
#pragma unroll
    for (int q = 0; q < 8; ++q) o[q] = MODE == 0 ? (v[i][q] - mean) * rstd * g[q] + b[q] : v[i][q] * rstd * g[q];
    st8(yr + c, o);
  }
  }
}

// BERT embeddings: y[t] = LN(word[ids[t]] + pos[t % S] + type[types ? types[t] : 0])
template <typename T, int NV>
__global__ void __launch_bounds__(256)
embed_ln_kernel(const int* __restrict__ ids, const int* __restrict__ types,
                const T* __restrict__ word, const T* __restrict__ pos, const T* __restrict__ typ,
                const T* __restrict__ gamma, const T* __restrict__ beta, T* __restrict__ y,
                int tokens, int S, int D, int vocab, float eps, float2* __restrict__ zst, int zn,
                int zstride) {
  const int lane = threadIdx.x & 63;
  const int t = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (t >= tokens) return;
  // zero this token's deferred-LayerNorm row statistics of every layer (the
  // folded forward's accumulators; models/bert.py fold_ln): saves a fill kernel
  for (int k = lane; k < zn; k += 64) zst[(size_t)k * zstride + t] = float2{0.f, 0.f};
  int id = ids[t];
  id = id < 0 ? 0 : (id >= vocab ? vocab - 1 : id);
  const int tt = types ? types[t] : 0;
  const int p = t % S;
  float v[NV][4];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    {
      const int c = i * 256 + lane * 4;
      float a[4], b[4], d[4];
      load4(word + (size_t)id * D + c, a);
      load4(pos + (size_t)p * D + c, b);
      load4(typ + (size_t)tt * D + c, d);
#pragma unroll
      for (int e = 0; e < 4; ++e) { v[i][e] = a[e] + b[e] + d[e]; s += v[i][e]; }
    }
  }
  const float mean = wave_sum(s) / D;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) { const float d = v[i][e] - mean; q += d * d; }
  const float rstd = rsqrtf(wave_sum(q) / D + eps);
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    {
      const int c = i * 256 + lane * 4;
      float g[4], b[4], o[4];
      load4(gamma + c, g);
      load4(beta + c, b);
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = (v[i][e] - mean) * rstd * g[e] + b[e];
      st4(y + (size_t)t * D + c, o);
    }
  }
}

// NV values instantiated: rows of 256 * NV elements.
#define RDB_NV_LIST(X) X(1) X(2) X(3) X(4) X(5) X(6) X(8) X(10) X(12) X(14) X(16) X(20) X(24) X(28) X(32)

static void check_d(int D) {
  const int nv = D / 256;
  bool ok = (D % 256 == 0);
  bool listed = false;
#define RDB_CHK(N) listed |= (nv == N);
  RDB_NV_LIST(RDB_CHK)
#undef RDB_CHK
  if (!ok || !listed)
    throw std::invalid_argument("norm: row length must be 256*NV with NV in {1..6,8,10,12,14,16,20,24,28,32}");
}

static int norm_nv(int D) {  // smallest instantiated NV covering the row
  const int need = (D + 255) / 256;
  int best = 1 << 30;
#define RDB_PICK(N) if (N >= need && N < best) best = N;
  RDB_NV_LIST(RDB_PICK)
#undef RDB_PICK
  return best;
}

template <typename T, int MODE>
static void launch_norm(dim3 grid, hipStream_t s, uintptr_t x, uintptr_t res, uintptr_t res_out,
                        uintptr_t gamma, uintptr_t beta, uintptr_t y, int rows, int D, int ldx, float eps) {
  const int nv = norm_nv(D);
#define RDB_CASE(N)                                                                             \
  if (nv == N) {                                                                                \
    hipLaunchKernelGGL((norm_kernel<T, MODE, N>), grid, dim3(256), 0, s, (const T*)x,          \
                       (const T*)res, (T*)res_out, (const T*)gamma, (const T*)beta, (T*)y, rows, \
                       D, ldx, eps);                                                            \
    return;                                                                                     \
  }
  RDB_NV_LIST(RDB_CASE)
#undef RDB_CASE
}

// Half-wave-per-token form of embed_ln_kernel (16-B accesses, 8 tokens per
// block; norm16_kernel's layout): half the memory instructions of the 8-B form
// and the row reductions stay inside the half wave.
template <typename T, int NV>
__global__ void __launch_bounds__(256)
embed16_kernel(const int* __restrict__ ids, const int* __restrict__ types, const T* __restrict__ word,
               const T* __restrict__ pos, const T* __restrict__ typ, const T* __restrict__ gamma,
               const T* __restrict__ beta, T* __restrict__ y, int tokens, int S, int D, int vocab, float eps,
               float2* __restrict__ zst, int zn, int zstride) {
  const int hl = threadIdx.x & 31;
  const int t = blockIdx.x * 8 + (threadIdx.x >> 5);
  if (t >= tokens) return;      // whole half waves only: the xor-16..1 reductions stay inside a half
  for (int k = hl; k < zn; k += 32) zst[(size_t)k * zstride + t] = float2{0.f, 0.f};
  int id = ids[t];
  id = id < 0 ? 0 : (id >= vocab ? vocab - 1 : id);
  const int tt = types ? types[t] : 0;
  const int p = t % S;
  float v[NV][8];
  float sm = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = i * 256 + hl * 8;
    float a[8], b[8], d[8];
    load8(word + (size_t)id * D + c, a);
    load8(pos + (size_t)p * D + c, b);
    load8(typ + (size_t)tt * D + c, d);
#pragma unroll
    for (int e = 0; e < 8; ++e) { v[i][e] = a[e] + b[e] + d[e]; sm += v[i][e]; }
  }
  const float mean = half_sum(sm) / D;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i)
#pragma unroll
    for (int e = 0; e < 8; ++e) { const float dd = v[i][e] - mean; q += dd * dd; }
  const float rstd = rsqrtf(half_sum(q) / D + eps);
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = i * 256 + hl * 8;
    float g[8], b[8], o[8];
    load8(gamma + c, g);
    load8(beta + c, b);
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = (v[i][e] - mean) * rstd * g[e] + b[e];
    st8(y + (size_t)t * D + c, o);
  }
}

template <typename T>
static bool launch_embed16(hipStream_t s, uintptr_t ids, uintptr_t types, uintptr_t word, uintptr_t pos,
                           uintptr_t typ, uintptr_t gamma, uintptr_t beta, uintptr_t y, int tokens, int S, int D,
                           int vocab, float eps, uintptr_t zst, int zn, int zstride) {
  if ((word | pos | typ | gamma | beta | y) & 15) return false;
  const dim3 grid((tokens + 7) / 8);
#define RDB_E16(NV)                                                                                          \
  if (D == 256 * NV) {                                                                                       \
    hipLaunchKernelGGL((embed16_kernel<T, NV>), grid, dim3(256), 0, s, (const int*)ids, (const int*)types,   \
                       (const T*)word, (const T*)pos, (const T*)typ, (const T*)gamma, (const T*)beta, (T*)y, \
                       tokens, S, D, vocab, eps, (float2*)zst, zn, zstride);                                 \
    return true;                                                                                             \
  }
  RDB_E16(1) RDB_E16(2) RDB_E16(3) RDB_E16(4) RDB_E16(8) RDB_E16(16)
#undef RDB_E16
  return false;
}

template <typename T>
static void launch_embed(dim3 grid, hipStream_t s, uintptr_t ids, uintptr_t types, uintptr_t word,
                         uintptr_t pos, uintptr_t typ, uintptr_t gamma, uintptr_t beta, uintptr_t y,
                         int tokens, int S, int D, int vocab, float eps, uintptr_t zst, int zn, int zstride) {
  const int nv = D / 256;
#define RDB_CASE(N)                                                                              \
  if (nv == N) {                                                                                 \
    hipLaunchKernelGGL((embed_ln_kernel<T, N>), grid, dim3(256), 0, s, (const int*)ids,         \
                       (const int*)types, (const T*)word, (const T*)pos, (const T*)typ,          \
                       (const T*)gamma, (const T*)beta, (T*)y, tokens, S, D, vocab, eps,         \
                       (float2*)zst, zn, zstride);                                              \
    return;                                                                                      \
  }
  RDB_NV_LIST(RDB_CASE)
#undef RDB_CASE
}

template <typename T, int MODE>
static bool launch_norm16(hipStream_t s, uintptr_t x, uintptr_t res, uintptr_t res_out, uintptr_t gamma,
                          uintptr_t beta, uintptr_t y, int rows, int D, int ldx, float eps) {
  static const int max_blocks = [] {
    const char* e = std::getenv("RDB_LN_BLOCKS");
    return e ? std::atoi(e) : 0;
  }();
  // RDB_LN_THREADS: 64 / 128 / 256 threads = 2 / 4 / 8 rows per block (A/B knob; default 256)
  static const int threads = [] {
    const char* e = std::getenv("RDB_LN_THREADS");
    const int t = e ? std::atoi(e) : 256;
    return (t == 64 || t == 128) ? t : 256;
  }();
  const int rpb = threads / 32;
  const int groups = (rows + rpb - 1) / rpb;
  const dim3 grid(max_blocks > 0 && groups > max_blocks ? max_blocks : groups), blk(threads);
#define RDB_N16(NV)                                                                                         \
  if (D == 256 * NV) {                                                                                      \
    hipLaunchKernelGGL((norm16_kernel<T, MODE, NV>), grid, blk, 0, s, (const T*)x, (const T*)res, (T*)res_out, \
                       (const T*)gamma, (const T*)beta, (T*)y, rows, ldx, eps);                              \
    return true;                                                                                            \
  }
  RDB_N16(1) RDB_N16(2) RDB_N16(3) RDB_N16(4) RDB_N16(8) RDB_N16(16)
#undef RDB_N16
  return false;
}

void norm_fwd(int dtype, int mode, uintptr_t x, uintptr_t res, uintptr_t res_out, uintptr_t gamma,
              uintptr_t beta, uintptr_t y, int rows, int D, int ldx, float eps, uintptr_t stream) {
  if (D % 4 != 0 || D <= 0 || D > 8192) throw std::invalid_argument("norm: D must be a multiple of 4, <= 8192");
  if (ldx < D || ldx % 4 != 0 || (ldx != D && res != 0)) throw std::invalid_argument("norm: bad x row stride");
  if (rows <= 0) return;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  // 16-B half-wave form when every operand allows it (RDB_NORM16=0 forces the 8-B form)
  static const bool n16_env = [] { const char* e = getenv("RDB_NORM16"); return !(e && e[0] == '0'); }();
  const bool a16 = ((x | res | res_out | gamma | beta | y) & 15) == 0 && ldx % 8 == 0 && D % 256 == 0;
  if (n16_env && a16) {
    bool ok;
    if (dtype == 0) ok = mode == 0 ? launch_norm16<bf16, 0>(s, x, res, res_out, gamma, beta, y, rows, D, ldx, eps)
                                   : launch_norm16<bf16, 1>(s, x, res, res_out, gamma, beta, y, rows, D, ldx, eps);
    else if (dtype == 1) ok = mode == 0 ? launch_norm16<f16, 0>(s, x, res, res_out, gamma, beta, y, rows, D, ldx, eps)
                                        : launch_norm16<f16, 1>(s, x, res, res_out, gamma, beta, y, rows, D, ldx, eps);
    else ok = false;
    if (ok) {
      RDB_HIP_CHECK(hipGetLastError());
      return;
    }
  }
  dim3 grid((rows + 3) / 4);
  if (dtype == 0) {
    if (mode == 0) launch_norm<bf16, 0>(grid, s, x, res, res_out, gamma, beta, y, rows, D, ldx, eps);
    else launch_norm<bf16, 1>(grid, s, x, res, res_out, gamma, beta, y, rows, D, ldx, eps);
  } else if (dtype == 1) {
    if (mode == 0) launch_norm<f16, 0>(grid, s, x, res, res_out, gamma, beta, y, rows, D, ldx, eps);
    else launch_norm<f16, 1>(grid, s, x, res, res_out, gamma, beta, y, rows, D, ldx, eps);
  } else {
    throw std::invalid_argument("norm: dtype must be bf16 or f16");
  }
  RDB_HIP_CHECK(hipGetLastError());
}

void embed_ln_fwd(int dtype, uintptr_t ids, uintptr_t types, uintptr_t word, uintptr_t pos,
                  uintptr_t typ, uintptr_t gamma, uintptr_t beta, uintptr_t y, int tokens, int S,
                  int D, int vocab, float eps, uintptr_t zero_stats, int zn, int zstride, uintptr_t stream) {
  check_d(D);
  if (zero_stats && (zn < 0 || zstride < tokens)) throw std::invalid_argument("embed_ln: bad zero_stats layout");
  if (!zero_stats) zn = 0;
  if (tokens <= 0) return;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  static const bool e16_env = [] { const char* e = getenv("RDB_EMBED16"); return !(e && e[0] == '0'); }();
  if (e16_env && dtype <= 1) {
    const bool ok = dtype == 0 ? launch_embed16<bf16>(s, ids, types, word, pos, typ, gamma, beta, y, tokens, S, D, vocab,
                                                      eps, zero_stats, zn, zstride)
                               : launch_embed16<f16>(s, ids, types, word, pos, typ, gamma, beta, y, tokens, S, D, vocab,
                                                     eps, zero_stats, zn, zstride);
    if (ok) {
      RDB_HIP_CHECK(hipGetLastError());
      return;
    }
  }
  dim3 grid((tokens + 3) / 4);
  if (dtype == 0)
    launch_embed<bf16>(grid, s, ids, types, word, pos, typ, gamma, beta, y, tokens, S, D, vocab, eps, zero_stats, zn, zstride);
  else if (dtype == 1)
    launch_embed<f16>(grid, s, ids, types, word, pos, typ, gamma, beta, y, tokens, S, D, vocab, eps, zero_stats, zn, zstride);
  else
    throw std::invalid_argument("embed_ln: dtype must be bf16 or f16");
  RDB_HIP_CHECK(hipGetLastError());
}

}  // namespace rdb
