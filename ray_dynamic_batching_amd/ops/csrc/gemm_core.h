// Core MFMA GEMM main loop shared by the dense GEMM (gemm.hip) and the
// implicit-GEMM NHWC convolution (conv.hip).  Only the A-operand loader differs:
// DenseLoader reads a row-major [M, K] matrix, Im2colLoader gathers the
// [N*P*Q, R*S*C] im2col matrix on the fly from an NHWC activation tensor (it is
// never materialised).
//
//   C[m, n] = act(alpha * sum_k A[m, k] * W[n, k] + bias[n] + R[m, n])
//
// Design (cdna_hip_programming.md §5):
//  * 256 threads = 4 waves in a 2x2 grid; each wave owns (BM/2)x(BN/2).
//  * v_mfma_f32_16x16x32_{bf16,f16} with SWAPPED operands (W fragment as the
//    MFMA A operand): the accumulator then holds 4 consecutive n for one m per
//    lane, so the fused epilogue stores 8 contiguous bytes per lane.
//  * BK = 64, two LDS stages filled by LDS-DMA (buffer_load ... lds, bounds-
//    checked: out-of-range rows/k read as 0 with no branch); the DMA of tile k+1
//    is issued before the MFMAs of tile k; one barrier per K-step.
//  * LDS rows are 128 B; the 16-B chunk index is XOR-swizzled with (row>>1)&7 so
//    each 16-lane group of ds_read_b128 hits 16 distinct bank quads (T2).
//  * XCD-aware bijective block remap: the N-tiles of one M-panel share an L2 (T1).
#pragma once
#include "common.h"
#include <algorithm>
#include <type_traits>

namespace rdb {

template <typename T> struct MfmaOp;
template <> struct MfmaOp<bf16> {
  typedef bf16x8 frag;
  static __device__ __forceinline__ f32x4 mma(frag a, frag b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
  }
};
template <> struct MfmaOp<f16> {
  typedef f16x8 frag;
  static __device__ __forceinline__ f32x4 mma(frag a, frag b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
  }
};

__device__ __forceinline__ int swz_off(int row, int chunk) {
  return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4);
}

template <typename OutT>
__device__ __forceinline__ void store4(OutT* p, float a, float b, float c, float d);
template <>
__device__ __forceinline__ void store4<bf16>(bf16* p, float a, float b, float c, float d) {
  bf16x4 v = {(bf16)a, (bf16)b, (bf16)c, (bf16)d};
  *reinterpret_cast<bf16x4*>(p) = v;
}
template <>
__device__ __forceinline__ void store4<f16>(f16* p, float a, float b, float c, float d) {
  f16x4 v = {(f16)a, (f16)b, (f16)c, (f16)d};
  *reinterpret_cast<f16x4*>(p) = v;
}
template <>
__device__ __forceinline__ void store4<float>(float* p, float a, float b, float c, float d) {
  *reinterpret_cast<f32x4*>(p) = f32x4{a, b, c, d};
}

__device__ __forceinline__ float act_rt(int act, float x) {
  switch (act) {
    case ACT_GELU: return apply_act<ACT_GELU>(x);
    case ACT_RELU: return apply_act<ACT_RELU>(x);
    case ACT_TANH: return apply_act<ACT_TANH>(x);
    case ACT_SILU: return apply_act<ACT_SILU>(x);
    case ACT_GELU_TANH: return apply_act<ACT_GELU_TANH>(x);
    case ACT_SIGMOID: return apply_act<ACT_SIGMOID>(x);
    default: return x;
  }
}

// ---- buffer-resource helpers (T8): out-of-range loads return 0 with no branch ----
constexpr uint32_t kOOB = 0x80000000u;  // voffset sentinel beyond every num_records
// The descriptor inputs are readfirstlane'd so hipcc can PROVE the SRD wave-
// uniform; otherwise it wraps every buffer op in a waterfall loop (guide T20).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* p, uint32_t bytes) {
  const uint64_t a = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  void* base = reinterpret_cast<void*>(((uint64_t)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(base, (short)0, (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}
__device__ __forceinline__ u32x4 bload16(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
}
__device__ __forceinline__ u32x2 bload8(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0);
}
__device__ __forceinline__ uint32_t bload4(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0);
}

// ---- A-operand loaders -------------------------------------------------------
// Staging is LDS-DMA (buffer_load ... lds): each wave instruction writes 1 KiB =
// 8 rows x 128 B of the tile LINEARLY into LDS, lane l -> row 8*j + l/8,
// physical chunk l%8.  The XOR swizzle of the LDS image is therefore applied on
// the SOURCE side (guide rule 21): lane l fetches logical chunk
// (l%8) ^ ((row>>1)&7).  Loaders return the byte offset of that 16-B chunk in
// their buffer resource, or kOOB (zero fill, no branch).
__device__ __forceinline__ int dma_row(int tid, int nch, int i) {
  return (((tid >> 6) * nch + i) << 3) + ((tid & 63) >> 3);
}
__device__ __forceinline__ int dma_chunk(int tid, int row) { return (tid & 7) ^ ((row >> 1) & 7); }

struct DenseParams {
  const void* A;
  int lda, M, K;
};
template <typename T, int NCH>
struct DenseLoader {
  typedef DenseParams Params;
  __amdgpu_buffer_rsrc_t rsrc;
  uint32_t rowoff[NCH];
  int chunk[NCH];
  int K;
  __device__ __forceinline__ void init(const Params& p, int tid, int m0) {
    K = p.K;
    rsrc = make_rsrc(p.A, (uint32_t)((size_t)(p.M - 1) * p.lda * sizeof(T) + (size_t)p.K * sizeof(T)));
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int row = dma_row(tid, NCH, i);
      chunk[i] = dma_chunk(tid, row);
      const int gm = m0 + row;
      rowoff[i] = gm < p.M ? (uint32_t)((size_t)gm * p.lda * sizeof(T)) : kOOB;
    }
  }
  __device__ __forceinline__ void prep(int) {}
  __device__ __forceinline__ uint32_t offset(int i, int k0) const {
    const int gk = k0 + chunk[i] * 8;
    return (gk < K && rowoff[i] != kOOB) ? rowoff[i] + (uint32_t)(gk * sizeof(T)) : kOOB;
  }
};

struct ConvParams {
  const void* x;  // NHWC
  int N, H, W, C, R, S, stride, pad, P, Q;
  int M, K;       // M = N*P*Q, K = R*S*C
};
template <typename T, int NCH>
struct Im2colLoader {
  typedef ConvParams Params;
  __amdgpu_buffer_rsrc_t rsrc;
  uint32_t imgoff[NCH];
  int h0[NCH], w0[NCH], chunk[NCH];
  int pix[NCH];        // fast path: (h0 * W + w0) * C + chunk * 8 (elements from the image base)
  int K, C, S, H, W;
  // C % 64 == 0 (every ResNet conv but the stem): a 64-deep K step lies inside
  // one filter tap, so (r, s, c0) are block-uniform -- decomposed ONCE per K
  // step by prep() instead of two integer divisions per lane and chunk
  bool fast;
  int ur, us, uoff;
  __device__ __forceinline__ void init(const Params& p, int tid, int m0) {
    K = p.K; C = p.C; S = p.S; H = p.H; W = p.W;
    fast = (p.C & 63) == 0;
    rsrc = make_rsrc(p.x, (uint32_t)((size_t)p.N * p.H * p.W * p.C * sizeof(T)));
#pragma unroll
    for (int i = 0; i < NCH; ++i) {
      const int row = dma_row(tid, NCH, i);
      chunk[i] = dma_chunk(tid, row);
      const int gm = m0 + row;
      const int pq = p.P * p.Q;
      const int n = gm / pq;
      const int rem = gm - n * pq;
      const int pp = rem / p.Q, qq = rem - pp * p.Q;
      h0[i] = gm < p.M ? pp * p.stride - p.pad : -(1 << 20);
      w0[i] = qq * p.stride - p.pad;
      pix[i] = gm < p.M ? ((pp * p.stride - p.pad) * p.W + w0[i]) * p.C + chunk[i] * 8 : 0;
      imgoff[i] = (uint32_t)((size_t)n * p.H * p.W * p.C * sizeof(T));
    }
  }
  __device__ __forceinline__ void prep(int k0) {
    if (fast) {
      const int rs = k0 / C, c0 = k0 - rs * C;
      ur = rs / S;
      us = rs - ur * S;
      uoff = (ur * W + us) * C + c0;
    }
  }
  __device__ __forceinline__ uint32_t offset(int i, int k0) const {
    if (fast) {
      const int h = h0[i] + ur, w = w0[i] + us;
      const bool ok = k0 < K && (unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W;
      return ok ? imgoff[i] + (uint32_t)((pix[i] + uoff) * (int)sizeof(T)) : kOOB;
    }
    const int gk = k0 + chunk[i] * 8;
    const int rs = gk / C;
    const int cc = gk - rs * C;
    const int r = rs / S, s = rs - r * S;
    const int h = h0[i] + r, w = w0[i] + s;
    const bool ok = gk < K && (unsigned)h < (unsigned)H && (unsigned)w < (unsigned)W;
    return ok ? imgoff[i] + (uint32_t)((((size_t)h * W + w) * C + cc) * sizeof(T)) : kOOB;
  }
};

typedef __attribute__((address_space(3))) void* lds_ptr_t;
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, char* lds, uint32_t off) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr_t)lds, 16, off, 0, 0, 0);
}

// ---- deferred-LayerNorm epilogue operands --------------------------------------
// A post-LN transformer's LayerNorm can be folded into the GEMMs around it
// (models/bert.py ``fold_ln``): the producing GEMM accumulates per-row (sum,
// sum of squares) of the values it stores (STATS), the consuming GEMM multiplies
// the RAW rows by W' = W * gamma and corrects in its epilogue (LNA):
//     LN(a) W^T + b = rstd[m] * (a W'^T - mean[m] * colsum(W')[n]) + (b + W beta)[n]
// and a residual operand that is a normalised row is normalised on load (LNR):
//     R'[m, n] = (R[m, n] - mean_R[m]) * rstd_R[m] * g[n] + be[n].
// No LayerNorm kernel runs and the normalised rows are never materialised.
// EPI_SELF (with LNA): the GEMM computes A's row statistics itself from the
// A fragments it already holds for the MFMAs (every block streams whole rows
// of A through the main loop) -- no producer-side statistics pass, no atomics.
// Blocks of the first N tile also store them to o_stats (plain stores, one
// writer per row) for a later LNR consumer of the same rows.
//
// EPI_LNOUT: y = LayerNorm(A W^T + bias + R) written directly -- the GEMM's
// row panel (the tiles_n blocks sharing BM rows) reduces each row's statistics
// through a zeroed workspace and a per-panel arrival counter (staged_ln_epilogue).
constexpr int EPI_LNA = 1, EPI_LNR = 2, EPI_STATS = 4, EPI_SELF = 8, EPI_LNOUT = 16;
// EPI_STG: the LayerNorm modes on the LDS-STAGED epilogue (ping-pong and 4-/8-wave
// tiles alike) with PARTIAL statistics: a producer (STATS) stores, per row, one
// (sum, sum of squares) per N-tile -- stats[m][tile_n] = partial over its BN
// columns, plain stores, no atomics, nothing to zero -- and a consumer (LNA /
// LNR) sums the row's `parts` partials.  The row statistics and the per-column
// vectors are staged in LDS by the kernel's prologue (ln_stage), so the
// epilogue reads them like the bias.
constexpr int EPI_STG = 32;
// EPI_SWG: the ping-pong kernels' SwiGLU instantiation (plain staged epilogue, N/2
// output columns; a separate kernel so the other epilogues' register allocation is
// untouched by the SiLU-pairing path)
constexpr int EPI_SWG = 64;
struct LnEpi {
  const float* a_stats;   // LNA: (sum, sumsq) of A's rows, row stride a_ld floats
  const float* a_colsum;  // LNA: colsum(W') [N]
  const float* a_bias;    // LNA: b + W beta [N] (f32)
  const float* r_stats;   // LNR: (sum, sumsq) of R's rows, row stride r_ld floats
  const void* r_g;        // LNR: gamma, beta [N] (element type T)
  const void* r_b;
  float* o_stats;         // STATS: += (sum, sumsq) of the stored rows, row stride o_ld floats
                          // LNOUT: zeroed [M, 2] workspace (row stride 2)
  int a_ld, r_ld, o_ld;
  float a_inv_d, r_inv_d, eps;
  int* panel;             // LNOUT: zeroed arrival counters, one per row panel (tiles_m)
  int* err;               // LNOUT: set to 1 if a panel wait timed out (never hangs)
  int a_parts, r_parts;   // STG: partials per row in a_stats / r_stats (row stride a_ld / r_ld floats)
  // split-K (plain epilogues, gridDim.y = splits > 1): split z runs K-steps
  // [z * sk_kper, (z + 1) * sk_kper); the last split of a tile to arrive at its
  // counter adds the others' f32 partials and runs the epilogue (no waiting)
  float* sk_part;         // [tiles][splits][BM * BN] f32 partial tiles
  int* sk_cnt;            // [tiles] arrival counters, zero between launches (the last arriver resets)
  int sk_kper;
};

// (sum, sum of squares) of the 8 elements of an MFMA fragment, accumulated with
// the packed dot instructions (v_dot2_f32_{bf16,f16}: 2 elements per VALU op)
template <typename T, typename F8>
__device__ __forceinline__ void frag_stats(const F8& f, float& s1, float& s2) {
  typedef T t2 __attribute__((ext_vector_type(2)));
  const T one = (T)1.0f;
  const t2 ones = {one, one};
#pragma unroll
  for (int e = 0; e < 8; e += 2) {
    const t2 p = {f[e], f[e + 1]};
    if constexpr (std::is_same<T, bf16>::value) {
      s1 = __builtin_amdgcn_fdot2_f32_bf16(p, ones, s1, false);
      s2 = __builtin_amdgcn_fdot2_f32_bf16(p, p, s2, false);
    } else {
      s1 = __builtin_amdgcn_fdot2(p, ones, s1, false);
      s2 = __builtin_amdgcn_fdot2(p, p, s2, false);
    }
  }
}

__device__ __forceinline__ void ln_row_stats(float2 v, float inv_d, float eps, float& mu, float& rstd) {
  mu = v.x * inv_d;
  rstd = rsqrtf(fmaxf(v.y * inv_d - mu * mu, 0.f) + eps);
}

// LDS regions of the staged LayerNorm epilogues (EPI_STG), after the staging
// buffers and the bias: per tile row (mean, rstd) of A (LNA) or of the
// residual (LNR); two f32 column vectors (LNA: colsum(W'), folded bias; LNR:
// gamma, beta); per tile row the (sum, sum of squares) accumulator of STATS.
template <int BM, int BN>
struct LnLds {
  static constexpr int ROWS = 0, COLA = BM * 8, COLB = COLA + BN * 4, RACC = COLB + BN * 4, BYTES = RACC + BM * 8;
};

// Kernel prologue of the EPI_STG modes (before the first LDS-DMA, like the bias
// staging: an ordinary load behind an in-flight DMA would drain it): fills
// the LnLds regions at `base`; visible after the prologue barrier.
template <typename T, int EPI, int BM, int BN, int NT>
__device__ __forceinline__ void ln_stage(char* base, const LnEpi& ln, int m0, int n0, int M, int N) {
  constexpr bool LNA = (EPI & EPI_LNA) != 0, LNR = (EPI & EPI_LNR) != 0, OST = (EPI & EPI_STATS) != 0;
  typedef LnLds<BM, BN> L;
  const int tid = threadIdx.x;
  if constexpr (LNA || LNR) {
    const float* st = LNA ? ln.a_stats : ln.r_stats;
    const int ld = LNA ? ln.a_ld : ln.r_ld, parts = LNA ? ln.a_parts : ln.r_parts;
    const float inv_d = LNA ? ln.a_inv_d : ln.r_inv_d;
    for (int r = tid; r < BM; r += NT) {
      const int m = m0 + r < M ? m0 + r : M - 1;
      const float* row = st + (size_t)m * ld;
      float s1 = 0.f, s2 = 0.f;
      for (int p = 0; p < parts; ++p) {
        const float2 v = *reinterpret_cast<const float2*>(row + 2 * p);
        s1 += v.x;
        s2 += v.y;
      }
      float mu, rs;
      ln_row_stats(float2{s1, s2}, inv_d, ln.eps, mu, rs);
      reinterpret_cast<float2*>(base + L::ROWS)[r] = float2{mu, rs};
    }
    for (int c = tid; c < BN; c += NT) {
      const int n = n0 + c < N ? n0 + c : N - 1;
      float a, b;
      if constexpr (LNA) {
        a = ln.a_colsum[n];
        b = ln.a_bias[n];
      } else {
        a = (float)static_cast<const T*>(ln.r_g)[n];
        b = (float)static_cast<const T*>(ln.r_b)[n];
      }
      reinterpret_cast<float*>(base + L::COLA)[c] = a;
      reinterpret_cast<float*>(base + L::COLB)[c] = b;
    }
  }
  if constexpr (OST)
    for (int r = tid; r < BM; r += NT) reinterpret_cast<float2*>(base + L::RACC)[r] = float2{0.f, 0.f};
}

// Epilogue end of EPI_STG | EPI_STATS: each tile row's partial (sum, sum of
// squares) of the values as STORED goes to o_stats[m][tile_n] (plain stores).
template <int BM, int BN, int NT>
__device__ __forceinline__ void ln_store_partials(const char* base, const LnEpi& ln, int m0, int M, int tile_n) {
  typedef LnLds<BM, BN> L;
  for (int r = threadIdx.x; r < BM; r += NT)
    if (m0 + r < M)
      *reinterpret_cast<float2*>(ln.o_stats + (size_t)(m0 + r) * ln.o_ld + 2 * tile_n) =
          reinterpret_cast<const float2*>(base + L::RACC)[r];
}

// ---- LDS-staged, row-coalesced epilogue ----------------------------------------
// The MFMA accumulator layout gives each lane 4 consecutive columns of one row,
// so a direct store is 8 B per lane and one wave-instruction touches 16 rows x
// 32 B: the epilogue then runs store-issue bound (measured 6.7k of a 256x128
// tile's 30k cycles at K = 768, bench/gemm_lab).  Instead every lane parks
// alpha*acc + bias (f32) in the now idle staging LDS, and the block re-reads it
// row-major: each lane owns 8 consecutive columns of a row, adds the residual
// with one 16-B load, applies the activation and writes 16 B -- a wave stores
// whole 128-B lines.  Tiles taller than the LDS are done in row chunks.
// Requirements (host/caller-checked): N % 8 == 0, ldc % 8 == 0, C (and R,
// ldr) 16-B aligned, 2-byte OutT.
template <int BM, int BN, int SMEM_BYTES>
struct StagedEpi {
  static constexpr int ROWB = BN * 4 + 16;                   // f32 row + 16 B (bank rotation)
  static constexpr int RC_MAX = (SMEM_BYTES / ROWB) / 16 * 16;
  static constexpr int pick() {
    int rc = RC_MAX < BM ? RC_MAX : BM;
    while (rc > 16 && BM % rc) rc -= 16;
    return rc;
  }
  static constexpr int RC = pick();                          // rows per chunk
  static constexpr int NV = BN / 8;                          // 8-column vectors per row
  static_assert(BN % 8 == 0 && RC >= 16 && BM % RC == 0, "staged epilogue geometry");
};

// Activation tag of the staged 16-bit epilogue for SwiGLU: W rows interleaved
// (gate_j, up_j), so a lane's 4 consecutive columns n..n+3 hold (g, u, g', u')
// and it parks silu(g) * u, silu(g') * u' at output columns n/2, n/2 + 1; the
// stored tile is BN/2 wide (output row stride ldc, N/2 columns).
struct SwigluAct {
  __device__ __forceinline__ float operator()(float x) const { return x; }
};

// 16-bit staging rows (residual-free epilogue): BN x 2 B + 32 B, so the 16 rows
// of one ds_write_b64 wave instruction start 8 banks apart.
template <int BM, int BN, int SMEM_BYTES>
struct StagedEpi16 {
  static constexpr int ROWB = BN * 2 + 32;
  static constexpr int RC_MAX = (SMEM_BYTES / ROWB) / 16 * 16;
  static constexpr int pick() {
    int rc = RC_MAX < BM ? RC_MAX : BM;
    while (rc > 16 && BM % rc) rc -= 16;
    return rc;
  }
  static constexpr int RC = pick();
  static constexpr int NV = BN / 8;
  static_assert(BN % 8 == 0 && RC >= 16 && BM % RC == 0, "staged 16-bit epilogue geometry");
};

// BIAS_LDS >= 0: the tile's bias was staged (f32) at smem + BIAS_LDS by the
// kernel's prologue, so no bias registers stay live across the epilogue.
// EPI (EPI_STG modes only) / LN_LDS: the LayerNorm epilogues, their operands
// staged by ln_stage at smem + LN_LDS (LnLds layout):
//   EPI_LNA   y = act(rstd[m] (alpha acc - mean[m] colsum[n]) + bias'[n])   (16-bit staging)
//   EPI_LNR   the residual is added as LayerNorm(R) (normalised on load)     (f32 staging)
//   EPI_STATS each tile row's (sum, sum of squares) of the stored values -> o_stats[m][tile_n]
template <typename T, typename OutT, int BM, int BN, int SMEM_BYTES, int NT, int TM, int TN, bool HAS_BIAS,
          bool HAS_RES, typename ActF, int BIAS_LDS = -1, int EPI = 0, int LN_LDS = -1>
__device__ __forceinline__ void staged_epilogue(char* smem, const f32x4 (&acc)[TN][TM], int row_base, int col_base,
                                                int m0, int n0, int M, int N, OutT* __restrict__ C, int ldc,
                                                const T* __restrict__ bias, const T* __restrict__ R, int ldr,
                                                float alpha, ActF actf, const LnEpi* ln = nullptr, int tile_n = 0) {
  typedef StagedEpi<BM, BN, SMEM_BYTES> E;
  constexpr bool SLNA = (EPI & EPI_STG) && (EPI & EPI_LNA), SLNR = (EPI & EPI_STG) && (EPI & EPI_LNR);
  constexpr bool SOST = (EPI & EPI_STG) && (EPI & EPI_STATS);
  static_assert(!(EPI & EPI_STG) || LN_LDS >= 0, "staged LN modes need their LDS operands");
  static_assert(!SLNA || (!HAS_RES && !HAS_BIAS && !SOST), "staged LNA: no residual, bias folded, no stats out");
  static_assert(!SLNR || HAS_RES, "staged LNR normalises the residual");
  typedef LnLds<BM, BN> LL;
  const char* lnb = smem + (LN_LDS >= 0 ? LN_LDS : 0);
  const int tid = threadIdx.x, lane = tid & 63;
  const int fr = lane & 15, fg = lane >> 4;
  // bias in the fragment layout (TN x 8 B per lane), fetched once for all chunks
  constexpr bool BREG = HAS_BIAS && BIAS_LDS < 0;
  float bv[BREG ? TN : 1][4];
#pragma unroll
  for (int i = 0; i < (BREG ? TN : 0); ++i) {
    const int n = n0 + col_base + i * 16 + fg * 4;
    if constexpr (BREG) {
      const __amdgpu_buffer_rsrc_t bsrc = make_rsrc(bias, (uint32_t)(N * sizeof(T)));
      const u32x2 raw = bload8(bsrc, (uint32_t)(n * sizeof(T)));
      const T* e = reinterpret_cast<const T*>(&raw);
#pragma unroll
      for (int q = 0; q < 4; ++q) bv[i][q] = (float)e[q];
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) bv[i][q] = 0.f;
    }
  }
#ifdef RDB_EPI_F32_STAGING
  constexpr bool kStage16 = false;   // A/B build: the f32-staged epilogue for every GEMM
#else
  constexpr bool kStage16 = !HAS_RES && sizeof(OutT) == 2 && !SOST;
#endif
  // SwigluAct is an identity functor: only the 16-bit staged branch pairs the
  // gate / up columns into silu(g) * u at half width.
  static_assert(kStage16 || !std::is_same<ActF, SwigluAct>::value,
                "SwiGLU needs the 16-bit staged epilogue (not in RDB_EPI_F32_STAGING builds)");
  if constexpr (kStage16) {
    // No residual: bias + activation run once on the accumulator registers,
    // the tile is parked as 16-bit output (half the LDS traffic of f32, twice
    // the rows per chunk) and phase 2 only moves 16-B row segments to global.
    typedef StagedEpi16<BM, BN, SMEM_BYTES> E16;
    // bias + activation fragment by fragment, each packed to 16-bit pairs and
    // parked right away: only the accumulators stay live.  (Building the
    // whole packed tile first held it beside the accumulators and the
    // activation temporaries -- 128 VGPRs spilled on the 2-blocks-per-CU
    // 256x128 FFN-up tile, 244 on 256x256.)  A fragment's 16 rows never
    // straddle a chunk (RC % 16 == 0), so the chunk test is wave-uniform; with
    // several chunks only the waves owning the chunk's rows compute in it.
    auto park = [&](int i, int j, int rt, int trow) {
      const int nt = col_base + i * 16 + fg * 4;
      f32x4 v = acc[i][j] * alpha;
      if constexpr (SLNA) {
        const float2 st = reinterpret_cast<const float2*>(lnb + LL::ROWS)[trow];
        const f32x4 cs = *reinterpret_cast<const f32x4*>(lnb + LL::COLA + nt * 4);
        const f32x4 bb = *reinterpret_cast<const f32x4*>(lnb + LL::COLB + nt * 4);
        v = (v - st.x * cs) * st.y + bb;
      } else if constexpr (BREG) {
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] += bv[i][q];
      } else if constexpr (HAS_BIAS) {
        v += *reinterpret_cast<const f32x4*>(smem + BIAS_LDS + nt * 4);
      }
      if constexpr (std::is_same<ActF, SwigluAct>::value) {
        OutT o2[2] = {(OutT)(apply_act<ACT_SILU>(v[0]) * v[1]), (OutT)(apply_act<ACT_SILU>(v[2]) * v[3])};
        *reinterpret_cast<uint32_t*>(smem + rt * E16::ROWB + nt) = *reinterpret_cast<const uint32_t*>(o2);
      } else {
        OutT o4[4] = {(OutT)actf(v[0]), (OutT)actf(v[1]), (OutT)actf(v[2]), (OutT)actf(v[3])};
        *reinterpret_cast<u32x2*>(smem + rt * E16::ROWB + nt * 2) = *reinterpret_cast<const u32x2*>(o4);
      }
    };
#pragma unroll 1
    for (int c = 0; c < BM / E16::RC; ++c) {
#pragma unroll
      for (int j = 0; j < TM; ++j) {
        const int rt = row_base + j * 16 + fr - c * E16::RC;
        if (rt >= 0 && rt < E16::RC) {
#pragma unroll
          for (int i = 0; i < TN; ++i) {
            park(i, j, rt, row_base + j * 16 + fr);
            // keep the scheduler from interleaving every fragment's activation
            // (the no-bias variants spilled 51..245 VGPRs without it)
            __builtin_amdgcn_sched_barrier(0);
          }
        }
      }
      __syncthreads();
      // SwiGLU: BN/2 output columns per row, starting at n0/2 (N/2 in all)
      constexpr bool SWG = std::is_same<ActF, SwigluAct>::value;
      static_assert(!SWG || (BN % 16 == 0), "staged SwiGLU: BN % 16 == 0");
      constexpr int NVO = SWG ? E16::NV / 2 : E16::NV;
      const int n_base = SWG ? (n0 >> 1) : n0, n_lim = SWG ? (N >> 1) : N;
#pragma unroll 4
      for (int idx = tid; idx < E16::RC * NVO; idx += NT) {
        const int r = idx / NVO, vcol = idx - r * NVO;
        const int m = m0 + c * E16::RC + r, n = n_base + vcol * 8;
        if (m < M && n < n_lim)
          *reinterpret_cast<u32x4*>(C + (size_t)m * ldc + n) =
              *reinterpret_cast<const u32x4*>(smem + r * E16::ROWB + vcol * 16);
      }
      __syncthreads();
    }
    return;
  }
  // Residual prefetch: this thread's phase-2 residual vectors are loaded BEFORE
  // phase 1, so their memory latency runs under the LDS parking and the
  // barrier instead of after it (at most 8 x 16 B per thread, beside the
  // accumulators).  The barrier then waits for LDS traffic only.  Probe on
  // MI355X (bench/gemm_probe.py --res): FFN-down 4096x768x3072 on the 256x128
  // ping-pong tile 42.2 -> 40.9 us (40.1 without a residual); the 4-wave
  // 128x96 o-proj got slower (11.6 -> 12.0 us), so 4-wave tiles keep the loop.
  // phase-2 finish of one 8-column vector of tile row trow: + residual (LNR:
  // normalised on load), activation, 16-B store; STATS: row sums into LDS
  auto finish = [&](float (&x)[8], const u32x4& rraw, int trow, int vcol, int m, int n) {
    if constexpr (HAS_RES) {
      const T* e = reinterpret_cast<const T*>(&rraw);
      if constexpr (SLNR) {
        const float2 st = reinterpret_cast<const float2*>(lnb + LL::ROWS)[trow];
        const f32x4* g = reinterpret_cast<const f32x4*>(lnb + LL::COLA + (n - n0) * 4);
        const f32x4* be = reinterpret_cast<const f32x4*>(lnb + LL::COLB + (n - n0) * 4);
        const f32x4 g0 = g[0], g1 = g[1], b0 = be[0], b1 = be[1];
        const float gg[8] = {g0[0], g0[1], g0[2], g0[3], g1[0], g1[1], g1[2], g1[3]};
        const float bb[8] = {b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
#pragma unroll
        for (int q = 0; q < 8; ++q) x[q] += ((float)e[q] - st.x) * st.y * gg[q] + bb[q];
      } else {
#pragma unroll
        for (int q = 0; q < 8; ++q) x[q] += (float)e[q];
      }
    }
    OutT o[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) o[q] = (OutT)actf(x[q]);
    *reinterpret_cast<u32x4*>(C + (size_t)m * ldc + n) = *reinterpret_cast<const u32x4*>(o);
    if constexpr (SOST) {
      // statistics of the values as STORED (what a LayerNorm reading C would see)
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const float y = (float)o[q];
        s1 += y;
        s2 += y * y;
      }
      float2* racc = reinterpret_cast<float2*>(const_cast<char*>(lnb) + LL::RACC);
      atomicAdd(&racc[trow].x, s1);
      atomicAdd(&racc[trow].y, s2);
    }
    (void)vcol;
  };
  constexpr int NVEC = E::RC * E::NV;
  constexpr int PER = (NVEC + NT - 1) / NT;
#ifdef RDB_EPI_NO_RES_PREFETCH
  constexpr bool PREF = false;
#else
  constexpr bool PREF = HAS_RES && PER <= 8 && NT >= 512;   // 8-wave tiles (4-wave o-proj: +0.4 us measured)
#endif
#pragma unroll 1
  for (int c = 0; c < BM / E::RC; ++c) {
    u32x4 rpre[PREF ? PER : 1];
    if constexpr (PREF) {
#pragma unroll
      for (int u = 0; u < PER; ++u) {
        const int idx = tid + u * NT;
        const int r = idx / E::NV, vcol = idx - r * E::NV;
        const int m = m0 + c * E::RC + r, n = n0 + vcol * 8;
        rpre[u] = u32x4{0u, 0u, 0u, 0u};
        if (idx < NVEC && m < M && n < N) rpre[u] = *reinterpret_cast<const u32x4*>(R + (size_t)m * ldr + n);
      }
    }
    // phase 1: alpha * acc + bias -> LDS (f32)
#pragma unroll
    for (int j = 0; j < TM; ++j) {
      const int rt = row_base + j * 16 + fr - c * E::RC;    // row inside this chunk
      if (rt >= 0 && rt < E::RC) {
#pragma unroll
        for (int i = 0; i < TN; ++i) {
          const int nt = col_base + i * 16 + fg * 4;
          f32x4 v = acc[i][j] * alpha;
          if constexpr (BREG) {
#pragma unroll
            for (int q = 0; q < 4; ++q) v[q] += bv[i][q];
          } else if constexpr (HAS_BIAS) {
            v += *reinterpret_cast<const f32x4*>(smem + BIAS_LDS + nt * 4);
          }
          *reinterpret_cast<f32x4*>(smem + rt * E::ROWB + nt * 4) = v;
        }
      }
    }
    if constexpr (PREF) {
      // LDS writes done and visible; the prefetched residual loads stay in flight
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0), vmcnt / expcnt untouched
      asm volatile("" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int u = 0; u < PER; ++u) {
        const int idx = tid + u * NT;
        const int r = idx / E::NV, vcol = idx - r * E::NV;
        const int m = m0 + c * E::RC + r, n = n0 + vcol * 8;
        if (idx < NVEC && m < M && n < N) {
          const f32x4 a = *reinterpret_cast<const f32x4*>(smem + r * E::ROWB + vcol * 32);
          const f32x4 b = *reinterpret_cast<const f32x4*>(smem + r * E::ROWB + vcol * 32 + 16);
          float x[8] = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
          finish(x, rpre[u], c * E::RC + r, vcol, m, n);
        }
      }
      __syncthreads();
      continue;
    }
    __syncthreads();
    // phase 2: row-major, 8 columns per lane, 16-B residual loads and stores of
    // whole lines; unrolled 4x so four residual loads are in flight at once
#pragma unroll 4
    for (int idx = tid; idx < E::RC * E::NV; idx += NT) {
      const int r = idx / E::NV, vcol = idx - r * E::NV;
      const int m = m0 + c * E::RC + r, n = n0 + vcol * 8;
      if (m < M && n < N) {
        u32x4 rraw = {0u, 0u, 0u, 0u};
        if constexpr (HAS_RES) rraw = *reinterpret_cast<const u32x4*>(R + (size_t)m * ldr + n);
        const f32x4 a = *reinterpret_cast<const f32x4*>(smem + r * E::ROWB + vcol * 32);
        const f32x4 b = *reinterpret_cast<const f32x4*>(smem + r * E::ROWB + vcol * 32 + 16);
        float x[8] = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
        finish(x, rraw, c * E::RC + r, vcol, m, n);
      }
    }
    __syncthreads();
  }
  if constexpr (SOST) ln_store_partials<BM, BN, NT>(lnb, *ln, m0, M, tile_n);
}

// ---- GEMM + residual + LayerNorm epilogue (EPI_LNOUT) ---------------------------
// y[m, :] = LN(alpha * acc + bias + R)[m, :] * gamma + beta for post-LN
// transformers (BERT's o-proj -> LN1, FFN-down -> LN2): no LayerNorm kernel and
// no pre-LN activation round trip.  A row's N columns are spread over the
// tiles_n blocks of its row panel, so:
//   1. the tile (+ bias + residual) is parked in LDS as f32 (staged layout),
//      each row's partial (sum, sum of squares) accumulated with LDS atomics;
//   2. one thread per row adds them to the zeroed workspace (system-scope float
//      atomics: performed past the per-XCD L2s, so a panel may straddle XCDs),
//      then thread 0 arrives on the panel's
//      counter and waits (bounded: ~20 ms, then ln.err = 1 -- a wrong result,
//      never a hang) until all tiles_n blocks arrived;
//   3. the block reads the full statistics and writes normalised rows, 16 B
//      per lane.
// Deadlock freedom: blocks are dispatched in blockIdx order and xcd_remap keeps
// a panel's tiles_n consecutive tiles on one XCD, so an incomplete panel only
// waits on blocks behind the dispatched prefix, which are dispatched as soon as
// complete panels (or other kernels) free their slots -- as long as an XCD has
// more block slots than tiles_n (host-checked).  The workspace must be zeroed
// before every launch (models/bert.py: the embedding kernel does it).
template <int BM, int BN, int SMEM_BYTES>
struct LnOutFit {
  typedef StagedEpi<BM, BN, SMEM_BYTES> E;
  static constexpr bool ok = E::RC == BM && BM * E::ROWB + BM * 8 <= SMEM_BYTES;
};

template <typename T, typename OutT, int BM, int BN, int SMEM_BYTES, int NT, int TM, int TN, int BIAS_LDS = -1>
__device__ __forceinline__ void staged_ln_epilogue(char* smem, const f32x4 (&acc)[TN][TM], int row_base, int col_base,
                                                   int m0, int n0, int M, int N, OutT* __restrict__ C, int ldc,
                                                   const T* __restrict__ bias, const T* __restrict__ R, int ldr,
                                                   float alpha, const LnEpi& ln, int tile_m, int tiles_n) {
  typedef StagedEpi<BM, BN, SMEM_BYTES> E;
  if constexpr (!LnOutFit<BM, BN, SMEM_BYTES>::ok) {
    __builtin_trap();   // host-side ln_out_tile_ok() never launches this
  } else {
    const int tid = threadIdx.x, lane = tid & 63;
    const int fr = lane & 15, fg = lane >> 4;
    float2* racc = reinterpret_cast<float2*>(smem + BM * E::ROWB);
    // phase 1: alpha * acc + bias -> LDS (f32)
#pragma unroll
    for (int i = 0; i < TN; ++i) {
      const int nt = col_base + i * 16 + fg * 4;
      f32x4 bv;
      if constexpr (BIAS_LDS >= 0) {
        bv = *reinterpret_cast<const f32x4*>(smem + BIAS_LDS + nt * 4);
      } else {
        const __amdgpu_buffer_rsrc_t bsrc = make_rsrc(bias, (uint32_t)(N * sizeof(T)));
        const u32x2 raw = bload8(bsrc, (uint32_t)((n0 + nt) * sizeof(T)));
        const T* e = reinterpret_cast<const T*>(&raw);
        bv = f32x4{(float)e[0], (float)e[1], (float)e[2], (float)e[3]};
      }
#pragma unroll
      for (int j = 0; j < TM; ++j)
        *reinterpret_cast<f32x4*>(smem + (row_base + j * 16 + fr) * E::ROWB + nt * 4) = acc[i][j] * alpha + bv;
    }
    for (int r = tid; r < BM; r += NT) racc[r] = float2{0.f, 0.f};
    __syncthreads();
    // phase 2a: + residual (16-B loads), x back to LDS, row partial sums (LDS atomics)
#pragma unroll 4
    for (int idx = tid; idx < BM * E::NV; idx += NT) {
      const int r = idx / E::NV, vcol = idx - r * E::NV;
      const int m = m0 + r, n = n0 + vcol * 8;
      if (m < M && n < N) {
        const u32x4 rraw = *reinterpret_cast<const u32x4*>(R + (size_t)m * ldr + n);
        f32x4* p = reinterpret_cast<f32x4*>(smem + r * E::ROWB + vcol * 32);
        f32x4 a = p[0], b = p[1];
        const T* e = reinterpret_cast<const T*>(&rraw);
        a += f32x4{(float)e[0], (float)e[1], (float)e[2], (float)e[3]};
        b += f32x4{(float)e[4], (float)e[5], (float)e[6], (float)e[7]};
        p[0] = a;
        p[1] = b;
        const float s = (a[0] + a[1]) + (a[2] + a[3]) + (b[0] + b[1]) + (b[2] + b[3]);
        const float q = a[0] * a[0] + a[1] * a[1] + a[2] * a[2] + a[3] * a[3] + b[0] * b[0] + b[1] * b[1] +
                        b[2] * b[2] + b[3] * b[3];
        atomicAdd(&racc[r].x, s);
        atomicAdd(&racc[r].y, q);
      }
    }
    __syncthreads();
    for (int r = tid; r < BM; r += NT) {
      const int m = m0 + r;
      if (m < M) {
        __hip_atomic_fetch_add(ln.o_stats + (size_t)m * 2, racc[r].x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_fetch_add(ln.o_stats + (size_t)m * 2 + 1, racc[r].y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
    // Ordering without L2-wide fences (a release / acquire here is a whole-L2
    // writeback / invalidate per block): every thread waits for ITS atomics to
    // be acknowledged (gfx9 counts no-return atomics in vmcnt), the barrier
    // joins them, then one relaxed arrival; readers poll and read with
    // system-scope loads, which are served past the non-coherent L2s.
    __builtin_amdgcn_s_waitcnt(0x70 | 0xF00);   // vmcnt(0)
    __syncthreads();
    if (tid == 0) {
      int* cnt = ln.panel + tile_m;
      __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();        // 100 MHz
      while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < tiles_n) {
        if (__builtin_amdgcn_s_memrealtime() - t0 > 2000000ull) {   // 20 ms
          if (ln.err) __hip_atomic_store(ln.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
    }
    __syncthreads();
    for (int r = tid; r < BM; r += NT) {
      const int m = m0 + r < M ? m0 + r : M - 1;
      const float sm = __hip_atomic_load(ln.o_stats + (size_t)m * 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      const float sq = __hip_atomic_load(ln.o_stats + (size_t)m * 2 + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      float mu, rstd;
      ln_row_stats(float2{sm, sq}, ln.r_inv_d, ln.eps, mu, rstd);
      racc[r] = float2{mu, rstd};
    }
    __syncthreads();
    // phase 2b: normalise, gamma / beta, 16-B stores of whole lines
    const T* g = static_cast<const T*>(ln.r_g);
    const T* be = static_cast<const T*>(ln.r_b);
#pragma unroll 4
    for (int idx = tid; idx < BM * E::NV; idx += NT) {
      const int r = idx / E::NV, vcol = idx - r * E::NV;
      const int m = m0 + r, n = n0 + vcol * 8;
      if (m < M && n < N) {
        const u32x4 graw = *reinterpret_cast<const u32x4*>(g + n);
        const u32x4 braw = *reinterpret_cast<const u32x4*>(be + n);
        const T* ge = reinterpret_cast<const T*>(&graw);
        const T* bb = reinterpret_cast<const T*>(&braw);
        const f32x4 a = *reinterpret_cast<const f32x4*>(smem + r * E::ROWB + vcol * 32);
        const f32x4 b = *reinterpret_cast<const f32x4*>(smem + r * E::ROWB + vcol * 32 + 16);
        const float2 st = racc[r];
        const float x[8] = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
        OutT o[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) o[q] = (OutT)((x[q] - st.x) * st.y * (float)ge[q] + (float)bb[q]);
        *reinterpret_cast<u32x4*>(C + (size_t)m * ldc + n) = *reinterpret_cast<const u32x4*>(o);
      }
    }
  }
}

template <typename T, typename OutT, bool HAS_RES>
__device__ __forceinline__ bool staged_epilogue_ok(int N, const OutT* C, int ldc, const T* bias, const T* R, int ldr) {
  if constexpr (sizeof(OutT) != 2) return false;
  bool ok = (N & 7) == 0 && (ldc & 7) == 0 && (reinterpret_cast<uintptr_t>(C) & 15) == 0;
  if constexpr (HAS_RES) ok = ok && (ldr & 7) == 0 && (reinterpret_cast<uintptr_t>(R) & 15) == 0;
  return ok;
}

// ---- the kernel ---------------------------------------------------------------
// 4 waves per block laid out WGM (along M) x 4/WGM (along N).  BN only has to
// be a multiple of 16 x (4/WGM): the W tile is DMA'd in whole 32-row wave
// pieces, rows past BN are zero-filled into LDS padding and never read --
// this is what allows quantisation-exact tiles such as 128x144 (N = 2304 in
// 16 column blocks, 512 tiles at M = 4096 = 2 per CU exactly).
//
// NW = 8 waves (512 threads, one block per CU) runs the big tiles (256x128,
// 256x192, ...): twice the MFMA work per staged byte of a 4-wave 128-row tile,
// which is what the L2-bandwidth-bound BERT shapes need (FFN2 at 128x48 moves
// ~14 TB/s through L2 for 0.5 PF).
template <typename T, typename OutT, int BM, int BN, template <typename, int> class LoaderT, bool HAS_BIAS,
          bool HAS_RES, int WGM = 2, int NW = 4, int EPI = 0, int DEEP = 0>
__global__ void __launch_bounds__(64 * NW, (NW == 4 && !DEEP) ? 2 : 1)
mfma_gemm_kernel(typename LoaderT<T, 1>::Params ap, const T* __restrict__ W, int ldw,
                 OutT* __restrict__ C, int ldc, const T* __restrict__ bias,
                 const T* __restrict__ R, int ldr, int M, int N, int K, float alpha, int act, LnEpi ln) {
  // STG: the staged-epilogue LayerNorm modes (operands in LDS, partial stats);
  // the other flags are the direct-epilogue (legacy) modes
  constexpr bool STG = (EPI & EPI_STG) != 0;
  constexpr bool LNA = !STG && (EPI & EPI_LNA) != 0, LNR = !STG && (EPI & EPI_LNR) != 0;
  constexpr bool OST = !STG && (EPI & EPI_STATS) != 0;
  constexpr bool SELF = (EPI & EPI_SELF) != 0;
  constexpr bool LNOUT = (EPI & EPI_LNOUT) != 0;
  static_assert(!SELF || (LNA && !OST), "SELF computes LNA's statistics; it writes o_stats itself");
  static_assert(!LNOUT || (EPI == EPI_LNOUT && HAS_BIAS && HAS_RES), "LNOUT: bias + residual, no other LN mode");
  static_assert(!LNA || !HAS_BIAS, "LNA takes its (folded) bias from ln.a_bias");
  static_assert(!LNR || HAS_RES, "LNR normalises the residual operand");
  constexpr int BK = 64;
  constexpr int WGN = NW / WGM;
  constexpr int NT = 64 * NW;                 // threads
  constexpr int WM = BM / WGM, WN = BN / WGN;
  constexpr int TM = WM / 16, TN = WN / 16;
  static_assert(WM % 16 == 0 && WN % 16 == 0 && BM % 32 == 0, "tile / wave layout mismatch");
  static_assert(WGM * WGN == NW && BM % (8 * NW) == 0, "wave layout / DMA split");
  constexpr int A_CH = BM * 8 / NT;                  // 16-B chunks per thread per A tile
  constexpr int W_CH = (BN + 8 * NW - 1) / (8 * NW);  // rounded up: rows >= BN are LDS padding
  constexpr int BNP = W_CH * 8 * NW;
  constexpr int kStage = (BM + BNP) * BK * 2;  // bytes per LDS stage (A tile, then W tile)
  // Three LDS stages (two K-tiles in flight across each barrier) whenever they
  // still fit two blocks per CU; the big tiles keep two stages.  DEEP: one
  // block per CU with up to 8 stages in ~150 KiB of LDS -- for grids of at most
  // ~one tile per CU, where a lone block otherwise waits out the DMA latency
  // every K step (a 128x128 tile has 2 stages: 1.75 us per K step measured on
  // the ResNet-50 layer-3 convolutions, ~10 % MFMA busy)
  constexpr int kStages = DEEP ? ((152 * 1024) / kStage < 8 ? (152 * 1024) / kStage : 8)
                               : ((3 * kStage <= (NW == 4 ? 80 : 160) * 1024) ? 3 : 2);
  static_assert(kStages >= 2, "LDS stages");
  typedef typename MfmaOp<T>::frag frag;

  constexpr int LN_OFF = kStages * kStage;
  __shared__ __attribute__((aligned(16))) char smem[LN_OFF + (STG ? LnLds<BM, BN>::BYTES : 0)];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wm = wid / WGN, wn = wid % WGN;

  const int tiles_n = (N + BN - 1) / BN;
  const int tiles_m = (M + BM - 1) / BM;
  const int nwg = tiles_m * tiles_n;
  const int t = xcd_remap(blockIdx.x, nwg);
  // row-major tile order: an XCD gets whole row panels.  A grouped (GM x N/GM
  // block per XCD) order lowers the per-XCD operand bytes on paper but measured
  // -5 % req/s (profiles/ab_r2.json): the row panels of consecutive kernels
  // then land on the XCD whose L2 holds the producer's rows.
  const int tile_m = t / tiles_n, tile_n = t - tile_m * tiles_n;
  const int m0 = tile_m * BM, n0 = tile_n * BN;

  LoaderT<T, A_CH> la;
  la.init(ap, tid, m0);

  const __amdgpu_buffer_rsrc_t wsrc = make_rsrc(W, (uint32_t)((size_t)(N - 1) * ldw * sizeof(T) + (size_t)K * sizeof(T)));
  uint32_t woff[W_CH];
  int wch[W_CH];
#pragma unroll
  for (int i = 0; i < W_CH; ++i) {
    const int row = dma_row(tid, W_CH, i);
    wch[i] = dma_chunk(tid, row);
    const int gn = n0 + row;
    woff[i] = (row < BN && gn < N) ? (uint32_t)((size_t)gn * ldw * sizeof(T)) : kOOB;
  }
  // wave-uniform LDS bases of this wave's DMA pieces
  const int wid_u = __builtin_amdgcn_readfirstlane(wid);
  auto stage = [&](int buf, int k0) {
    char* base = smem + buf * kStage;
    la.prep(k0);
#pragma unroll
    for (int i = 0; i < A_CH; ++i) dma16(la.rsrc, base + (wid_u * A_CH + i) * 1024, la.offset(i, k0));
#pragma unroll
    for (int i = 0; i < W_CH; ++i) {
      const int gk = k0 + wch[i] * 8;
      const uint32_t off = (gk < K && woff[i] != kOOB) ? woff[i] + (uint32_t)(gk * sizeof(T)) : kOOB;
      dma16(wsrc, base + BM * BK * 2 + (wid_u * W_CH + i) * 1024, off);
    }
  };

  f32x4 acc[TN][TM];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fg = lane >> 4;
  // SELF: per-lane partial (sum, sum of squares) of A rows wm*WM + j*16 + fr over
  // this lane's k slice; the 4 lanes of a row are combined after the loop
  float st1[SELF ? TM : 1], st2[SELF ? TM : 1];
#pragma unroll
  for (int j = 0; j < (SELF ? TM : 1); ++j) st1[j] = st2[j] = 0.f;
  auto compute = [&](int buf, int k0) {
    const char* sa = smem + buf * kStage;
    const char* sw = sa + BM * BK * 2;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      frag wf[TN], af[TM];
      const int chunk = ks * 4 + fg;
#pragma unroll
      for (int i = 0; i < TN; ++i)
        wf[i] = *reinterpret_cast<const frag*>(sw + swz_off(wn * WN + i * 16 + fr, chunk));
#pragma unroll
      for (int j = 0; j < TM; ++j)
        af[j] = *reinterpret_cast<const frag*>(sa + swz_off(wm * WM + j * 16 + fr, chunk));
      if constexpr (SELF) {
        // k >= K reads as zero (DMA bounds check): contributes nothing to either sum
#pragma unroll
        for (int j = 0; j < TM; ++j) frag_stats<T>(af[j], st1[j], st2[j]);
        (void)k0;
      }
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int j = 0; j < TM; ++j) acc[i][j] = MfmaOp<T>::mma(wf[i], af[j], acc[i][j]);
      // keep the two K-halves' fragments from being hoisted together (register
      // pressure: the big tiles spilled without it)
      if constexpr (TM * TN >= 16) __builtin_amdgcn_sched_barrier(0);
    }
  };

  // deferred-LN row statistics are fetched before the main loop: their latency
  // hides under it instead of opening the epilogue
  float2 ast[LNA ? TM : 1], rst[LNR ? TM : 1];
  if constexpr ((LNA && !SELF) || LNR) {
#pragma unroll
    for (int j = 0; j < TM; ++j) {
      const int m = m0 + wm * WM + j * 16 + fr;
      const size_t ms = (size_t)(m < M ? m : M - 1);
      if constexpr (LNA && !SELF) ast[j] = *reinterpret_cast<const float2*>(ln.a_stats + ms * ln.a_ld);
      if constexpr (LNR) rst[j] = *reinterpret_cast<const float2*>(ln.r_stats + ms * ln.r_ld);
    }
  }

  if constexpr (STG) ln_stage<T, EPI, BM, BN, NT>(smem + LN_OFF, ln, m0, n0, M, N);   // before the first DMA
  // split-K: this block's K-steps [kb, kb + nk) (host: every split non-empty)
  const int nk_all = (K + BK - 1) / BK;
  const int kb = EPI == 0 && gridDim.y > 1 ? (int)blockIdx.y * ln.sk_kper : 0;
  const int nk = EPI == 0 && gridDim.y > 1 ? min(ln.sk_kper, nk_all - kb) : nk_all;
  if constexpr (kStages == 2) {
    // Two LDS stages: the DMA of tile k+1 runs under the MFMAs of tile k; the
    // __syncthreads() at the end of a step waits the issuing waves' DMA
    // (vmcnt(0)) and orders every wave's reads before the buffer is refilled.
    stage(0, kb * BK);
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      if (kt + 1 < nk) stage((kt + 1) & 1, (kb + kt + 1) * BK);
      compute(kt & 1, (kb + kt) * BK);
      __syncthreads();
    }
  } else {
    // Three LDS stages (guide §5 "Pipelining across barriers"): tiles k+1 and
    // k+2 stay in flight while tile k is consumed.  Each wave retires ITS OWN
    // DMA of tile k with a counted vmcnt (leaving tile k+1's kLoads pending),
    // then a RAW s_barrier (no __syncthreads: its fence would drain vmcnt to 0)
    // makes every wave's pieces of tile k visible.  Buffer (k+2)%3 was last
    // read by compute(k-1), which every wave finished before this barrier, so
    // it is refilled right after it (WAR-safe).
    // (kStages > 3, DEEP: kStages - 1 tiles in flight, the same protocol)
    constexpr int kLoads = A_CH + W_CH;                  // DMA instructions per wave per stage
    constexpr int kPend = kLoads * (kStages - 2);        // younger tiles' DMAs left pending
    constexpr int kWaitPend = (kPend & 15) | ((kPend >> 4) << 14) | 0x70 | 0xF00;   // vmcnt(kPend)
    constexpr int kWaitAll = 0x70 | 0xF00;                                           // vmcnt(0)
    static_assert(kPend < 64, "vmcnt field is 6 bits");
#pragma unroll
    for (int p = 0; p < kStages - 1; ++p)
      if (p < nk) stage(p, (kb + p) * BK);
    int buf = 0;
    for (int kt = 0; kt < nk; ++kt) {
      if (kt + kStages - 2 < nk) __builtin_amdgcn_s_waitcnt(kWaitPend);
      else __builtin_amdgcn_s_waitcnt(kWaitAll);       // the tail: fewer younger tiles in flight
      asm volatile("" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (kt + kStages - 1 < nk)
        stage(buf == 0 ? kStages - 1 : buf - 1, (kb + kt + kStages - 1) * BK);
      compute(buf, (kb + kt) * BK);
      buf = buf == kStages - 1 ? 0 : buf + 1;
    }
    __syncthreads();
  }
  if constexpr (EPI == 0) {
    if (gridDim.y > 1) {
      // ---- split-K hand-off (the gemm_sk.h protocol): partials are stored and
      // loaded sc1; a storing block drains vmcnt, meets at a barrier, then one
      // lane adds to the tile's counter (agent scope).  The last arriver --
      // told by the counter -- resets it, folds the other splits in and goes on
      // to the epilogue; every other block is done.  Nobody waits.
      __shared__ int sk_flag;
      const int splits = gridDim.y, z = blockIdx.y;
      int* cnt = ln.sk_cnt + t;
      const __amdgpu_buffer_rsrc_t psrc =
          make_rsrc(ln.sk_part, (uint32_t)((size_t)nwg * splits * BM * BN * sizeof(float)));
      auto slot_off = [&](int zz, int i, int j) {
        return (uint32_t)(((((size_t)t * splits + zz) * (TN * TM) + i * TM + j) * NT + tid) * 16);
      };
      if (tid == 0) sk_flag = __hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == splits - 1;
      __syncthreads();
      bool last = sk_flag != 0;
      __syncthreads();
      if (!last) {
#pragma unroll
        for (int i = 0; i < TN; ++i)
#pragma unroll
          for (int j = 0; j < TM; ++j)
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[i][j]), psrc, slot_off(z, i, j), 0, 16);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0)
          sk_flag = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == splits - 1;
        __syncthreads();
        last = sk_flag != 0;
      }
      if (!last) return;
      if (tid == 0) __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      for (int zz = 0; zz < splits; ++zz) {
        if (zz == z) continue;
#pragma unroll
        for (int i = 0; i < TN; ++i)
#pragma unroll
          for (int j = 0; j < TM; ++j)
            acc[i][j] += __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(psrc, slot_off(zz, i, j), 0, 16));
      }
    }
  }
  if constexpr (SELF) {
#pragma unroll
    for (int j = 0; j < TM; ++j) {
      float a = st1[j], q = st2[j];
      a += __shfl_xor(a, 16, 64);
      q += __shfl_xor(q, 16, 64);
      a += __shfl_xor(a, 32, 64);
      q += __shfl_xor(q, 32, 64);
      ast[j] = float2{a, q};
      const int m = m0 + wm * WM + j * 16 + fr;
      if (ln.o_stats != nullptr && tile_n == 0 && wn == 0 && fg == 0 && m < M)
        *reinterpret_cast<float2*>(ln.o_stats + (size_t)m * ln.o_ld) = ast[j];
    }
  }

  if constexpr (LNOUT && sizeof(OutT) == 2) {
    // host-checked: N % 8, ldc % 8, 16-B aligned C / R, ldr % 8, no activation
    staged_ln_epilogue<T, OutT, BM, BN, kStages * kStage, NT, TM, TN>(smem, acc, wm * WM, wn * WN, m0, n0, M, N, C,
                                                                     ldc, bias, R, ldr, alpha, ln, tile_m, tiles_n);
    return;
  }
  // ---- LDS-staged coalesced epilogue (plain modes; LN / SwiGLU keep the direct one) ----
  if constexpr ((EPI == 0 || STG) && sizeof(OutT) == 2) {
    // (STG launches are host-checked for the staged epilogue's requirements)
    // SwiGLU stages too when there is no residual (N/2 output columns, N % 16, BN % 16)
    const bool swg_ok = !HAS_RES && (N & 15) == 0 && BN % 16 == 0;
    if (STG || ((act != ACT_SWIGLU || swg_ok) && staged_epilogue_ok<T, OutT, HAS_RES>(N, C, ldc, bias, R, ldr))) {
      constexpr int SB = kStages * kStage;
      auto go = [&](auto actf) {
        staged_epilogue<T, OutT, BM, BN, SB, NT, TM, TN, HAS_BIAS, HAS_RES, decltype(actf), -1, EPI,
                        STG ? LN_OFF : -1>(smem, acc, wm * WM, wn * WN, m0, n0, M, N, C, ldc, bias, R, ldr, alpha,
                                           actf, &ln, tile_n);
      };
      if constexpr (!HAS_RES && !STG && BN % 16 == 0) {
        if (act == ACT_SWIGLU) { go(SwigluAct{}); return; }
      }
      switch (act) {
        case ACT_GELU: go([](float x) { return apply_act<ACT_GELU>(x); }); break;
        case ACT_RELU: go([](float x) { return apply_act<ACT_RELU>(x); }); break;
        case ACT_TANH: go([](float x) { return apply_act<ACT_TANH>(x); }); break;
        case ACT_SILU: go([](float x) { return apply_act<ACT_SILU>(x); }); break;
        case ACT_GELU_TANH: go([](float x) { return apply_act<ACT_GELU_TANH>(x); }); break;
        case ACT_SIGMOID: go([](float x) { return apply_act<ACT_SIGMOID>(x); }); break;
        default: go([](float x) { return x; }); break;
      }
      return;
    }
  }

  // ---- fused epilogue: lane holds C[m][n..n+3] ----
  // All bias / residual loads are issued up front as vector buffer loads (OOB ->
  // 0, no per-element branch or wait), then the activation is applied in a loop
  // selected ONCE (no per-element switch).
  const bool swiglu = act == ACT_SWIGLU;
  const int n_out = swiglu ? (N >> 1) : N;
  float bv[TN][4];
  float cs[LNA ? TN : 1][4];
  u32x2 rg[LNR ? TN : 1], rb[LNR ? TN : 1];
#pragma unroll
  for (int i = 0; i < TN; ++i) {
    const int n = n0 + wn * WN + i * 16 + fg * 4;
    if constexpr (LNA) {
      // N % 4 == 0 in the LN modes (host-checked): n < N covers n..n+3
      const f32x4 z = {0.f, 0.f, 0.f, 0.f};
      const f32x4 b4 = n < N ? *reinterpret_cast<const f32x4*>(ln.a_bias + n) : z;
      const f32x4 c4 = n < N ? *reinterpret_cast<const f32x4*>(ln.a_colsum + n) : z;
#pragma unroll
      for (int q = 0; q < 4; ++q) { bv[i][q] = b4[q]; cs[i][q] = c4[q]; }
      continue;
    }
    if constexpr (LNR) {
      const u32x2 z = {0u, 0u};
      rg[i] = n < N ? *reinterpret_cast<const u32x2*>(static_cast<const T*>(ln.r_g) + n) : z;
      rb[i] = n < N ? *reinterpret_cast<const u32x2*>(static_cast<const T*>(ln.r_b) + n) : z;
    }
    if constexpr (HAS_BIAS) {
      const __amdgpu_buffer_rsrc_t bsrc = make_rsrc(bias, (uint32_t)(N * sizeof(T)));
      const u32x2 raw = bload8(bsrc, (uint32_t)(n * sizeof(T)));
      const T* e = reinterpret_cast<const T*>(&raw);
#pragma unroll
      for (int q = 0; q < 4; ++q) bv[i][q] = (float)e[q];
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) bv[i][q] = 0.f;
    }
  }
  // residual kept PACKED (4 x 16-bit in 2 VGPRs) until it is added: halves the
  // epilogue's register footprint (the unpacked tile made 128x128+ spill)
  u32x2 rraw[TM][TN];
  if constexpr (HAS_RES) {
    const __amdgpu_buffer_rsrc_t rsrc = make_rsrc(R, (uint32_t)((size_t)(M - 1) * ldr * sizeof(T) + (size_t)n_out * sizeof(T)));
#pragma unroll
    for (int j = 0; j < TM; ++j) {
      const int m = m0 + wm * WM + j * 16 + fr;
#pragma unroll
      for (int i = 0; i < TN; ++i) {
        const int n = n0 + wn * WN + i * 16 + fg * 4;
        if (!swiglu) {
          const uint32_t off = (m < M && n < N) ? (uint32_t)(((size_t)m * ldr + n) * sizeof(T)) : kOOB;
          rraw[j][i] = bload8(rsrc, off);
        } else {
          const uint32_t off = (m < M && n < N) ? (uint32_t)(((size_t)m * ldr + (n >> 1)) * sizeof(T)) : kOOB;
          rraw[j][i] = u32x2{bload4(rsrc, off), 0u};
        }
      }
    }
  }
  auto rv = [&](int j, int i, int q) -> float {
    const T* e = reinterpret_cast<const T*>(&rraw[j][i]);
    return (float)e[q];
  };
  if (swiglu) {
#pragma unroll
    for (int j = 0; j < TM; ++j) {
      const int m = m0 + wm * WM + j * 16 + fr;
#pragma unroll
      for (int i = 0; i < TN; ++i) {
        const int n = n0 + wn * WN + i * 16 + fg * 4;
        float x[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) x[q] = alpha * acc[i][j][q] + bv[i][q];
        float r0 = apply_act<ACT_SILU>(x[0]) * x[1];
        float r1 = apply_act<ACT_SILU>(x[2]) * x[3];
        if constexpr (HAS_RES) { r0 += rv(j, i, 0); r1 += rv(j, i, 1); }
        if (m < M && n < N) {
          OutT* cp = C + (size_t)m * ldc + (n >> 1);
          cp[0] = (OutT)r0;
          cp[1] = (OutT)r1;
        }
      }
    }
    return;
  }
  // y = act(alpha * acc + bias + residual), computed and stored fragment by
  // fragment: only the accumulators stay live (a separate activation pass over
  // the whole tile made the big tiles spill).  One switch selects the
  // activation for the whole tile.
  const bool vec_ok = ((ldc & 3) == 0);
  auto store_tile = [&](auto actf) {
#pragma unroll
    for (int j = 0; j < TM; ++j) {
      const int m = m0 + wm * WM + j * 16 + fr;
      float amu = 0.f, ar = 1.f, rmu = 0.f, rr = 1.f, ssum = 0.f, ssq = 0.f;
      if constexpr (LNA) ln_row_stats(ast[j], ln.a_inv_d, ln.eps, amu, ar);
      if constexpr (LNR) ln_row_stats(rst[j], ln.r_inv_d, ln.eps, rmu, rr);
#pragma unroll
      for (int i = 0; i < TN; ++i) {
        const int n = n0 + wn * WN + i * 16 + fg * 4;
        float y[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          float x;
          if constexpr (LNA) x = alpha * ar * (acc[i][j][q] - amu * cs[i][q]) + bv[i][q];
          else x = alpha * acc[i][j][q] + bv[i][q];
          if constexpr (HAS_RES) {
            float r = rv(j, i, q);
            if constexpr (LNR) {
              const T* g = reinterpret_cast<const T*>(&rg[i]);
              const T* be = reinterpret_cast<const T*>(&rb[i]);
              r = (r - rmu) * rr * (float)g[q] + (float)be[q];
            }
            x += r;
          }
          y[q] = actf(x);
          if constexpr (OST) {
            // statistics of the values as STORED (rounded to OutT), as a
            // LayerNorm kernel reading this output would see them
            const float yr = (float)(OutT)y[q];
            if (n + q < N) { ssum += yr; ssq += yr * yr; }
          }
        }
        if (m >= M || n >= N) continue;
        OutT* cp = C + (size_t)m * ldc + n;
        if (n + 3 < N && vec_ok) {
          store4<OutT>(cp, y[0], y[1], y[2], y[3]);
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (n + e < N) cp[e] = (OutT)y[e];
        }
      }
      if constexpr (OST) {
        // the 4 lanes holding row m (lane, lane^16, ^32, ^48) combine, one adds
        ssum += __shfl_xor(ssum, 16, 64);
        ssq += __shfl_xor(ssq, 16, 64);
        ssum += __shfl_xor(ssum, 32, 64);
        ssq += __shfl_xor(ssq, 32, 64);
        if (fg == 0 && m < M) {
          unsafeAtomicAdd(ln.o_stats + (size_t)m * ln.o_ld, ssum);
          unsafeAtomicAdd(ln.o_stats + (size_t)m * ln.o_ld + 1, ssq);
        }
      }
    }
  };
  switch (act) {
    case ACT_GELU: store_tile([](float x) { return apply_act<ACT_GELU>(x); }); break;
    case ACT_RELU: store_tile([](float x) { return apply_act<ACT_RELU>(x); }); break;
    case ACT_TANH: store_tile([](float x) { return apply_act<ACT_TANH>(x); }); break;
    case ACT_SILU: store_tile([](float x) { return apply_act<ACT_SILU>(x); }); break;
    case ACT_GELU_TANH: store_tile([](float x) { return apply_act<ACT_GELU_TANH>(x); }); break;
    case ACT_SIGMOID: store_tile([](float x) { return apply_act<ACT_SIGMOID>(x); }); break;
    default: store_tile([](float x) { return x; }); break;
  }
}

}  // namespace rdb
#include "gemm_pp.h"
namespace rdb {

// Tile table (index = the `cfg` argument): BM x BN with WGM waves along M.
// LDS = 2 stages x (BM + BN rounded to 32) x 64 x 2 B.  The host picks the
// entry (autotuned per shape from Python, or the heuristic below): for the
// serving shapes the dominant effect is wave quantisation -- #tiles vs 256
// CUs x blocks/CU -- hence the non-power-of-two tiles: 128x192 (N = 3072),
// 128x144 (N = 2304), 64x96 / 128x48 (N = 768) each give exactly 512 tiles
// at M = 4096 (BERT-base, batch 32).
// 19..22 are the ping-pong kernel (gemm_pp.h, 8 waves in two staggered groups;
// 22 = 256x256 at BK = 32 with 4 LDS stages, the best tile on large GEMMs:
// 1.06 PF/s at 4096^3 vs 0.90 for 19, bench/gemm_lab).
// 23 = 256x128 at BK = 32 with 3 stages (74 KiB) compiled for TWO co-resident
// blocks per CU (<= 128 VGPRs): one block's epilogue (FFN-up's GELU: ~13k
// VALU cycles per tile) runs beside the other block's MFMAs -- 3 % over 22 on
// the FFN-up shape in the two-stream lab (profiles/gemm_lab_r3_gelu_epilogue.txt).
// 24 / 25 = ping-pong 256x192 at BK = 32 with 3 / 4 stages (89 / 119 KiB): a
// 4096 x 3072 GEMM (BERT FFN-up) is exactly 256 tiles = one per CU, where 23
// leaves 1.5 blocks per CU, at 1/110 operand bytes per FLOP vs 1/85 for 256x128.
// 26 / 27 / 28 = the 4-wave VGPR-staged tiles of gemm_v4.h (128x96, 128x128,
// 256x192; one block per CU; own translation unit gemm_v4.hip, K % 64 == 0).
// 29 = ping-pong 256x224 at BK = 32, 4 stages (123 KiB): the Llama-3-8B SwiGLU
// gate-up projection (N = 28672 = 128 x 224) at 1024 / 512 tokens is exactly
// 2 / 1 rounds of 256 blocks, where 256x256 leaves the last round 3/4 / 7/8 full.
constexpr int kNumTiles = 30;
//                                 0    1    2    3    4    5    6    7    8    9   10   11   12 | 8-wave: 13   14   15   16   17   18 | pp: 19   20   21   22   23   24   25
constexpr int kTileBM[kNumTiles] = {128, 64, 128, 64, 128, 192, 256, 128, 128, 64, 128, 256, 128, 256, 128, 256, 256, 128, 256, 256, 256, 128, 256, 256, 256, 256, 128, 128, 256, 256};
constexpr int kTileBN[kNumTiles] = {128, 128, 64, 64, 192, 128, 128, 256, 144, 96, 96, 144, 48, 128, 256, 192, 144, 96, 96, 128, 144, 256, 256, 128, 192, 192, 96, 128, 192, 224};
// tile cfg flag: the DEEP (one block per CU, up to 8 LDS stages) variant of
// 4-wave tiles 0, 1, 2, 3, 6, 7, 9, 10 (plain epilogues); other tiles ignore it
constexpr int kDeepFlag = 1 << 12;
constexpr int kTileWGM[kNumTiles] = {2, 2, 2, 2, 2, 2, 2, 2, 4, 2, 2, 4, 4, 4, 2, 4, 8, 4, 8, 4, 8, 2, 4, 4, 4, 4, 2, 2, 2, 4};
constexpr int kTileNW[kNumTiles] = {4, 4, 4, 4, 4, 4, 4, 4, 4, 4, 4, 4, 4, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 8, 4, 4, 4, 8};

// gemm_v4.hip (tile cfgs 26..28): dtype 0 = bf16, 1 = f16; 16-bit output, plain epilogues
void launch_gemm_v4_cfg(int cfg, int dtype, const void* A, int lda, const void* W, int ldw, void* C, int ldc,
                        const void* bias, const void* R, int ldr, int M, int N, int K, float alpha, int act,
                        hipStream_t s);

inline int tile_blocks_per_cu(int cfg) {
  if (cfg == 23) return 2;
  if (cfg >= 19) return 1;
  const int q = 8 * kTileNW[cfg];
  const int bnp = (kTileBN[cfg] + q - 1) / q * q;
  const int lds = 2 * (kTileBM[cfg] + bnp) * 64 * 2;
  return std::min(8 / kTileNW[cfg], 163840 / lds);
}
// Whether tile cfg (0..18) can run the GEMM + residual + LayerNorm epilogue:
// the whole f32 tile plus per-row accumulators must fit the staging LDS
// (mirrors mfma_gemm_kernel's kStages / kStage and LnOutFit).
inline bool ln_out_tile_ok(int cfg) {
  if (cfg < 0 || cfg >= 19) return false;
  const int nw = kTileNW[cfg], bm = kTileBM[cfg], bn = kTileBN[cfg];
  const int wch = (bn + 8 * nw - 1) / (8 * nw);
  const int stage = (bm + wch * 8 * nw) * 64 * 2;
  const int stages = (3 * stage <= (nw == 4 ? 80 : 160) * 1024) ? 3 : 2;
  return bm * (bn * 4 + 16) + bm * 8 <= stages * stage;
}

// Tiles the staged-LayerNorm modes run (EPI_STG; launch_mfma_gemm_t): a
// producer's partial-statistics count per row is ceil(N / BN) of its tile.
constexpr int kStgTiles[] = {0, 9, 10, 12, 19, 21, 23, 24};
inline int stg_tile_cfg(int cfg) {
  for (int c : kStgTiles)
    if (c == cfg) return cfg;
  return 10;
}

// Heuristic: minimise (rounds of blocks over 256 CUs) x (tile work / tile efficiency).
constexpr int kNumTiles4 = 13;  // tiles 0..12 are 4-wave (every loader); 13.. are 8-wave (dense only)
inline int pick_tile_cfg(int M, int N, bool dense) {
  int best = 3;
  double best_t = 1e30;
  for (int c = 0; c < (dense ? 19 : kNumTiles4); ++c) {   // the pp tiles (19..) are chosen by tuning only
    const int bm = kTileBM[c], bn = kTileBN[c];
    const long tiles = (long)((M + bm - 1) / bm) * ((N + bn - 1) / bn);
    const long slots = 256L * tile_blocks_per_cu(c);
    const long rounds = (tiles + slots - 1) / slots;
    const double eff = 1.0 / (1.0 + 48.0 / bm + 48.0 / bn);        // LDS/issue overhead per FLOP
    const double t = (double)rounds * bm * bn * tile_blocks_per_cu(c) / eff;
    if (t < best_t * 0.98) { best_t = t; best = c; }
  }
  return best;
}

template <typename T, typename OutT, template <typename, int> class LoaderT, bool HB, bool HR, int BM, int BN,
          int WGM = 2, int NW = 4, int EPI = 0, int DEEP = 0, typename P>
void launch_one(const P& ap, const T* W, int ldw, OutT* C, int ldc, const T* bias, const T* R, int ldr, int M,
                int N, int K, float alpha, int act, hipStream_t s, const LnEpi& ln = LnEpi{}) {
  const int nwg = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  int splits = 1;
  if (EPI == 0 && ln.sk_kper > 0) {
    // split-K: ceil(nk / kper) non-empty splits; the workspace must hold every
    // (tile, split) partial and the tile counters (checked by splitk_fits)
    const int nk = (K + 63) / 64;
    splits = (nk + ln.sk_kper - 1) / ln.sk_kper;
  }
  hipLaunchKernelGGL((mfma_gemm_kernel<T, OutT, BM, BN, LoaderT, HB, HR, WGM, NW, EPI, DEEP>), dim3(nwg, splits),
                     dim3(64 * NW), 0, s, ap, W, ldw, C, ldc, bias, R, ldr, M, N, K, alpha, act, ln);
}

template <typename T, typename OutT, template <typename, int> class LoaderT, bool HB, bool HR, int EPI = 0,
          typename P>
void launch_mfma_gemm_t(const P& ap, const T* W, int ldw, OutT* C, int ldc, const T* bias, const T* R,
                        int ldr, int M, int N, int K, float alpha, int act, hipStream_t s, int cfg,
                        const LnEpi& ln = LnEpi{}) {
  const bool deep = cfg >= 0 && (cfg & kDeepFlag) != 0;
  (void)deep;
  if (cfg >= 0) cfg &= 0xFF;
#define RDB_TILE(IDX, BM_, BN_, WGM_, NW_)                                                                    \
  case IDX:                                                                                                  \
    launch_one<T, OutT, LoaderT, HB, HR, BM_, BN_, WGM_, NW_, EPI>(ap, W, ldw, C, ldc, bias, R, ldr, M, N, K, \
                                                                  alpha, act, s, ln);                        \
    return;
  if constexpr (std::is_same<OutT, float>::value) {
    // f32 output is only used by small heads: one tile shape
    launch_one<T, OutT, LoaderT, HB, HR, 64, 64>(ap, W, ldw, C, ldc, bias, R, ldr, M, N, K, alpha, act, s);
  } else if constexpr ((EPI & EPI_STG) != 0) {
    // staged-LayerNorm modes: the 4-wave tiles of the o-projection class and the
    // ping-pong tiles of FFN-up / FFN-down (a subset keeps the build small);
    // any other cfg runs 128x96
    const T* A = static_cast<const T*>(ap.A);
    switch (cfg) {
      RDB_TILE(0, 128, 128, 2, 4)
      RDB_TILE(9, 64, 96, 2, 4)
      RDB_TILE(12, 128, 48, 4, 4)
      case 19: launch_gemm_pp_ln<T, OutT, 8, 256, 128, 2, 2, 3, 64, 2, EPI>(A, ap.lda, W, ldw, C, ldc, bias, R, ldr, M,
                                                                            N, K, alpha, act, s, ln);
        return;
      case 21: launch_gemm_pp_ln<T, OutT, 8, 128, 256, 1, 4, 3, 64, 2, EPI>(A, ap.lda, W, ldw, C, ldc, bias, R, ldr, M,
                                                                            N, K, alpha, act, s, ln);
        return;
      case 23: launch_gemm_pp_ln<T, OutT, 8, 256, 128, 2, 2, 3, 32, 4, EPI>(A, ap.lda, W, ldw, C, ldc, bias, R, ldr, M,
                                                                            N, K, alpha, act, s, ln);
        return;
      case 24: launch_gemm_pp_ln<T, OutT, 8, 256, 192, 2, 2, 3, 32, 2, EPI>(A, ap.lda, W, ldw, C, ldc, bias, R, ldr, M,
                                                                            N, K, alpha, act, s, ln);
        return;
      default: break;
    }
    launch_one<T, OutT, LoaderT, HB, HR, 128, 96, 2, 4, EPI>(ap, W, ldw, C, ldc, bias, R, ldr, M, N, K, alpha, act, s,
                                                            ln);
  } else {
    // the ping-pong tiles (19..) take plain staged epilogues only: deferred-LN modes,
    // SwiGLU and unaligned / N % 8 != 0 outputs run the 8-wave 256x192 tile instead
    // (so do the VGPR-staged tiles 26..28 outside the experimental build)
    if (cfg >= 19 && (EPI != 0 || !gemm_pp_ok(N, ldc, ldr, C, bias, R, act) ||
                      (cfg >= 26 && cfg <= 28 && (!RDB_EXPERIMENTAL || K % 64 != 0 || act == ACT_SWIGLU)))) {
      cfg = 15;
      if (EPI == 0 && ln.sk_kper > 0) {   // split-K was requested for the pp tile: the 8-wave fallback runs unsplit
        launch_mfma_gemm_t<T, OutT, LoaderT, HB, HR, EPI>(ap, W, ldw, C, ldc, bias, R, ldr, M, N, K, alpha, act, s, 15,
                                                          LnEpi{});
        return;
      }
    }
    if constexpr (EPI == 0 && sizeof(OutT) == 2) {
      if (deep) {
#define RDB_TILE_DEEP(IDX, BM_, BN_)                                                                             \
  case IDX:                                                                                                      \
    launch_one<T, OutT, LoaderT, HB, HR, BM_, BN_, 2, 4, 0, 1>(ap, W, ldw, C, ldc, bias, R, ldr, M, N, K, alpha, \
                                                              act, s, ln);                                       \
    return;
        switch (cfg) {
          RDB_TILE_DEEP(0, 128, 128)
          RDB_TILE_DEEP(1, 64, 128)
          RDB_TILE_DEEP(2, 128, 64)
          RDB_TILE_DEEP(3, 64, 64)
          RDB_TILE_DEEP(9, 64, 96)
          RDB_TILE_DEEP(10, 128, 96)
          // 4-wave 256x128 / 128x256: 128x64 / 64x128 accumulators per wave (in
          // AGPRs), only spill-free with the whole register file of a 1-block CU
          RDB_TILE_DEEP(6, 256, 128)
          RDB_TILE_DEEP(7, 128, 256)
          default: break;
        }
#undef RDB_TILE_DEEP
      }
    }
    switch (cfg) {
      RDB_TILE(0, 128, 128, 2, 4)
      RDB_TILE(1, 64, 128, 2, 4)
      RDB_TILE(2, 128, 64, 2, 4)
      RDB_TILE(4, 128, 192, 2, 4)
      RDB_TILE(5, 192, 128, 2, 4)
      RDB_TILE(6, 256, 128, 2, 4)
      RDB_TILE(7, 128, 256, 2, 4)
      RDB_TILE(8, 128, 144, 4, 4)
      RDB_TILE(9, 64, 96, 2, 4)
      RDB_TILE(10, 128, 96, 2, 4)
      RDB_TILE(11, 256, 144, 4, 4)
      RDB_TILE(12, 128, 48, 4, 4)
      default: break;
    }
    if constexpr (std::is_same<LoaderT<T, 1>, DenseLoader<T, 1>>::value) {
      // 8-wave big tiles: dense operands only (keeps the conv build small)
      switch (cfg) {
        RDB_TILE(13, 256, 128, 4, 8)
        RDB_TILE(14, 128, 256, 2, 8)
        RDB_TILE(15, 256, 192, 4, 8)
        RDB_TILE(16, 256, 144, 8, 8)
        RDB_TILE(17, 128, 96, 4, 8)
        RDB_TILE(18, 256, 96, 8, 8)
        default: break;
      }
      if constexpr (EPI == 0 && sizeof(OutT) == 2) {
        switch (cfg) {
          case 19:
            if (ln.sk_kper > 0)
              launch_gemm_pp_sk<T, OutT, 8, 256, 128, 2, 2, 3>(static_cast<const T*>(ap.A), ap.lda, W, ldw, C, ldc,
                                                               bias, R, ldr, M, N, K, alpha, act, s, ln);
            else
              launch_gemm_pp<T, OutT, 8, 256, 128, 2, 2, 3>(static_cast<const T*>(ap.A), ap.lda, W, ldw, C, ldc,
                                                            bias, R, ldr, M, N, K, alpha, act, s);
            return;
          case 20: launch_gemm_pp<T, OutT, 8, 256, 144, 4, 1, 3>(static_cast<const T*>(ap.A), ap.lda, W, ldw, C, ldc,
                                                                  bias, R, ldr, M, N, K, alpha, act, s);
            return;
          case 21:
            if (ln.sk_kper > 0)
              launch_gemm_pp_sk<T, OutT, 8, 128, 256, 1, 4, 3>(static_cast<const T*>(ap.A), ap.lda, W, ldw, C, ldc,
                                                               bias, R, ldr, M, N, K, alpha, act, s, ln);
            else
              launch_gemm_pp<T, OutT, 8, 128, 256, 1, 4, 3>(static_cast<const T*>(ap.A), ap.lda, W, ldw, C, ldc,
                                                            bias, R, ldr, M, N, K, alpha, act, s);
            return;
          case 22: launch_gemm_pp<T, OutT, 8, 256, 256, 2, 2, 4, 32>(static_cast<const T*>(ap.A), ap.lda, W, ldw, C,
                                                                      ldc, bias, R, ldr, M, N, K, alpha, act, s);
            return;
          case 23: launch_gemm_pp<T, OutT, 8, 256, 128, 2, 2, 3, 32, 4>(static_cast<const T*>(ap.A), ap.lda, W, ldw,
                                                                         C, ldc, bias, R, ldr, M, N, K, alpha, act, s);
            return;
          case 24: launch_gemm_pp<T, OutT, 8, 256, 192, 2, 2, 3, 32>(static_cast<const T*>(ap.A), ap.lda, W, ldw, C,
                                                                      ldc, bias, R, ldr, M, N, K, alpha, act, s);
            return;
          case 25: launch_gemm_pp<T, OutT, 8, 256, 192, 2, 2, 4, 32>(static_cast<const T*>(ap.A), ap.lda, W, ldw, C,
                                                                      ldc, bias, R, ldr, M, N, K, alpha, act, s);
            return;
          case 29: launch_gemm_pp<T, OutT, 8, 256, 224, 2, 2, 4, 32>(static_cast<const T*>(ap.A), ap.lda, W, ldw, C,
                                                                      ldc, bias, R, ldr, M, N, K, alpha, act, s);
            return;
          case 26:
          case 27:
          case 28:
            launch_gemm_v4_cfg(cfg, std::is_same<T, bf16>::value ? 0 : 1, ap.A, ap.lda, W, ldw, C, ldc, bias, R, ldr,
                               M, N, K, alpha, act, s);
            return;
          default: break;
        }
      }
    }
    launch_one<T, OutT, LoaderT, HB, HR, 64, 64, 2, 4, EPI>(ap, W, ldw, C, ldc, bias, R, ldr, M, N, K, alpha, act, s,
                                                           ln);
  }
#undef RDB_TILE
}

// Split-K workspace: tile arrival counters in the first 64 KiB (zeroed once;
// every launch leaves them zero), then the f32 partial tiles.
constexpr size_t kSplitKHeader = 65536;
constexpr int kSplitKMaxTiles = (int)(kSplitKHeader / sizeof(int));
inline size_t splitk_bytes(int M, int N, int cfg, int splits) {
  const int bm = kTileBM[cfg], bn = kTileBN[cfg];
  const size_t tiles = (size_t)((M + bm - 1) / bm) * ((N + bn - 1) / bn);
  return kSplitKHeader + tiles * splits * bm * bn * sizeof(float);
}
// LnEpi carrying a split-K request, or none (splits < 2, no / too small
// workspace, too many tiles, > 2^31 partial bytes): the launch then runs unsplit.
inline LnEpi splitk_epi(int M, int N, int K, int cfg, int splits, void* ws, size_t ws_bytes) {
  LnEpi e{};
  // the 4-wave tiles, and the BK 64 ping-pong tiles 19 / 21 (gemm_pp.h SK instantiations)
  if (splits < 2 || ws == nullptr || cfg < 0 || (cfg >= kNumTiles4 && cfg != 19 && cfg != 21)) return e;
  const int nk = (K + 63) / 64;
  const int kper = (nk + splits - 1) / splits;
  const int eff = (nk + kper - 1) / kper;
  const int bm = kTileBM[cfg], bn = kTileBN[cfg];
  const long tiles = (long)((M + bm - 1) / bm) * ((N + bn - 1) / bn);
  const size_t need = splitk_bytes(M, N, cfg, eff);
  if (eff < 2 || tiles > kSplitKMaxTiles || need > ws_bytes || need - kSplitKHeader > (size_t(1) << 31)) return e;
  e.sk_cnt = static_cast<int*>(ws);
  e.sk_part = reinterpret_cast<float*>(static_cast<char*>(ws) + kSplitKHeader);
  e.sk_kper = kper;
  return e;
}

template <typename T, typename OutT, template <typename, int> class LoaderT, typename P>
void launch_mfma_gemm(const P& ap, const T* W, int ldw, OutT* C, int ldc, const T* bias, const T* R,
                      int ldr, int M, int N, int K, float alpha, int act, hipStream_t s, int cfg,
                      const LnEpi& ln = LnEpi{}) {
  constexpr bool dense = std::is_same<LoaderT<T, 1>, DenseLoader<T, 1>>::value;
  const int deep = (cfg >= 0 && (cfg & kDeepFlag) != 0) ? kDeepFlag : 0;
  if (cfg >= 0) cfg &= 0xFF;
  if (cfg < 0 || cfg >= (dense ? kNumTiles : kNumTiles4)) cfg = pick_tile_cfg(M, N, dense);
  // split-K runs on the 4-wave tiles (0..12) and the ping-pong tiles 19 / 21: their kernels carry the hand-off
  const LnEpi e = (ln.sk_kper > 0 && (cfg < kNumTiles4 || cfg == 19 || cfg == 21) && act != ACT_SWIGLU) ? ln : LnEpi{};
  cfg |= deep;
  if (bias && R)
    launch_mfma_gemm_t<T, OutT, LoaderT, true, true>(ap, W, ldw, C, ldc, bias, R, ldr, M, N, K, alpha, act, s, cfg, e);
  else if (bias)
    launch_mfma_gemm_t<T, OutT, LoaderT, true, false>(ap, W, ldw, C, ldc, bias, R, ldr, M, N, K, alpha, act, s, cfg, e);
  else if (R)
    launch_mfma_gemm_t<T, OutT, LoaderT, false, true>(ap, W, ldw, C, ldc, bias, R, ldr, M, N, K, alpha, act, s, cfg, e);
  else
    launch_mfma_gemm_t<T, OutT, LoaderT, false, false>(ap, W, ldw, C, ldc, bias, R, ldr, M, N, K, alpha, act, s, cfg, e);
}

}  // namespace rdb
