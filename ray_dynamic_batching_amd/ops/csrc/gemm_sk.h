// Stream-K ping-pong GEMM for gfx950: the serving GEMMs whose tile count
// leaves most of the 256 CUs idle (BERT FFN-down / o-proj, N = 768: 96 tiles of
// 256 x 128 at M = 4096).
//
//   C[m, n] = act(alpha * sum_k A[m, k] * W[n, k] + bias[n] + R[m, n])
//
// The (tile, K-step) iteration space of the whole GEMM (tiles x nk units) is
// cut into G equal contiguous ranges, one per workgroup (G <= the CU count, one
// 8-wave block per CU): every CU runs the same number of K-steps, whatever the
// tile count.  A range covers the TAIL of one tile, whole tiles, then the HEAD
// of another.  Its workgroup
//   * runs the tail first and publishes the f32 partial tile (write-through
//     stores in the accumulators' own per-thread order, so the read-back is
//     coalesced and needs no transpose) with a state word;
//   * stores whole tiles through the normal fused epilogue;
//   * runs the head of a tile last; the segment that arrives last at a split
//     tile folds the other segments' partials into its accumulators and runs
//     the fused epilogue.
// Because every head is run at the END of a range and every tail at the START,
// the head is almost always the last arriver and publishes nothing.
//
// No workgroup ever WAITS (so no co-residency assumption: the engine runs two
// streams and another kernel may hold CUs): a split tile is finished by
// whichever of its segments arrives LAST at the tile's arrival counter (the
// split-K last-arriver rule, one counter per tile).  A segment that sees every
// other segment already arrived skips publishing its own partial.  The last
// arriver resets the counter, so the workspace is clean for the next launch
// (one workspace per stream: two launches must never share one).
//
// Hand-off (MI355X_MICROARCH.md, "Valid forms", sc1 row): partial stores and
// loads are all sc1 (buffer ops, aux = 16); every storing wave waits
// vmcnt(0), a workgroup barrier, then one lane adds to the tile's counter
// (agent-scope atomic); the last arriver, told by its add's return value (or
// by an agent-scope load of the counter), loads after a workgroup barrier.
//
// Measured (profiles/gemm_lab_r4_streamk.txt): FFN-down 4096x768x3072 35.9 us
// on 192 workgroups vs 42.1 us for the 96-tile ping-pong kernel ALONE, but
// 28.3 vs 24.1 us per GEMM with two streams, where the other stream already
// fills the idle CUs -- a latency tool for single-stream replicas, not the
// throughput path.
//
// The main loop is the ping-pong body of gemm_pp.h (two staggered wave groups,
// LDS-DMA staging, counted vmcnt), run once per segment.
#pragma once
#include <stdexcept>
// Include after gemm_core.h (uses its PPGeom / staged_epilogue); built in its
// own translation unit (gemm_sk.hip) so edits here rebuild one object.

namespace rdb {

struct SkWorkspace {
  float* part;      // [2 G][NACC][NT] f32 partial tiles (slots 2w: a range's tail, 2w+1: its head)
  int* state;       // [tiles] arrival counters (0 between launches)
};

// bytes of workspace a launch with G workgroups needs for this tile
template <int NW, int BM, int BN>
constexpr size_t sk_part_bytes(int G) {
  return (size_t)G * BM * BN * 4;
}

__device__ __forceinline__ void sk_store16(__amdgpu_buffer_rsrc_t r, uint32_t off, f32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, off, 0, 16);   // sc1
}
__device__ __forceinline__ f32x4 sk_load16(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 16));   // sc1
}

template <typename T, typename OutT, int NW, int BM, int BN, int GM, int GN, int STAGES, bool HAS_BIAS, bool HAS_RES,
          int BK_ = 64>
__global__ void __launch_bounds__(64 * NW, 2)
gemm_sk_kernel(const T* __restrict__ A, int lda, const T* __restrict__ W, int ldw, OutT* __restrict__ C, int ldc,
               const T* __restrict__ bias, const T* __restrict__ R, int ldr, int M, int N, int K, float alpha,
               int act, SkWorkspace ws) {
  typedef PPGeom<NW, BM, BN, BK_> G;
  constexpr int BK = G::BK;
  constexpr int KS = BK / 32;
  constexpr int GW = NW / 2;
  static_assert(GM * GN == GW, "group wave layout");
  constexpr int GBM = BM / 2;
  constexpr int WM = GBM / GM, WN = BN / GN;
  constexpr int TM = WM / 16, TN = WN / 16;
  static_assert(WM % 16 == 0 && WN % 16 == 0, "wave tile must be whole 16x16 fragments");
  constexpr int L = G::LOADS;
  static_assert(STAGES >= 3 && (STAGES - 2) * L < 64, "pipeline depth / vmcnt field");
  constexpr int NACC4 = TN * TM;              // f32x4 accumulators per thread
  typedef typename MfmaOp<T>::frag frag;

  constexpr int SB = STAGES * G::STAGE_BYTES;
  constexpr int FLAG_OFF = SB;                // one broadcast word, inside the single LDS array
  __shared__ __attribute__((aligned(16))) char smem[SB + 16];
  int* bcast = reinterpret_cast<int*>(smem + FLAG_OFF);

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int grp = wid / GW, gw = wid % GW;
  const int wm = gw / GN, wn = gw % GN;
  const int wid_u = __builtin_amdgcn_readfirstlane(wid);

  const int tiles_n = (N + BN - 1) / BN, tiles_m = (M + BM - 1) / BM;
  const int nk = (K + BK - 1) / BK;
  const int64_t U = (int64_t)tiles_m * tiles_n * nk;
  const int Gn = gridDim.x;
  // consecutive ranges (which share tiles) on one XCD: their partials and
  // operand panels stay in that XCD's L2
  const int w = xcd_remap(blockIdx.x, Gn);
  auto ubeg = [&](int x) -> int64_t { return (int64_t)x * U / Gn; };
  const int64_t u0 = ubeg(w), u1 = ubeg(w + 1);

  const __amdgpu_buffer_rsrc_t asrc = make_rsrc(A, (uint32_t)((size_t)(M - 1) * lda * sizeof(T) + (size_t)K * sizeof(T)));
  const __amdgpu_buffer_rsrc_t wsrc = make_rsrc(W, (uint32_t)((size_t)(N - 1) * ldw * sizeof(T) + (size_t)K * sizeof(T)));
  const __amdgpu_buffer_rsrc_t psrc = make_rsrc(ws.part, (uint32_t)((size_t)2 * Gn * NACC4 * G::NT * 16));

  f32x4 acc[TN][TM];
  const int fr = lane & 15, fg = lane >> 4;
  const int arow0 = grp * GBM + wm * WM + fr;
  const int wrow0 = wn * WN + fr;

  // one segment of tile (tm, tn): K-steps [k0, k1), accumulated into acc
  auto run_segment = [&](int tm, int tn, int k0, int k1) {
    const int m0 = tm * BM, n0 = tn * BN;
    uint32_t aoff[G::A_PW], woff[G::W_PW];
    int ach[G::A_PW], wch[G::W_PW];
#pragma unroll
    for (int i = 0; i < G::A_PW; ++i) {
      const int row = (wid * G::A_PW + i) * G::PR + lane / G::CPR;
      ach[i] = (lane % G::CPR) ^ G::swz(row);
      const int gm = m0 + row;
      aoff[i] = gm < M ? (uint32_t)((size_t)gm * lda * sizeof(T)) : kOOB;
    }
#pragma unroll
    for (int i = 0; i < G::W_PW; ++i) {
      const int row = (wid * G::W_PW + i) * G::PR + lane / G::CPR;
      wch[i] = (lane % G::CPR) ^ G::swz(row);
      const int gn = n0 + row;
      woff[i] = (row < BN && gn < N) ? (uint32_t)((size_t)gn * ldw * sizeof(T)) : kOOB;
    }
    auto wdst = [&](char* base, int i) -> char* {
      const int piece = wid_u * G::W_PW + i;
      return base + (piece < G::W_PIECES ? G::W_OFF + piece * 1024 : G::DUMMY_OFF);
    };
    auto stage = [&](int buf, int kk) {
      char* base = smem + buf * G::STAGE_BYTES;
#pragma unroll
      for (int i = 0; i < G::A_PW; ++i) {
        const int gk = kk + ach[i] * 8;
        dma16(asrc, base + (wid_u * G::A_PW + i) * 1024, (gk < K && aoff[i] != kOOB) ? aoff[i] + (uint32_t)(gk * sizeof(T)) : kOOB);
      }
#pragma unroll
      for (int i = 0; i < G::W_PW; ++i) {
        const int gk = kk + wch[i] * 8;
        dma16(wsrc, wdst(base, i), (gk < K && woff[i] != kOOB) ? woff[i] + (uint32_t)(gk * sizeof(T)) : kOOB);
      }
    };
    frag af[KS][TM], wf[KS][TN];
    auto read_tile = [&](int buf) {
      const char* sa = smem + buf * G::STAGE_BYTES;
      const char* sw = sa + G::W_OFF;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const int chunk = ks * 4 + fg;
#pragma unroll
        for (int i = 0; i < TN; ++i) wf[ks][i] = *reinterpret_cast<const frag*>(sw + G::off(wrow0 + i * 16, chunk));
#pragma unroll
        for (int j = 0; j < TM; ++j) af[ks][j] = *reinterpret_cast<const frag*>(sa + G::off(arow0 + j * 16, chunk));
      }
    };
    auto barrier = [] {
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
    };
    constexpr int kVmSteady = (((STAGES - 2) * L) & 15) | ((((STAGES - 2) * L) >> 4) << 14) | 0x70 | 0xF00;
    constexpr int kVm0 = 0x70 | 0xF00;
    constexpr int kLgkm0 = 0xC07F;
    const int n = k1 - k0;
#pragma unroll
    for (int s = 0; s < STAGES - 1; ++s)
      if (s < n) stage(s, (k0 + s) * BK);
    if (n >= STAGES - 1) __builtin_amdgcn_s_waitcnt(kVmSteady);
    else __builtin_amdgcn_s_waitcnt(kVm0);
    barrier();
    if (grp == 1) barrier();
    int buf = 0;
    for (int kt = 0; kt < n; ++kt) {
      read_tile(buf);
      const bool steady = kt + STAGES - 1 < n;
      if (steady) stage((kt + STAGES - 1) % STAGES, (k0 + kt + STAGES - 1) * BK);
      __builtin_amdgcn_s_waitcnt(kLgkm0);
      if (steady) __builtin_amdgcn_s_waitcnt(kVmSteady);
      else __builtin_amdgcn_s_waitcnt(kVm0);
      barrier();
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
#pragma unroll
        for (int i = 0; i < TN; ++i)
#pragma unroll
          for (int j = 0; j < TM; ++j) acc[i][j] = MfmaOp<T>::mma(wf[ks][i], af[ks][j], acc[i][j]);
      __builtin_amdgcn_s_setprio(0);
      barrier();
      buf = buf == STAGES - 1 ? 0 : buf + 1;
    }
    if (grp == 0) barrier();
    __syncthreads();   // every wave is past its last read: the LDS may be restaged / reused
  };
  auto zero_acc = [&] {
#pragma unroll
    for (int i = 0; i < TN; ++i)
#pragma unroll
      for (int j = 0; j < TM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  };
  auto epilogue = [&](int tm, int tn) {
    const int m0 = tm * BM, n0 = tn * BN;
    auto go = [&](auto actf) {
      staged_epilogue<T, OutT, BM, BN, SB, G::NT, TM, TN, HAS_BIAS, HAS_RES, decltype(actf)>(
          smem, acc, grp * GBM + wm * WM, wn * WN, m0, n0, M, N, C, ldc, bias, R, ldr, alpha, actf);
    };
    switch (act) {
      case ACT_GELU: go([](float x) { return apply_act<ACT_GELU>(x); }); break;
      case ACT_RELU: go([](float x) { return apply_act<ACT_RELU>(x); }); break;
      case ACT_SILU: go([](float x) { return apply_act<ACT_SILU>(x); }); break;
      case ACT_GELU_TANH: go([](float x) { return apply_act<ACT_GELU_TANH>(x); }); break;
      default: go([](float x) { return x; }); break;
    }
  };
  // ---- walk this range's segments ----
  // the workgroup whose range holds unit x (ranges are non-empty: U >= grid)
  auto range_of = [&](int64_t x) -> int {
    int c = (int)((x * Gn) / U);
    while (c + 1 < Gn && ubeg(c + 1) <= x) ++c;
    while (c > 0 && ubeg(c) > x) --c;
    return c;
  };
  int64_t u = u0;
  while (u < u1) {
    const int t = (int)(u / nk);
    const int k0 = (int)(u - (int64_t)t * nk);
    const int64_t tbeg = (int64_t)t * nk, tend = tbeg + nk;
    const int k1 = (int)((u1 < tend ? u1 : tend) - tbeg);
    const int tm = t / tiles_n, tn = t - tm * tiles_n;
    zero_acc();
    run_segment(tm, tn, k0, k1);
    if (k0 == 0 && k1 == nk) {
      epilogue(tm, tn);
    } else {
      // tile t is split over ranges c_first (its head) .. c_last: whoever
      // arrives LAST folds the others' partials in and stores the tile
      const int c_first = range_of(tbeg), c_last = range_of(tend - 1);
      const int nseg = c_last - c_first + 1;
      int* cnt = ws.state + t;
      const int my_slot = k0 > 0 ? 2 * w : 2 * w + 1;
      if (tid == 0) {
        // every other segment already published: last without writing a partial
        const int seen = __hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *bcast = seen == nseg - 1 ? 1 : 0;
      }
      __syncthreads();
      bool last = *bcast != 0;
      __syncthreads();
      if (!last) {
        const uint32_t base = (uint32_t)((size_t)my_slot * NACC4 * G::NT * 16);
#pragma unroll
        for (int i = 0; i < TN; ++i)
#pragma unroll
          for (int j = 0; j < TM; ++j) sk_store16(psrc, base + (uint32_t)(((i * TM + j) * G::NT + tid) * 16), acc[i][j]);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) {
          const int prev = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          *bcast = prev == nseg - 1 ? 1 : 0;
        }
        __syncthreads();
        last = *bcast != 0;
        __syncthreads();
      }
      if (last) {
        if (tid == 0) __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // clean for the next launch
        for (int c = c_first; c <= c_last; ++c) {
          if (c == w) continue;
          const int slot = c == c_first ? 2 * c + 1 : 2 * c;
          const uint32_t base = (uint32_t)((size_t)slot * NACC4 * G::NT * 16);
#pragma unroll
          for (int i = 0; i < TN; ++i)
#pragma unroll
            for (int j = 0; j < TM; ++j) acc[i][j] += sk_load16(psrc, base + (uint32_t)(((i * TM + j) * G::NT + tid) * 16));
        }
        epilogue(tm, tn);
      }
    }
    u = tbeg + k1;
  }
}

// Workspace layout (independent of the grid, so one zeroed buffer serves every
// tile / grid choice): one arrival counter per tile in the first 64 KiB, the
// f32 partial tiles after it.
constexpr int kSkMaxGrid = 1024;
constexpr int kSkMaxTiles = 16384;
constexpr size_t kSkHeader = 65536;   // one arrival counter per tile
template <int BM, int BN>
inline size_t gemm_sk_workspace_bytes(int grid) {
  return kSkHeader + 2 * (size_t)grid * BM * BN * 4;   // two partial slots per range (tail, head)
}

inline SkWorkspace sk_workspace_from(void* p) {
  char* b = static_cast<char*>(p);
  SkWorkspace w;
  w.state = reinterpret_cast<int*>(b);
  w.part = reinterpret_cast<float*>(b + kSkHeader);
  return w;
}

// The workspace must be zeroed once before its first launch and never be used
// by two launches at the same time (one per stream).
template <typename T, typename OutT, int NW, int BM, int BN, int GM, int GN, int STAGES, int BK = 64>
void launch_gemm_sk(const T* A, int lda, const T* W, int ldw, OutT* C, int ldc, const T* bias, const T* R, int ldr,
                    int M, int N, int K, float alpha, int act, void* workspace, int grid, hipStream_t s) {
  const int64_t tiles = (int64_t)((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  const int64_t units = tiles * ((K + BK - 1) / BK);
  if (units < grid) grid = (int)units;                  // every range non-empty
  if (grid < 1 || grid > kSkMaxGrid || tiles > kSkMaxTiles || workspace == nullptr)
    throw std::runtime_error("gemm_sk: bad grid / workspace");
  const SkWorkspace ws = sk_workspace_from(workspace);
  const dim3 g(grid), block(64 * NW);
  if (bias && R)
    hipLaunchKernelGGL((gemm_sk_kernel<T, OutT, NW, BM, BN, GM, GN, STAGES, true, true, BK>), g, block, 0, s, A, lda, W,
                       ldw, C, ldc, bias, R, ldr, M, N, K, alpha, act, ws);
  else if (bias)
    hipLaunchKernelGGL((gemm_sk_kernel<T, OutT, NW, BM, BN, GM, GN, STAGES, true, false, BK>), g, block, 0, s, A, lda, W,
                       ldw, C, ldc, bias, R, ldr, M, N, K, alpha, act, ws);
  else if (R)
    hipLaunchKernelGGL((gemm_sk_kernel<T, OutT, NW, BM, BN, GM, GN, STAGES, false, true, BK>), g, block, 0, s, A, lda, W,
                       ldw, C, ldc, bias, R, ldr, M, N, K, alpha, act, ws);
  else
    hipLaunchKernelGGL((gemm_sk_kernel<T, OutT, NW, BM, BN, GM, GN, STAGES, false, false, BK>), g, block, 0, s, A, lda,
                       W, ldw, C, ldc, bias, R, ldr, M, N, K, alpha, act, ws);
}

}  // namespace rdb
