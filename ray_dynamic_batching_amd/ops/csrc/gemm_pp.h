// "Ping-pong" MFMA GEMM for gfx950: the serving GEMMs of BERT / ViT / Llama
// prefill (M = 1k..8k rows, N, K = 768..4096) at one or two blocks per CU.
//
//   C[m, n] = act(alpha * sum_k A[m, k] * W[n, k] + bias[n] + R[m, n])
//
// Why a second GEMM body next to gemm_core.h: that kernel reads every K-tile's
// fragments and runs its MFMAs in the same wave, so a SIMD's matrix pipe idles
// while its waves wait on LDS reads and barriers (PMC: 14-22 % of the MFMA peak
// on the BERT shapes).  Here the block's waves form TWO GROUPS that split the
// tile's rows, and group 1 runs one barrier interval behind group 0
// (MI355X_MICROARCH.md "Two waves per SIMD": each SIMD alternates one wave in a
// matrix segment with its partner in a load segment):
//
//   interval i   : group 0 = MFMAs of tile k      | group 1 = LDS reads of tile k (+ DMA issue)
//   interval i+1 : group 0 = reads of tile k+1    | group 1 = MFMAs of tile k
//
// Each group owns (BM/2) x BN of the output; its GM x GN waves own
// (BM/2/GM) x (BN/GN) each.  Staging: both operands by LDS-DMA (buffer_load ...
// lds, 16 B per lane, source-side XOR swizzle, out-of-range -> 0), STAGES LDS
// buffers, tile k+STAGES-1 issued during tile k's read interval, retired with a
// counted vmcnt (never 0 in steady state) and raw s_barrier (no __syncthreads:
// its fence would drain the DMA).  Hazard bookkeeping (per wave, interval =
// between two consecutive block barriers):
//   RAW: every wave retires ITS pieces of tile k+1 at the end of its read
//        interval of tile k (vmcnt((STAGES-2) * loads)); group 1 does that one
//        interval later than group 0, i.e. before the barrier after which
//        group 0 reads tile k+1.
//   WAR: tile k+STAGES-1 overwrites buffer (k-1) % STAGES; its last reader
//        (group 1, read interval of tile k-1) drained its ds_reads (lgkmcnt(0))
//        before the barrier that starts group 0's read interval of tile k, in
//        which the first overwrite is issued.
// Both groups execute the same number of s_barrier: group 1 one extra at the
// start, group 0 one extra at the end.
#pragma once
// Included by gemm_core.h (after the shared helpers, before the tile table);
// not meant to be included on its own.

// RDB_PP_LATE_PCT (A/B builds): share of a wave's DMA pieces per K-tile issued in
// the matrix interval; -1: half on the BK 64 tiles, none on the BK 32 ones.
// Default 0: the lab gain on the BK 64 tiles (-4..6 % alone, -2.5..4 % on two
// streams) did not carry into the engines -- BERT 34.77k +- 0.40 vs 34.93k +- 0.20,
// ResNet-50 tie, Llama-3-8B prefill +3 % (profiles/gemm_lab_r5_late_dma.txt,
// profiles/ab_r5_late_dma.json)
#ifndef RDB_PP_LATE_PCT
#define RDB_PP_LATE_PCT 0
#endif

namespace rdb {

#ifdef RDB_PP_STAMPS
__device__ unsigned long long* rdb_pp_stamps;
#endif

template <int NW, int BM, int BN, int BK_>
struct PPGeom {
  static constexpr int BK = BK_;                             // 32 or 64
  static constexpr int NT = 64 * NW;
  static constexpr int ROWB = BK * 2;                        // LDS bytes per tile row
  static constexpr int CPR = BK / 8;                         // 16-B chunks per row
  static constexpr int PR = 1024 / ROWB;                     // rows per 1-KiB DMA piece
  static constexpr int A_PIECES = BM / PR;
  static constexpr int W_PIECES = (BN + PR - 1) / PR;
  static constexpr int A_PW = A_PIECES / NW;                 // pieces per wave
  static constexpr int W_PW = (W_PIECES + NW - 1) / NW;      // rounded up: surplus pieces go to a dummy slot
  static constexpr bool DUMMY = W_PW * NW != W_PIECES;       // (every wave issues the same count: one vmcnt)
  static constexpr int LOADS = A_PW + W_PW;                  // DMA instructions per wave per tile
  static constexpr int W_OFF = BM * ROWB;
  static constexpr int DUMMY_OFF = W_OFF + W_PIECES * 1024;
  static constexpr int STAGE_BYTES = DUMMY_OFF + (DUMMY ? 1024 : 0);
  static_assert(BK == 32 || BK == 64, "BK 32 or 64");
  static_assert(BM % (PR * NW) == 0, "A tile must split into whole pieces per wave");
  // XOR swizzle of the 16-B chunk index so that every lane group of a
  // ds_read_b128 hits 16 distinct bank quads.  The groups are NOT 16
  // consecutive lanes (MI355X_MICROARCH.md §LDS): group 0 = lanes {0-3, 12-15,
  // 20-27}, i.e. fragment rows 0-3 and 12-15 of chunk c plus rows 4-11 of chunk
  // c^1 (group 1 the complement).  128-B rows pair up per bank row ->
  // chunk ^ ((row>>1)&7) is conflict-free for these groups.  64-B rows come four
  // per bank row: with q = (row>>2)&3 the four rows sharing a bank quad column
  // need {s(0), s(3), 1^s(1), 1^s(2)} and {s(1), s(2), 1^s(0), 1^s(3)} distinct;
  // s(q) = q (the old form) gives a 2-way conflict on every read (PMC round 3:
  // 53 % of the BK32 FFN-up kernel's LDS cycles), s = {0, 2, 3, 1} gives none.
  static __device__ __forceinline__ int swz(int row) {
#ifdef RDB_PP_SWZ_LEGACY   // A/B build only: the round-3 conflicting BK32 form
    return BK == 64 ? ((row >> 1) & 7) : ((row >> 2) & 3);
#else
    return BK == 64 ? ((row >> 1) & 7) : ((0x78 >> (((row >> 2) & 3) * 2)) & 3);
#endif
  }
  static __device__ __forceinline__ int off(int row, int chunk) { return row * ROWB + ((chunk ^ swz(row)) << 4); }
};

// Implicit-GEMM convolution operand (CONV instantiations): A is the im2col view
// of an NHWC f16 image, A[m, k] = x[n, p*stride - pad + r, q*stride - pad + s, c]
// with m = (n, p, q), k = (r, s, c).  C % BK == 0, so every K-tile lies inside one
// filter tap: the tap (r, s) and channel offset are block-uniform per K-tile, and
// each lane's 16-B DMA piece is one contiguous channel chunk of one input pixel
// (padding -> kOOB -> zero fill).  The 9 taps of a 3x3 conv re-read the image
// through L2 (the patch is L2-resident), never through an im2col buffer.
struct ConvGeom {
  int H, W, C, S, stride, pad, P, Q;
  uint32_t img_bytes;   // N * H * W * C * 2: the A buffer resource's extent
};

// OCC = waves per SIMD the register budget must allow: 2 = one 8-wave block
// per CU (<= 256 VGPRs), 4 = two co-resident blocks (<= 128 VGPRs; the tile's
// LDS must then fit twice in 160 KiB)
// EPI: 0, EPI_SWG (SwiGLU) or an EPI_STG LayerNorm mode (gemm_core.h): LN operands
// are staged in LDS after the bias by the prologue and applied by the staged epilogue.
// CONV: A is the im2col view described by `cv` (lda unused).  SK: the launch may
// split K over gridDim.y (ln.sk_* : the gemm_core.h split-K hand-off).
template <typename T, typename OutT, int NW, int BM, int BN, int GM, int GN, int STAGES, bool HAS_BIAS, bool HAS_RES,
          int BK_ = 64, int OCC = 2, int EPI = 0, bool CONV = false, bool SK = CONV>
__global__ void __launch_bounds__(64 * NW, OCC)
gemm_pp_kernel(const T* __restrict__ A, int lda, const T* __restrict__ W, int ldw, OutT* __restrict__ C, int ldc,
               const T* __restrict__ bias, const T* __restrict__ R, int ldr, int M, int N, int K, float alpha,
               int act, LnEpi ln, ConvGeom cv) {
  typedef PPGeom<NW, BM, BN, BK_> G;
  constexpr int BK = G::BK;
  constexpr int KS = BK / 32;                // MFMA k-steps per tile
  constexpr int GW = NW / 2;                 // waves per group
  static_assert(GM * GN == GW, "group wave layout");
  constexpr int GBM = BM / 2;                // rows per group
  constexpr int WM = GBM / GM, WN = BN / GN;
  constexpr int TM = WM / 16, TN = WN / 16;
  static_assert(WM % 16 == 0 && WN % 16 == 0, "wave tile must be whole 16x16 fragments");
  constexpr int L = G::LOADS;
  static_assert(STAGES >= 3 && (STAGES - 2) * L < 64, "pipeline depth / vmcnt field");
  typedef typename MfmaOp<T>::frag frag;

  // staging buffers, then the tile's bias as f32 (read by the epilogue)
  constexpr int BIAS_OFF = STAGES * G::STAGE_BYTES;
  constexpr int LN_OFF = BIAS_OFF + (HAS_BIAS ? BN * 4 : 0);
  constexpr bool SWG = EPI == EPI_SWG;       // SwiGLU instantiation: plain epilogue otherwise
  constexpr int LEPI = SWG ? 0 : EPI;
  constexpr int LN_BYTES = LEPI ? LnLds<BM, BN>::BYTES : 0;
  static_assert(LEPI == 0 || (LEPI & EPI_STG), "ping-pong tiles: plain, SwiGLU or staged-LN epilogues");
  static_assert(!SWG || (!HAS_RES && BN % 16 == 0), "ping-pong SwiGLU: no residual, BN % 16 == 0");
  __shared__ __attribute__((aligned(16))) char smem[LN_OFF + LN_BYTES];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int grp = wid / GW, gw = wid % GW;
  const int wm = gw / GN, wn = gw % GN;
  const int wid_u = __builtin_amdgcn_readfirstlane(wid);

  const int tiles_n = (N + BN - 1) / BN, tiles_m = (M + BM - 1) / BM;
  const int t = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  // Wide grids (>= 12 tile columns) walk their tiles in groups of 4 tile rows,
  // column-major inside a group: an XCD's contiguous chunk of tiles is then a
  // 4 x (chunk / 4) block, so its L2 holds fewer distinct A and W panels
  // (profiles/gemm_lab_r5_group.txt: FFN-up -2..3 %, 4096^3 -3 %; narrow grids
  // such as N = 768 keep the row-major walk)
  int tile_m, tile_n;
  if (tiles_n >= 12 && tiles_m >= 8) {
    const int gsize = 4 * tiles_n;
    const int g = t / gsize, first = 4 * g;
    const int gm = tiles_m - first < 4 ? tiles_m - first : 4;
    const int r = t - g * gsize;
    tile_m = first + r % gm;
    tile_n = r / gm;
  } else {
    tile_m = t / tiles_n;
    tile_n = t - tile_m * tiles_n;
  }
  const int m0 = tile_m * BM, n0 = tile_n * BN;

  // ---- DMA addressing (wave wid_u owns A pieces [wid*A_PW, ...) and W pieces [wid*W_PW, ...)) ----
  const __amdgpu_buffer_rsrc_t asrc =
      CONV ? make_rsrc(A, cv.img_bytes)
           : make_rsrc(A, (uint32_t)((size_t)(M - 1) * lda * sizeof(T) + (size_t)K * sizeof(T)));
  const __amdgpu_buffer_rsrc_t wsrc = make_rsrc(W, (uint32_t)((size_t)(N - 1) * ldw * sizeof(T) + (size_t)K * sizeof(T)));
  uint32_t aoff[G::A_PW], woff[G::W_PW];
  int ach[G::A_PW], wch[G::W_PW];
  // CONV: per piece the output pixel's top-left input corner (ah, aw) and its
  // element offset (corner pixel + this lane's channel chunk; may be negative
  // at the padding, never dereferenced there)
  constexpr int CA = CONV ? G::A_PW : 1;
  int ah[CA], aw[CA];
#pragma unroll
  for (int i = 0; i < G::A_PW; ++i) {
    const int row = (wid * G::A_PW + i) * G::PR + lane / G::CPR;
    ach[i] = (lane % G::CPR) ^ G::swz(row);
    const int gm = m0 + row;
    if constexpr (CONV) {
      const int pq = cv.P * cv.Q;
      const int n = gm / pq, rem = gm - n * pq;
      const int pp = rem / cv.Q, qq = rem - pp * cv.Q;
      ah[i] = gm < M ? pp * cv.stride - cv.pad : -(1 << 20);
      aw[i] = qq * cv.stride - cv.pad;
      aoff[i] = (uint32_t)(((n * cv.H + ah[i]) * cv.W + aw[i]) * cv.C + ach[i] * 8);
    } else {
      aoff[i] = gm < M ? (uint32_t)((size_t)gm * lda * sizeof(T)) : kOOB;
    }
  }
#pragma unroll
  for (int i = 0; i < G::W_PW; ++i) {
    const int row = (wid * G::W_PW + i) * G::PR + lane / G::CPR;
    wch[i] = (lane % G::CPR) ^ G::swz(row);
    const int gn = n0 + row;
    woff[i] = (row < BN && gn < N) ? (uint32_t)((size_t)gn * ldw * sizeof(T)) : kOOB;
  }
  auto wdst = [&](char* base, int i) -> char* {   // surplus pieces land in the dummy slot
    const int piece = wid_u * G::W_PW + i;
    return base + (piece < G::W_PIECES ? G::W_OFF + piece * 1024 : G::DUMMY_OFF);
  };
  // one DMA piece p of a K-tile (p < A_PW: A pieces, then W pieces); stage_rng
  // issues pieces [p0, p1) (compile-time bounds after inlining)
  auto stage_rng = [&](int buf, int k0, int p0, int p1) {
    char* base = smem + buf * G::STAGE_BYTES;
    if constexpr (CONV) {
      const int tap = k0 / cv.C, c0 = k0 - tap * cv.C;
      const int ur = tap / cv.S, us = tap - ur * cv.S;
      const int uoff = (ur * cv.W + us) * cv.C + c0;
#pragma unroll
      for (int i = 0; i < G::A_PW; ++i) {
        if (i < p0 || i >= p1) continue;
        const int h = ah[i] + ur, w = aw[i] + us;
        const bool ok = k0 < K && (unsigned)h < (unsigned)cv.H && (unsigned)w < (unsigned)cv.W;
        dma16(asrc, base + (wid_u * G::A_PW + i) * 1024,
              ok ? (uint32_t)(((int)aoff[i] + uoff) * (int)sizeof(T)) : kOOB);
      }
    } else {
#pragma unroll
      for (int i = 0; i < G::A_PW; ++i) {
        if (i < p0 || i >= p1) continue;
        const int gk = k0 + ach[i] * 8;
        dma16(asrc, base + (wid_u * G::A_PW + i) * 1024,
              (gk < K && aoff[i] != kOOB) ? aoff[i] + (uint32_t)(gk * sizeof(T)) : kOOB);
      }
    }
#pragma unroll
    for (int i = 0; i < G::W_PW; ++i) {
      if (G::A_PW + i < p0 || G::A_PW + i >= p1) continue;
      const int gk = k0 + wch[i] * 8;
      dma16(wsrc, wdst(base, i), (gk < K && woff[i] != kOOB) ? woff[i] + (uint32_t)(gk * sizeof(T)) : kOOB);
    }
  };
  auto stage = [&](int buf, int k0) {
    char* base = smem + buf * G::STAGE_BYTES;
    if constexpr (CONV) {
      // block-uniform tap of this K-tile
      const int tap = k0 / cv.C, c0 = k0 - tap * cv.C;
      const int ur = tap / cv.S, us = tap - ur * cv.S;
      const int uoff = (ur * cv.W + us) * cv.C + c0;
#pragma unroll
      for (int i = 0; i < G::A_PW; ++i) {
        const int h = ah[i] + ur, w = aw[i] + us;
        const bool ok = k0 < K && (unsigned)h < (unsigned)cv.H && (unsigned)w < (unsigned)cv.W;
        dma16(asrc, base + (wid_u * G::A_PW + i) * 1024,
              ok ? (uint32_t)(((int)aoff[i] + uoff) * (int)sizeof(T)) : kOOB);
      }
    } else {
#pragma unroll
      for (int i = 0; i < G::A_PW; ++i) {
        const int gk = k0 + ach[i] * 8;
        dma16(asrc, base + (wid_u * G::A_PW + i) * 1024,
              (gk < K && aoff[i] != kOOB) ? aoff[i] + (uint32_t)(gk * sizeof(T)) : kOOB);
      }
    }
#pragma unroll
    for (int i = 0; i < G::W_PW; ++i) {
      const int gk = k0 + wch[i] * 8;
      dma16(wsrc, wdst(base, i), (gk < K && woff[i] != kOOB) ? woff[i] + (uint32_t)(gk * sizeof(T)) : kOOB);
    }
  };

  f32x4 acc[TN][TM];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fg = lane >> 4;
  const int arow0 = grp * GBM + wm * WM + fr;   // this lane's fragment rows in the A / W tiles
  const int wrow0 = wn * WN + fr;
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
  // Late DMA pieces (RDB_PP_LATE_PCT % of a wave's L pieces per K-tile): issued
  // by the MATRIX interval, spread between its MFMAs, instead of the read
  // interval.  An LDS-DMA issue holds its wave for ~60 cycles among bare MFMAs
  // but 100-185 inside a read burst (MI355X_MICROARCH.md, LDS-DMA piece issue
  // cost), so a read interval carrying all L pieces outlasts the partner's
  // MFMAs.  Hazards: the late pieces of tile kt+STAGES-1 go to the buffer of
  // tile kt-1, whose last reader (group 1's read interval of kt-1) ended before
  // this group's matrix interval of kt began (both groups); they are retired
  // by the read interval of tile kt+STAGES-2 like the early ones (vmcnt counts
  // them in issue order), one or more barriers before any read of that tile.
  constexpr int NMF = KS * TN * TM;
  constexpr int LPCT = RDB_PP_LATE_PCT >= 0 ? RDB_PP_LATE_PCT : (BK == 64 ? 50 : 0);
  constexpr int LB = L * LPCT / 100 < L ? L * LPCT / 100 : L - 1;
  constexpr int LGAP = NMF / (LB + 1);
  auto mfma_tile = [&](bool late, int lbuf, int lk0) {
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int j = 0; j < TM; ++j) {
          acc[i][j] = MfmaOp<T>::mma(wf[ks][i], af[ks][j], acc[i][j]);
          if constexpr (LB > 0) {
            const int q = (ks * TN + i) * TM + j + 1;       // MFMAs issued so far
            if (q % LGAP == 0 && q / LGAP <= LB && late) stage_rng(lbuf, lk0, L - LB + q / LGAP - 1, L - LB + q / LGAP);
          }
        }
  };
  // sched_barrier(0) pins the intervals: no MFMA may be hoisted into a read
  // interval (or LDS read sunk into a matrix interval) across a block barrier
  auto barrier = [] {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };
  // s_waitcnt immediates (gfx9 encoding: vmcnt lo[3:0] hi[15:14], expcnt[6:4], lgkmcnt[11:8])
  constexpr int kVmPro = (((STAGES - 2) * L) & 15) | ((((STAGES - 2) * L) >> 4) << 14) | 0x70 | 0xF00;
  // in the loop the late pieces of the newest tile are not issued yet when the read interval waits
  constexpr int kVmSteady = (((STAGES - 2) * L - LB) & 15) | ((((STAGES - 2) * L - LB) >> 4) << 14) | 0x70 | 0xF00;
  constexpr int kVm0 = 0x70 | 0xF00;
  constexpr int kLgkm0 = 0xC07F;            // lgkmcnt(0), vmcnt and expcnt at max

  // split-K (SK launches with gridDim.y > 1): this block runs K-tiles [kb, kb + nk)
  int kb = 0, nk = (K + BK - 1) / BK;
  if constexpr (SK) {
    if (gridDim.y > 1) {
      kb = blockIdx.y * ln.sk_kper;
      nk = min(ln.sk_kper, nk - kb);
    }
  }
#ifdef RDB_PP_STAMPS
  // diagnostic build only (bench/gemm_lab): per-block cycle stamps
  unsigned long long* stp = rdb_pp_stamps + (size_t)blockIdx.x * 8;
  const unsigned long long t_start = __builtin_amdgcn_s_memtime();
#endif
  if constexpr (HAS_BIAS) {
    // bias -> LDS (f32), visible after the prologue barrier.  Issued BEFORE the
    // first DMA: hipcc waits vmcnt(0) at the use of an ordinary load while an
    // LDS-DMA is in flight, which here would drain the prologue tiles.
    for (int q = tid; q < BN / 4; q += G::NT) {
      const __amdgpu_buffer_rsrc_t bsrc = make_rsrc(bias, (uint32_t)(N * sizeof(T)));
      const u32x2 raw = bload8(bsrc, (uint32_t)((n0 + q * 4 < N ? n0 + q * 4 : N) * sizeof(T)));
      const T* e = reinterpret_cast<const T*>(&raw);
      *reinterpret_cast<f32x4*>(smem + BIAS_OFF + q * 16) = f32x4{(float)e[0], (float)e[1], (float)e[2], (float)e[3]};
    }
  }
  if constexpr (LEPI != 0) ln_stage<T, LEPI, BM, BN, G::NT>(smem + LN_OFF, ln, m0, n0, M, N);
  // prologue: tiles 0 .. STAGES-2 in flight, tile 0 retired and visible
#pragma unroll
  for (int s = 0; s < STAGES - 1; ++s)
    if (s < nk) stage(s, (kb + s) * BK);
  if (nk >= STAGES - 1) __builtin_amdgcn_s_waitcnt(kVmPro);
  else __builtin_amdgcn_s_waitcnt(kVm0);
  barrier();
#ifdef RDB_PP_STAMPS
  const unsigned long long t_pro = __builtin_amdgcn_s_memtime();
#endif
  if (grp == 1) barrier();   // stagger: group 1 one interval behind

  int buf = 0;
  for (int kt = 0; kt < nk; ++kt) {
    // ---- read interval: fragments of tile kt, DMA of tile kt+STAGES-1 ----
    read_tile(buf);
    const bool steady = kt + STAGES - 1 < nk;
    const int nbuf = (kt + STAGES - 1) % STAGES, nk0 = (kb + kt + STAGES - 1) * BK;
    if (steady) stage_rng(nbuf, nk0, 0, L - LB);
    __builtin_amdgcn_s_waitcnt(kLgkm0);           // my reads of this buffer are done (WAR)
    if (steady) __builtin_amdgcn_s_waitcnt(kVmSteady);  // my pieces of tile kt+1 landed (RAW)
    else __builtin_amdgcn_s_waitcnt(kVm0);
    barrier();
    // ---- matrix interval (+ the late DMA pieces of tile kt+STAGES-1) ----
    __builtin_amdgcn_s_setprio(1);
    mfma_tile(steady, nbuf, nk0);
    __builtin_amdgcn_s_setprio(0);
    barrier();
    buf = buf == STAGES - 1 ? 0 : buf + 1;
  }
  if (grp == 0) barrier();
#ifdef RDB_PP_STAMPS
  const unsigned long long t_loop = __builtin_amdgcn_s_memtime();
#endif
  if constexpr (SK) {
    if (gridDim.y > 1) {
      // ---- split-K hand-off (mfma_gemm_kernel's protocol): a non-last split
      // stores its f32 partial (sc1), drains, meets at a barrier and one lane
      // bumps the tile's counter; the last arriver resets the counter, folds the
      // other partials in and runs the epilogue.  Nobody waits on anybody.
      __shared__ int sk_flag;
      const int splits = gridDim.y, z = blockIdx.y;
      int* cnt = ln.sk_cnt + t;
      const int nwg = tiles_m * tiles_n;
      const __amdgpu_buffer_rsrc_t psrc =
          make_rsrc(ln.sk_part, (uint32_t)((size_t)nwg * splits * BM * BN * sizeof(float)));
      auto slot_off = [&](int zz, int i, int j) {
        return (uint32_t)(((((size_t)t * splits + zz) * (TN * TM) + i * TM + j) * G::NT + tid) * 16);
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

  // ---- epilogue: LDS-staged, row-coalesced (launch_gemm_pp's caller guarantees
  // its requirements: 16-bit output, N % 8 == 0 (SwiGLU: N % 16, no residual), 16-B alignment) ----
  static_assert(sizeof(OutT) == 2, "ping-pong GEMM stores 16-bit outputs");
  constexpr int SB = STAGES * G::STAGE_BYTES;
  auto go = [&](auto actf) {
    staged_epilogue<T, OutT, BM, BN, SB, G::NT, TM, TN, HAS_BIAS, HAS_RES, decltype(actf), BIAS_OFF, LEPI,
                    LEPI ? LN_OFF : -1>(smem, acc, grp * GBM + wm * WM, wn * WN, m0, n0, M, N, C, ldc, bias, R, ldr,
                                       alpha, actf, &ln, tile_n);
  };
  if constexpr (SWG) {
    go(SwigluAct{});   // host-checked: no residual, N % 16 == 0 (gemm_pp_ok)
  } else {
    switch (act) {
      case ACT_GELU: go([](float x) { return apply_act<ACT_GELU>(x); }); break;
      case ACT_RELU: go([](float x) { return apply_act<ACT_RELU>(x); }); break;
      case ACT_TANH: go([](float x) { return apply_act<ACT_TANH>(x); }); break;
      case ACT_SILU: go([](float x) { return apply_act<ACT_SILU>(x); }); break;
      case ACT_GELU_TANH: go([](float x) { return apply_act<ACT_GELU_TANH>(x); }); break;
      case ACT_SIGMOID: go([](float x) { return apply_act<ACT_SIGMOID>(x); }); break;
      default: go([](float x) { return x; }); break;
    }
  }
#ifdef RDB_PP_STAMPS
  if (tid == 0) {
    stp[0] = t_start;
    stp[1] = t_pro;
    stp[2] = t_loop;
    stp[3] = __builtin_amdgcn_s_memtime();
  }
#endif
}

// Host-side precondition of the ping-pong kernels' staged epilogue.
inline bool gemm_pp_ok(int N, int ldc, int ldr, const void* C, const void* bias, const void* R, int act) {
  auto al = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  // SwiGLU: staged epilogue with N/2 output columns -- no residual, N % 16 == 0 (every pp tile's BN % 16 == 0)
  if (act == ACT_SWIGLU) return R == nullptr && N % 16 == 0 && ldc % 8 == 0 && al(C);
  return N % 8 == 0 && ldc % 8 == 0 && al(C) && (R == nullptr || (ldr % 8 == 0 && al(R)));
}

template <typename T, typename OutT, int NW, int BM, int BN, int GM, int GN, int STAGES, int BK = 64, int OCC = 2>
void launch_gemm_pp(const T* A, int lda, const T* W, int ldw, OutT* C, int ldc, const T* bias, const T* R, int ldr,
                    int M, int N, int K, float alpha, int act, hipStream_t s) {
  const int nwg = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  const dim3 grid(nwg), block(64 * NW);
  const LnEpi ln{};
  if (act == ACT_SWIGLU) {   // gemm_pp_ok: R == nullptr
    if (bias)
      hipLaunchKernelGGL((gemm_pp_kernel<T, OutT, NW, BM, BN, GM, GN, STAGES, true, false, BK, OCC, EPI_SWG>), grid, block,
                         0, s, A, lda, W, ldw, C, ldc, bias, R, ldr, M, N, K, alpha, act, ln, ConvGeom{});
    else
      hipLaunchKernelGGL((gemm_pp_kernel<T, OutT, NW, BM, BN, GM, GN, STAGES, false, false, BK, OCC, EPI_SWG>), grid, block,
                         0, s, A, lda, W, ldw, C, ldc, bias, R, ldr, M, N, K, alpha, act, ln, ConvGeom{});
    return;
  }
  if (bias && R)
    hipLaunchKernelGGL((gemm_pp_kernel<T, OutT, NW, BM, BN, GM, GN, STAGES, true, true, BK, OCC>), grid, block, 0, s, A, lda, W,
                       ldw, C, ldc, bias, R, ldr, M, N, K, alpha, act, ln, ConvGeom{});
  else if (bias)
    hipLaunchKernelGGL((gemm_pp_kernel<T, OutT, NW, BM, BN, GM, GN, STAGES, true, false, BK, OCC>), grid, block, 0, s, A, lda, W,
                       ldw, C, ldc, bias, R, ldr, M, N, K, alpha, act, ln, ConvGeom{});
  else if (R)
    hipLaunchKernelGGL((gemm_pp_kernel<T, OutT, NW, BM, BN, GM, GN, STAGES, false, true, BK, OCC>), grid, block, 0, s, A, lda, W,
                       ldw, C, ldc, bias, R, ldr, M, N, K, alpha, act, ln, ConvGeom{});
  else
    hipLaunchKernelGGL((gemm_pp_kernel<T, OutT, NW, BM, BN, GM, GN, STAGES, false, false, BK, OCC>), grid, block, 0, s, A, lda,
                       W, ldw, C, ldc, bias, R, ldr, M, N, K, alpha, act, ln, ConvGeom{});
}

// Split-K on a ping-pong tile (sk from splitk_epi: K-steps of 64 per split =
// BK 64 tiles only): gridDim.y = the number of non-empty splits.
template <typename T, typename OutT, int NW, int BM, int BN, int GM, int GN, int STAGES>
void launch_gemm_pp_sk(const T* A, int lda, const T* W, int ldw, OutT* C, int ldc, const T* bias, const T* R, int ldr,
                       int M, int N, int K, float alpha, int act, hipStream_t s, const LnEpi& sk) {
  const int nwg = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  const int nk = (K + 63) / 64;
  const dim3 grid(nwg, (nk + sk.sk_kper - 1) / sk.sk_kper), block(64 * NW);
  if (bias && R)
    hipLaunchKernelGGL((gemm_pp_kernel<T, OutT, NW, BM, BN, GM, GN, STAGES, true, true, 64, 2, 0, false, true>), grid,
                       block, 0, s, A, lda, W, ldw, C, ldc, bias, R, ldr, M, N, K, alpha, act, sk, ConvGeom{});
  else if (bias)
    hipLaunchKernelGGL((gemm_pp_kernel<T, OutT, NW, BM, BN, GM, GN, STAGES, true, false, 64, 2, 0, false, true>), grid,
                       block, 0, s, A, lda, W, ldw, C, ldc, bias, R, ldr, M, N, K, alpha, act, sk, ConvGeom{});
  else if (R)
    hipLaunchKernelGGL((gemm_pp_kernel<T, OutT, NW, BM, BN, GM, GN, STAGES, false, true, 64, 2, 0, false, true>), grid,
                       block, 0, s, A, lda, W, ldw, C, ldc, bias, R, ldr, M, N, K, alpha, act, sk, ConvGeom{});
  else
    hipLaunchKernelGGL((gemm_pp_kernel<T, OutT, NW, BM, BN, GM, GN, STAGES, false, false, 64, 2, 0, false, true>), grid,
                       block, 0, s, A, lda, W, ldw, C, ldc, bias, R, ldr, M, N, K, alpha, act, sk, ConvGeom{});
}

// The staged-LayerNorm modes (EPI_STG | ...) on a ping-pong tile.  LNA: no bias
// (folded), no residual; STATS with or without LNR: bias + residual.
template <typename T, typename OutT, int NW, int BM, int BN, int GM, int GN, int STAGES, int BK, int OCC, int EPI>
void launch_gemm_pp_ln(const T* A, int lda, const T* W, int ldw, OutT* C, int ldc, const T* bias, const T* R, int ldr,
                       int M, int N, int K, float alpha, int act, hipStream_t s, const LnEpi& ln) {
  const int nwg = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  constexpr bool RES = (EPI & (EPI_LNR | EPI_STATS)) != 0;
  hipLaunchKernelGGL((gemm_pp_kernel<T, OutT, NW, BM, BN, GM, GN, STAGES, RES, RES, BK, OCC, EPI>), dim3(nwg),
                     dim3(64 * NW), 0, s, A, lda, W, ldw, C, ldc, bias, R, ldr, M, N, K, alpha, act, ln, ConvGeom{});
}

}  // namespace rdb
