// Halo-tile 3x3 convolution (pad 1, stride 1 or 2, NHWC f16) on MFMA -- the
// ResNet-50 bottleneck 3x3 layers (the reference serves
// torchvision's ResNet-50, 293-project/profiling/resnet50_*_summary.csv).
// Stride 2 reads patch rows 2p + r / columns 2q + s (the formulas below are
// written for stride 1); split-K over channel blocks and a persistent
// resident-weight variant follow the streamed kernel.
//
// The im2col kernels (gemm_core.h Im2colLoader, gemm_pp.h CONV) stage one
// (tap, 64-channel) K-tile at a time: every output pixel's input is fetched
// from L2 nine times, and a 64-output-channel layer (stage 1) re-stages a
// 128-row A tile per 64 x 64 x 64 MFMA step.  Here a block owns TH whole output
// rows of G images x BN output channels and, per 64-channel block of the input:
//   * stages the (G x (TH+2) x (W+2)) input PATCH into LDS once (LDS-DMA,
//     zero-filled halo: out-of-image pixels are kOOB -> 0, no branches),
//   * streams the 9 taps' BN x 64 weight tiles through a 4-deep LDS ring, and
//   * feeds all 9 taps from the one patch: tap (r, s) of output pixel (p, q) is
//     patch row (p + r) * (W + 2) + q + s, i.e. the same A fragments shifted by
//     a block-uniform row offset.
// A K-step is one (channel block, tap): one raw s_barrier per step with a
// counted vmcnt (the tap's weight tile and -- at tap 0 -- the channel block's
// patch, issued 3 / 9 steps earlier), the next patch loads under the 9 taps of
// the current one.  The accumulators go through the LDS-staged coalesced
// epilogue of the other GEMMs (bias + residual + activation, 16-B row stores).
//
// 4 waves (one per SIMD), WGM x WGN wave grid, each wave TM x TN fragments of
// v_mfma_f32_16x16x32_f16 with the weight fragment as the MFMA A operand (the
// accumulator holds 4 consecutive output channels of one pixel per lane).
#include "gemm_core.h"
#include <stdexcept>

namespace rdb {

constexpr int kConvHaloFlag = 1 << 18;

struct HaloGeom {
  int N, H, W, C, K;   // input [N, H, W, C]; output [N, P, Q, K] (3x3, pad 1, stride S)
  int TH, G;           // output rows per tile; images per tile (G > 1 only with TH == P)
  int Wp, PR;          // patch width S * (Q - 1) + 3; patch rows G * THp * Wp
  int tiles_m;         // ceil(N / G) * ceil(P / TH)
  int cpb;             // split-K: 64-channel blocks per split (gridDim.y splits; cpb = C / 64 unsplit)
  int P, Q, S, THp;    // output rows / columns, stride, patch rows per image S * (TH - 1) + 3
};

// Diagnostic build only (bench/gemm_lab/halo_lab.hip defines RDB_HALO_STAMPS): per-wave
// s_memtime sums of the resident-weight kernel's loop segments, never in the real build.
#ifdef RDB_HALO_STAMPS
__device__ unsigned long long rdb_halo_stamps[4096][8];
#define HSTAMP(t)                                                                        \
  do {                                                                                   \
    __builtin_amdgcn_sched_barrier(0);                                                   \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");            \
    __builtin_amdgcn_sched_barrier(0);                                                   \
  } while (0)
#else
#define HSTAMP(t) \
  do {            \
  } while (0)
#endif

// Patch swizzle: 16-B chunk c of patch row r lives at slot c ^ (r & 7).  The GEMM tiles'
// c ^ ((r >> 1) & 7) (swz_off) is conflict-free for 16 consecutive 16-aligned fragment
// rows; the patch is read at rows prow + toff -- any offset, wrapping at the padded
// image width, and 2 apart at stride 2 -- where that key costs 1.7-3.0x the LDS cycles
// of a conflict-free ds_read_b128 and r & 7 1.1-2.0x (tools/lds_conflict_model_halo.py;
// PMC: 0.39-0.41 of the halo kernels' LDS cycles were bank conflicts,
// profiles/pmc_resnet50_forward_r6_cs1.json).  Weights keep swz_off.
__device__ __forceinline__ int pswz_off(int row, int chunk) { return row * 128 + ((chunk ^ (row & 7)) << 4); }
// the DMA side of it: lane slot (tid & 7) of patch row `row` loads chunk slot ^ (row & 7)
__device__ __forceinline__ int pdma_chunk(int tid, int row) { return (tid & 7) ^ (row & 7); }

template <int N>
__device__ __forceinline__ void vm_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt field is 6 bits");
  __builtin_amdgcn_s_waitcnt((N & 15) | ((N >> 4) << 14) | 0x70 | 0xF00);
}

// TM x TN fragments per wave on a WGM x WGN wave grid; PROWS patch rows per LDS
// patch buffer; NPB patch buffers (1: a single 64-channel block, C == 64, nothing
// to prefetch; 2: the next channel block's patch loads under this one's taps);
// WST weight-ring slots; OCC blocks per CU the LDS and register budgets allow
// (2 keeps a second block -- of this launch or another stream's -- resident to
// cover the patch latency and the epilogue).
// SK: split-K over the 64-channel blocks -- split z = blockIdx.y runs blocks
// [z * cpb, z * cpb + cpb); partial tiles go to `sk_part` and the last split of a
// tile to arrive at its `sk_cnt` counter adds the others and runs the epilogue
// (the gemm_core.h hand-off: sc1 stores / loads, relaxed agent-scope counter, the
// last arriver resets it).  For the small-image layers (ResNet-50 stages 3 / 4:
// 128 / 64 tiles of 256 px) whose tile grid leaves most CUs idle.
template <int TM, int TN, int WGM, int WGN, int PROWS, int NPB, int WST, int OCC, bool HAS_RES, bool SK = false>
__global__ void __launch_bounds__(256, OCC)
conv3x3_halo_kernel(const f16* __restrict__ x, const f16* __restrict__ w, f16* __restrict__ y,
                    const f16* __restrict__ bias, const f16* __restrict__ res, HaloGeom g, int act,
                    float* __restrict__ sk_part, int* __restrict__ sk_cnt) {
  static_assert(WGM * WGN == 4, "4 waves");
  constexpr int BK = 64, NT = 256;
  constexpr int WM = TM * 16, WN = TN * 16, BM = WGM * WM, BN = WGN * WN;
  static_assert(BN % 32 == 0 && PROWS % 32 == 0, "whole 4-wave DMA rounds (8 rows per wave instruction)");
  static_assert(NPB == 1 || NPB == 2, "patch buffers");
  static_assert(WST >= 3 && WST <= 8, "weight ring");
  constexpr int P_BYTES = PROWS * 128, W_BYTES = BN * 128;
  constexpr int LP = PROWS / 32, LW = BN / 32;     // DMA instructions per wave: patch, one tap's weights
  static_assert((WST - 2) * LW + LP < 64, "vmcnt");
  constexpr int W_OFF = NPB * P_BYTES;
  constexpr int SMEM = W_OFF + WST * W_BYTES;
  static_assert(SMEM * OCC <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(16))) char smem[SMEM];
  typedef f16x8 frag;

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WGN, wn = wid % WGN;
  const int wid_u = __builtin_amdgcn_readfirstlane(wid);
  const int fr = lane & 15, fg = lane >> 4;

  const int tiles_n = (g.K + BN - 1) / BN;
  const int t = xcd_remap(blockIdx.x, g.tiles_m * tiles_n);
  const int tile_m = t / tiles_n, tile_n = t - tile_m * tiles_n;
  const int rb_per_img = (g.P + g.TH - 1) / g.TH;
  const int grp = tile_m / rb_per_img, rb = tile_m - grp * rb_per_img;
  const int n_first = grp * g.G, p0 = rb * g.TH;
  const int PQ = g.P * g.Q;
  const int m0 = n_first * PQ + p0 * g.Q, n0 = tile_n * BN;
  const int bmv = g.G * min(g.TH, g.P - p0) * g.Q;   // the last row block of an image may be partial
  const int m_lim = min(g.N * PQ, m0 + bmv);
  const int Kg = 9 * g.C;
  const int THp = g.THp;

  const __amdgpu_buffer_rsrc_t xsrc = make_rsrc(x, (uint32_t)((size_t)g.N * g.H * g.W * g.C * 2));
  const __amdgpu_buffer_rsrc_t wsrc = make_rsrc(w, (uint32_t)((size_t)g.K * Kg * 2));

  // this lane's patch DMA pieces: rows (wid * LP + i) * 8 + lane / 8, i.e. 8 rows apart --
  // decomposed once into (image, patch row, patch column) and stepped, no per-piece division
  uint32_t poff[LP];
  {
    int row = dma_row(tid, LP, 0);
    int gi = row / (THp * g.Wp);
    int rem = row - gi * THp * g.Wp;
    int ph = rem / g.Wp, pw = rem - ph * g.Wp;
#pragma unroll
    for (int i = 0; i < LP; ++i) {
      const int ch = pdma_chunk(tid, row);
      const int n = n_first + gi, h = g.S * p0 - 1 + ph, ww = pw - 1;
      const bool ok = row < g.PR && n < g.N && (unsigned)h < (unsigned)g.H && (unsigned)ww < (unsigned)g.W;
      poff[i] = ok ? (uint32_t)((((n * g.H + h) * g.W + ww) * g.C) * 2 + ch * 16) : kOOB;
      row += 8;
      pw += 8;
      if (pw >= g.Wp) { pw -= g.Wp; ++ph; }     // Wp >= 9 > 8: one carry at most
      if (ph >= THp) { ph -= THp; ++gi; }
    }
  }
  // weight pieces: row n0 + r of W [K, 3, 3, C], 16-B chunk, at (tap 0, channel 0)
  uint32_t wof[LW];
#pragma unroll
  for (int i = 0; i < LW; ++i) {
    const int row = dma_row(tid, LW, i);
    const int ch = dma_chunk(tid, row);
    wof[i] = n0 + row < g.K ? (uint32_t)((n0 + row) * Kg * 2 + ch * 16) : kOOB;
  }
  // the A fragment rows: patch row of output pixel wm*WM + j*16 + fr at tap (0, 0)
  // (output (p, q) reads patch rows S*p + r, columns S*q + s)
  int prow[TM];
  {
    const int l0 = wm * WM + fr;
    const int per = g.TH * g.Q;
    int gi = l0 / per;
    int rem = l0 - gi * per;
    int p = rem / g.Q, q = rem - p * g.Q;
#pragma unroll
    for (int j = 0; j < TM; ++j) {
      prow[j] = wm * WM + j * 16 + fr < bmv ? gi * THp * g.Wp + g.S * (p * g.Wp + q) : 0;
      q += 16;
      while (q >= g.Q) { q -= g.Q; ++p; }
      while (p >= g.TH) { p -= g.TH; ++gi; }
    }
  }

  // this split's channel blocks [cb0, cb0 + ncb); cb below counts from cb0
  const int cb0 = SK ? (int)blockIdx.y * g.cpb : 0;
  const int ncb = SK ? min(g.cpb, g.C / BK - cb0) : g.C / BK, nsteps = ncb * 9;
  auto issue_w = [&](int s) {
    const int cb = s / 9, tap = s - cb * 9;
    char* base = smem + W_OFF + (s % WST) * W_BYTES;
    const uint32_t add = (uint32_t)((tap * g.C + (cb0 + cb) * BK) * 2);
#pragma unroll
    for (int i = 0; i < LW; ++i) dma16(wsrc, base + (wid_u * LW + i) * 1024, wof[i] == kOOB ? kOOB : wof[i] + add);
  };
  auto issue_p = [&](int cb) {
    char* base = smem + (NPB == 2 ? (cb & 1) * P_BYTES : 0);
    const uint32_t add = (uint32_t)((cb0 + cb) * BK * 2);
#pragma unroll
    for (int i = 0; i < LP; ++i) dma16(xsrc, base + (wid_u * LP + i) * 1024, poff[i] == kOOB ? kOOB : poff[i] + add);
  };

  f32x4 acc[TN][TM];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  issue_p(0);
#pragma unroll
  for (int s = 0; s < WST - 1; ++s)
    if (s < nsteps) issue_w(s);

  for (int s = 0; s < nsteps; ++s) {
    const int cb = s / 9, tap = s - cb * 9;
    // retire W(s) (and, older still, this block's patch): what stays in flight is the
    // younger weight tiles W(s+1 .. s+WST-2) and a patch issued at one of the last WST-1 steps
    const int nyw = min(WST - 2, nsteps - 1 - s);
    bool pp = false;
    if constexpr (NPB == 2) {
      int sp = s - (s % 9);                      // latest tap-0 step <= s ...
      if (sp == s) sp -= 9;                      // ... strictly before s
      pp = sp >= 0 && sp >= s - (WST - 1) && sp / 9 + 1 < ncb;
    }
    if (pp) {
      switch (nyw) {
        case 0: vm_wait<LP>(); break;
        case 1: vm_wait<LW + LP>(); break;
        case 2: vm_wait<2 * LW + LP>(); break;
        case 3: vm_wait<3 * LW + LP>(); break;
        case 4: vm_wait<4 * LW + LP>(); break;
        case 5: vm_wait<5 * LW + LP>(); break;
        default: vm_wait<(WST - 2) * LW + LP>(); break;
      }
    } else {
      switch (nyw) {
        case 0: vm_wait<0>(); break;
        case 1: vm_wait<LW>(); break;
        case 2: vm_wait<2 * LW>(); break;
        case 3: vm_wait<3 * LW>(); break;
        case 4: vm_wait<4 * LW>(); break;
        case 5: vm_wait<5 * LW>(); break;
        default: vm_wait<(WST - 2) * LW>(); break;
      }
    }
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    // refill the ring slot compute(s-1) read, and at a channel block's first tap the
    // other patch buffer (read by the previous block's taps, all done before the barrier)
    if (s + WST - 1 < nsteps) issue_w(s + WST - 1);
    if (NPB == 2 && tap == 0 && cb + 1 < ncb) issue_p(cb + 1);

    const char* pa = smem + (NPB == 2 ? (cb & 1) * P_BYTES : 0);
    const char* pw = smem + W_OFF + (s % WST) * W_BYTES;
    const int r3 = tap / 3;
    const int toff = r3 * g.Wp + (tap - r3 * 3);
    // both k-halves' fragments are read before the first MFMA: the second half's LDS
    // latency runs under the first half's MFMAs (k-step 1 is chunk fg + 4 = byte ^ 64)
    frag wf[2][TN], af[2][TM];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
      for (int i = 0; i < TN; ++i)
        wf[ks][i] = *reinterpret_cast<const frag*>(pw + swz_off(wn * WN + i * 16 + fr, ks * 4 + fg));
#pragma unroll
      for (int j = 0; j < TM; ++j)
        af[ks][j] = *reinterpret_cast<const frag*>(pa + (pswz_off(prow[j] + toff, fg) ^ (ks << 6)));
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int j = 0; j < TM; ++j) acc[i][j] = MfmaOp<f16>::mma(wf[ks][i], af[ks][j], acc[i][j]);
  }
  __syncthreads();
  if constexpr (SK) {
    if (gridDim.y > 1) {
      __shared__ int sk_flag;
      const int splits = gridDim.y, z = blockIdx.y;
      const int nwg = g.tiles_m * tiles_n;
      int* cnt = sk_cnt + t;
      const __amdgpu_buffer_rsrc_t psrc =
          make_rsrc(sk_part, (uint32_t)((size_t)nwg * splits * BM * BN * sizeof(float)));
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

  auto go = [&](auto actf) {
    staged_epilogue<f16, f16, BM, BN, SMEM, NT, TM, TN, true, HAS_RES, decltype(actf)>(
        smem, acc, wm * WM, wn * WN, m0, n0, m_lim, g.K, y, g.K, bias, res, g.K, 1.f, actf);
  };
  switch (act) {
    case ACT_RELU: go([](float v) { return apply_act<ACT_RELU>(v); }); break;
    case ACT_SILU: go([](float v) { return apply_act<ACT_SILU>(v); }); break;
    default: go([](float v) { return v; }); break;
  }
}

// ---- resident-weight persistent variant -------------------------------------------
// A block owns ONE output-channel slice (BN) and a contiguous run of `tpb` spatial
// tiles of it (host: tpb divides the tile rows, one run per block, <= one block per
// CU).  The slice's weights for all 9 taps and all channel blocks (9 * C/64 * BN rows
// of 128 B) are DMA'd into LDS once; per (tile, 64-channel block) unit only the
// input patch moves, through NPB rotating LDS buffers (NPB - 1 units in flight).
// One raw barrier per unit (9 taps x 2 MFMA k-steps between barriers), the
// epilogue stores straight from the accumulators (buffer stores, out-of-tile rows
// dropped by the range check: a fixed store count per wave, so the counted
// vmcnt waits stay exact -- loads, stores and LDS-DMA retire in issue order).
// For the layers whose weight slice fits LDS: ResNet-50 stage 1 (64 x 576 f16 =
// 72 KiB, the whole layer) and stage 2 in 32-channel slices.
template <int TM, int TN, int WGM, int WGN, int PROWS, int NPB, int WROWS>
__global__ void __launch_bounds__(256, 1)
conv3x3_halo_rw_kernel(const f16* __restrict__ x, const f16* __restrict__ w, f16* __restrict__ y,
                       const f16* __restrict__ bias, HaloGeom g, int act, int tpb) {
  static_assert(WGM * WGN == 4, "4 waves");
  constexpr int BK = 64;
  constexpr int WM = TM * 16, WN = TN * 16, BN = WGN * WN;
  static_assert(PROWS % 32 == 0 && WROWS % 32 == 0, "whole 4-wave DMA rounds");
  static_assert(NPB == 2 || NPB == 3, "patch buffers");
  constexpr int P_BYTES = PROWS * 128, W_BYTES = WROWS * 128;
  constexpr int LP = PROWS / 32, LWT = WROWS / 32;
  constexpr int PPT = (LP + 8) / 9;                 // patch pieces issued per tap
  constexpr int S = TM * TN;                        // epilogue stores per wave per tile
  static_assert(LP + 2 * S < 64 && LWT + 2 * LP < 64, "vmcnt");
  constexpr int SMEM = W_BYTES + NPB * P_BYTES;
  static_assert(SMEM <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(16))) char smem[SMEM];
  typedef f16x8 frag;

#ifdef RDB_HALO_STAMPS
  unsigned long long tk0 = 0, tk1 = 0;
  HSTAMP(tk0);
#endif
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WGN, wn = wid % WGN;
  const int wid_u = __builtin_amdgcn_readfirstlane(wid);
  const int fr = lane & 15, fg = lane >> 4;

  const int runs_per_slice = g.tiles_m / tpb;
  const int tile_n = blockIdx.x / runs_per_slice;
  const int tm_first = (blockIdx.x - tile_n * runs_per_slice) * tpb;
  const int n0 = tile_n * BN;
  const int HW = g.H * g.W, M = g.N * HW;
  const int bmv = g.G * g.TH * g.W;
  const int Kg = 9 * g.C, ncb = g.C / BK;
  const int THp = g.TH + 2, rb_per_img = g.H / g.TH;
  const int U = tpb * ncb;

  // bias of this lane's output channels (ordinary loads, before any LDS-DMA)
  float bv[TN][4];
  {
    const __amdgpu_buffer_rsrc_t bsrc = make_rsrc(bias, (uint32_t)(g.K * 2));
#pragma unroll
    for (int i = 0; i < TN; ++i) {
      const u32x2 raw = bload8(bsrc, (uint32_t)((n0 + wn * WN + i * 16 + fg * 4) * 2));   // K % 4 == 0: all or none
      const f16* e = reinterpret_cast<const f16*>(&raw);
#pragma unroll
      for (int q = 0; q < 4; ++q) bv[i][q] = (float)e[q];
    }
  }
  vm_wait<0>();      // the bias is in registers before the first LDS-DMA is counted
#ifdef RDB_HALO_STAMPS
  HSTAMP(tk1);
#endif

  const __amdgpu_buffer_rsrc_t xsrc = make_rsrc(x, (uint32_t)((size_t)M * g.C * 2));
  const __amdgpu_buffer_rsrc_t wsrc = make_rsrc(w, (uint32_t)((size_t)g.K * Kg * 2));
  const __amdgpu_buffer_rsrc_t ysrc = make_rsrc(y, (uint32_t)((size_t)M * g.K * 2));

  // the slice's weights: LDS row r = (cb * 9 + tap) * BN + n_local
  {
    const int wr = 9 * ncb * BN;
#pragma unroll 4
    for (int i = 0; i < LWT; ++i) {
      const int row = dma_row(tid, LWT, i);
      const int ch = dma_chunk(tid, row);
      const int ct = row / BN, nl = row - ct * BN;
      const int cb = ct / 9, tap = ct - cb * 9;
      const bool ok = row < wr && n0 + nl < g.K;
      dma16(wsrc, smem + (wid_u * LWT + i) * 1024,
            ok ? (uint32_t)(((n0 + nl) * Kg + tap * g.C + cb * BK) * 2 + ch * 16) : kOOB);
    }
  }

  // this lane's patch pieces (rows (wid*LP + i)*8 + lane/8, 8 rows apart): byte offset
  // relative to the tile's patch origin pixel (n_first, p0 - 1, -1), the patch row
  // (for the image-edge test) and image index; the column test is tile-independent
  int prel[LP], pph[LP], pgi[LP];
  unsigned pwok = 0;
  {
    int row = dma_row(tid, LP, 0);
    int gi = row / (THp * g.Wp);
    int rem = row - gi * THp * g.Wp;
    int ph = rem / g.Wp, pw = rem - ph * g.Wp;
#pragma unroll
    for (int i = 0; i < LP; ++i) {
      const int ch = pdma_chunk(tid, row);
      prel[i] = ((gi * g.H + ph) * g.W + pw) * g.C * 2 + ch * 16;
      pph[i] = ph;
      pgi[i] = row < g.PR ? gi : 1 << 20;             // rows past the patch: never valid
      if ((unsigned)(pw - 1) < (unsigned)g.W) pwok |= 1u << i;
      row += 8;
      pw += 8;
      if (pw >= g.Wp) { pw -= g.Wp; ++ph; }
      if (ph >= THp) { ph -= THp; ++gi; }
    }
  }
  // per-unit (wave-uniform) patch origin: image, first output row, byte base
  struct PatchOrg { int gmax, p0, base; };
  auto patch_org = [&](int u) {
    const int k = u / ncb, cb = u - k * ncb;
    const int tm = tm_first + k;
    const int grp = tm / rb_per_img;
    const int n_first = grp * g.G, p0 = (tm - grp * rb_per_img) * g.TH;
    return PatchOrg{g.N - n_first, p0, ((n_first * g.H + p0 - 1) * g.W - 1) * g.C * 2 + cb * BK * 2};
  };
  auto issue_piece = [&](const PatchOrg& o, int u, int i) {
    const int h = o.p0 - 1 + pph[i];
    const bool ok = ((pwok >> i) & 1) && (unsigned)h < (unsigned)g.H && pgi[i] < o.gmax;
    dma16(xsrc, smem + W_BYTES + (u % NPB) * P_BYTES + (wid_u * LP + i) * 1024, ok ? (uint32_t)(o.base + prel[i]) : kOOB);
  };
  auto issue_p = [&](int u) {
    const PatchOrg o = patch_org(u);
#pragma unroll
    for (int i = 0; i < LP; ++i) issue_piece(o, u, i);
  };
  // A fragment rows (tile-independent): patch row of output pixel wm*WM + j*16 + fr at tap (0, 0)
  int prow[TM];
  {
    const int l0 = wm * WM + fr;
    const int per = g.TH * g.W;
    int gi = l0 / per;
    int rem = l0 - gi * per;
    int p = rem / g.W, q = rem - p * g.W;
#pragma unroll
    for (int j = 0; j < TM; ++j) {
      prow[j] = wm * WM + j * 16 + fr < bmv ? gi * THp * g.Wp + p * g.Wp + q : 0;
      q += 16;
      while (q >= g.W) { q -= g.W; ++p; }
      while (p >= g.TH) { p -= g.TH; ++gi; }
    }
  }
  // swizzled LDS byte offsets of the A fragments at every tap (k-step 0; k-step 1 is ^ 64:
  // chunk fg + 4 = fg ^ 4 since fg < 4)
  int aoff[9][TM];
#pragma unroll
  for (int tap = 0; tap < 9; ++tap)
#pragma unroll
    for (int j = 0; j < TM; ++j) aoff[tap][j] = pswz_off(prow[j] + (tap / 3) * g.Wp + tap % 3, fg);
  // epilogue addressing (tile-independent parts): output row offsets and column offsets
  int lrow[TM];
#pragma unroll
  for (int j = 0; j < TM; ++j) lrow[j] = wm * WM + j * 16 + fr < bmv ? wm * WM + j * 16 + fr : -1;

  f32x4 acc[TN][TM];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  issue_p(0);
  if (NPB == 3 && U > 1) issue_p(1);
#ifdef RDB_HALO_STAMPS
  unsigned long long ts0 = 0, ta = 0, tb = 0, sw = 0, sb = 0, si = 0, sc = 0, se = 0;
  HSTAMP(ts0);
#endif

  for (int u = 0; u < U; ++u) {
#ifdef RDB_HALO_STAMPS
    HSTAMP(ta);
#endif
    const int k = u / ncb, cb = u - k * ncb;
    // retire P(u) (the weights are older still); younger in flight: the next
    // patch(es) already issued and the stores of the tiles that ended since
    const bool end1 = u >= 1 && (u - 1) % ncb == ncb - 1;   // unit u-1 ended a tile
    const bool end2 = u >= 2 && (u - 2) % ncb == ncb - 1;
    int code;
    if constexpr (NPB == 3) {
      const bool p1 = u + 1 < U;                             // P(u+1) issued before this wait
      code = (p1 ? 1 : 0) + 2 * ((end1 ? 1 : 0) + (end2 ? 1 : 0));
    } else {
      code = 2 * (end1 ? 1 : 0);
    }
    switch (code) {
      case 0: vm_wait<0>(); break;
      case 1: vm_wait<LP>(); break;
      case 2: vm_wait<S>(); break;
      case 3: vm_wait<LP + S>(); break;
      case 4: vm_wait<2 * S>(); break;
      default: vm_wait<LP + 2 * S>(); break;
    }
#ifdef RDB_HALO_STAMPS
    HSTAMP(tb);
    sw += tb - ta;
    ta = tb;
#endif
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
#ifdef RDB_HALO_STAMPS
    HSTAMP(tb);
    sb += tb - ta;
    ta = tb;
#endif
    // refill the buffer unit u-1 read (every wave is past it)
    const bool refill = u + NPB - 1 < U;
#ifdef RDB_HALO_STAMPS
    HSTAMP(tb);
    si += tb - ta;
    ta = tb;
#endif
    // 18 MFMA k-steps (9 taps x 2): the fragments of step st+1 are read while the
    // MFMAs of step st run (one wave per SIMD: nothing else hides the LDS latency),
    // and the next unit's patch pieces go out one per tap between them
    const char* pa = smem + W_BYTES + (u % NPB) * P_BYTES;
    const char* pwb = smem + cb * 9 * BN * 128;
    const PatchOrg nxt = patch_org(refill ? u + NPB - 1 : u);
    auto ld = [&](int st, frag (&wf)[TN], frag (&af)[TM]) {
      const int tap = st >> 1, chunk = (st & 1) * 4 + fg;
      const char* pw = pwb + tap * BN * 128;
#pragma unroll
      for (int i = 0; i < TN; ++i) wf[i] = *reinterpret_cast<const frag*>(pw + swz_off(wn * WN + i * 16 + fr, chunk));
#pragma unroll
      for (int j = 0; j < TM; ++j) af[j] = *reinterpret_cast<const frag*>(pa + (aoff[tap][j] ^ ((st & 1) << 6)));
    };
    auto mma = [&](const frag (&wf)[TN], const frag (&af)[TM]) {
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int j = 0; j < TM; ++j) acc[i][j] = MfmaOp<f16>::mma(wf[i], af[j], acc[i][j]);
    };
    {
      frag w0[TN], a0[TM], w1[TN], a1[TM];
      ld(0, w0, a0);
#pragma unroll
      for (int st = 0; st < 18; st += 2) {
        ld(st + 1, w1, a1);
#pragma unroll
        for (int pc = 0; pc < PPT; ++pc)
          if (refill && (st >> 1) * PPT + pc < LP) issue_piece(nxt, u + NPB - 1, (st >> 1) * PPT + pc);
        mma(w0, a0);
        if (st + 2 < 18) ld(st + 2, w0, a0);
        mma(w1, a1);
      }
    }

#ifdef RDB_HALO_STAMPS
    HSTAMP(tb);
    sc += tb - ta;
    ta = tb;
#endif
    if (cb == ncb - 1) {
      // epilogue of tile k: bias + activation, 8-B stores of 4 channels per lane
      const bool relu = act == ACT_RELU;
      const int tm = tm_first + k;
      const int grp = tm / rb_per_img;
      const int m0 = grp * g.G * HW + (tm - grp * rb_per_img) * g.TH * g.W;
#pragma unroll
      for (int j = 0; j < TM; ++j) {
        const int m = m0 + lrow[j];
        const bool mok = lrow[j] >= 0 && m < M;
#pragma unroll
        for (int i = 0; i < TN; ++i) {
          const int n = n0 + wn * WN + i * 16 + fg * 4;
          float v[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float a = acc[i][j][q] + bv[i][q];
            v[q] = relu ? fmaxf(a, 0.f) : a;                 // host: ReLU or none
          }
          const f16x4 o = {(f16)v[0], (f16)v[1], (f16)v[2], (f16)v[3]};
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, o), ysrc,
                                                mok && n < g.K ? (uint32_t)((m * g.K + n) * 2) : kOOB, 0, 0);
          acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
      }
    }
#ifdef RDB_HALO_STAMPS
    HSTAMP(tb);
    se += tb - ta;
#endif
  }
#ifdef RDB_HALO_STAMPS
  HSTAMP(tb);
  if (lane == 0 && blockIdx.x * 4 + wid < 4096) {
    unsigned long long* o = rdb_halo_stamps[blockIdx.x * 4 + wid];
    o[0] = tb - ts0; o[1] = sw; o[2] = tk1 - tk0; o[3] = ts0 - tk1; o[4] = sc; o[5] = se; o[6] = (unsigned long long)U; o[7] = tk0;
  }
#endif
}

// Tile variants (force_cfg = kConvHaloFlag | v):
//   v  TM TN WGM WGN  BM x BN  patch rows x buffers  ring  blocks/CU  ResNet-50 bs32 layer
//   0   4  4  4   1  256 x  64    352 x 1            4     2         stage 1 (56 x 56 x 64): 4 rows x 56
//   1   7  1  1   4  112 x  64    256 x 1            4     2         stage 1: 2 rows x 56 (896 blocks)
//   2   7  1  1   4  112 x  64    192 x 2            3     2         stage 2: 4 rows x 28; stage 3: 7 x 14; stage 4: 2 images
//   3   4  1  1   4   64 x  64     96 x 2            4     2         stage 4: one 7 x 7 image (256 blocks)
//   4   7  2  2   2  224 x  64    288 x 2            3     1         stage 2: 7 rows x 28; stage 3: one image
//   5   7  4  2   2  224 x 128    288 x 2            3     1         stage 2 / 3 with the whole 128-channel tile
//   6   2  2  2   2   64 x  64    192 x 3   resident weights (576 rows), persistent   stage 1: 1 row x 56
//   7   2  2  4   1  128 x  32    192 x 3   resident weights (576 rows), persistent   stage 2: 4 rows x 28, 32-ch slices
//   8   4  4  4   1  256 x  64    352 x 2   resident weights (576 rows), persistent   stage 1: 4 rows x 56 (160 KiB LDS)
//   9   4  4  4   1  256 x  64    352 x 2            4     1         stages 3 / 4 (a 14 x 14 image; four 7 x 7 images), split-K
//  10   4  2  1   4   64 x 128    288 x 2            3     1         stride 2: 2 rows x 28 of 56 x 56; 4 of 28; one 7 x 7
//  11   4  1  1   4   64 x  64    288 x 2            4     1         stride 2, 64-channel N tiles
// Split-K (force_cfg | splits << 8): the two-patch-buffer streamed tiles (2, 3, 4, 5, 9, 10, 11).
// Stride 2 (pad 1): the streamed tiles; output (p, q) reads patch rows 2p + r, columns 2q + s.
// (one patch buffer: a single 64-channel block, C == 64; resident weights: 9 * C/64 * BN <= 576 rows.
//  Measured and dropped: weights held in VGPRs per wave -- loading 72 KiB per wave from L2 costs more
//  than it saves, and above 256 VGPRs the fragments spill or bounce through AGPRs,
//  profiles/resnet50_conv_halo_r6.json)
constexpr int kNumHalo = 12;
constexpr int kHaloBM[kNumHalo] = {256, 112, 112, 64, 224, 224, 64, 128, 256, 256, 64, 64};
constexpr int kHaloBN[kNumHalo] = {64, 64, 64, 64, 64, 128, 64, 32, 64, 64, 128, 64};
constexpr int kHaloPM[kNumHalo] = {352, 256, 192, 96, 288, 288, 192, 192, 352, 352, 288, 288};
constexpr int kHaloNPB[kNumHalo] = {1, 1, 2, 2, 2, 2, 3, 3, 2, 2, 2, 2};
constexpr int kHaloWR[kNumHalo] = {0, 0, 0, 0, 0, 0, 576, 576, 576, 0, 0, 0};   // resident weight rows (0: streamed)

static bool halo_splittable(int v) { return kHaloNPB[v] == 2 && kHaloWR[v] == 0; }

// (TH, G) of variant v for an H x W input at stride S (pad 1; output P x Q): the most
// output rows (then images) whose pixels fit BM and whose patch -- S * (TH - 1) + 3 rows
// of S * (Q - 1) + 3 pixels -- fits the LDS patch buffer.  Stride 1: TH divides P;
// stride 2: the last row block of an image may be partial.
static bool halo_geom(int v, int N, int H, int W, int C, int S, int& TH, int& G) {
  const int bm = kHaloBM[v], pm = kHaloPM[v];
  TH = 0;
  G = 1;
  if (S != 1 && S != 2) return false;
  const int P = (H - 1) / S + 1, Q = (W - 1) / S + 1, Wp = S * (Q - 1) + 3;
  if (C % 64 != 0 || (kHaloNPB[v] == 1 && C != 64) || Wp < 9) return false;
  if (kHaloWR[v] && (S != 1 || 9 * (C / 64) * kHaloBN[v] > kHaloWR[v])) return false;
  for (int th = P; th >= 1; --th)
    if ((S == 2 || P % th == 0) && th * Q <= bm && (S * (th - 1) + 3) * Wp <= pm) { TH = th; break; }
  if (TH == 0) return false;
  const int THp = S * (TH - 1) + 3;
  if (TH == P)
    while (G < N && (G + 1) * P * Q <= bm && (G + 1) * THp * Wp <= pm) ++G;
  return true;
}

template <int TM, int TN, int WGM, int WGN, int PROWS, int NPB, int WST, int OCC>
static void launch_halo(const HaloGeom& g, const f16* x, const f16* w, f16* y, const f16* bias, const f16* res, int act,
                        hipStream_t s, int eff, float* part, int* cnt) {
  constexpr int BN = WGN * TN * 16;
  const dim3 grid(g.tiles_m * ((g.K + BN - 1) / BN), eff), block(256);
  if constexpr (NPB == 2) {
    if (eff > 1) {
      if (res)
        hipLaunchKernelGGL((conv3x3_halo_kernel<TM, TN, WGM, WGN, PROWS, NPB, WST, OCC, true, true>), grid, block, 0, s,
                           x, w, y, bias, res, g, act, part, cnt);
      else
        hipLaunchKernelGGL((conv3x3_halo_kernel<TM, TN, WGM, WGN, PROWS, NPB, WST, OCC, false, true>), grid, block, 0, s,
                           x, w, y, bias, res, g, act, part, cnt);
      return;
    }
  }
  if (res)
    hipLaunchKernelGGL((conv3x3_halo_kernel<TM, TN, WGM, WGN, PROWS, NPB, WST, OCC, true>), grid, block, 0, s, x, w, y,
                       bias, res, g, act, part, cnt);
  else
    hipLaunchKernelGGL((conv3x3_halo_kernel<TM, TN, WGM, WGN, PROWS, NPB, WST, OCC, false>), grid, block, 0, s, x, w,
                       y, bias, res, g, act, part, cnt);
}

// Resident-weight launches: runs of tpb tiles (tpb divides the tile rows of a
// slice), at most one block per CU.
static int device_cus() {
  static int cus[64] = {0};
  int dev = 0;
  RDB_HIP_CHECK(hipGetDevice(&dev));
  if (dev < 0 || dev >= 64) return 256;
  if (cus[dev] == 0) RDB_HIP_CHECK(hipDeviceGetAttribute(&cus[dev], hipDeviceAttributeMultiprocessorCount, dev));
  return cus[dev];
}

static int rw_tpb(int tiles_m, int tiles_n, int cus) {
  const int want = (tiles_m * tiles_n + cus - 1) / cus;
  for (int tpb = want < 1 ? 1 : want; tpb <= tiles_m; ++tpb)
    if (tiles_m % tpb == 0) return tpb;
  return tiles_m;
}

template <int TM, int TN, int WGM, int WGN, int PROWS, int NPB, int WROWS>
static void launch_halo_rw(const HaloGeom& g, const f16* x, const f16* w, f16* y, const f16* bias, int act,
                           hipStream_t s) {
  constexpr int BN = WGN * TN * 16;
  const int tiles_n = (g.K + BN - 1) / BN;
  const int tpb = rw_tpb(g.tiles_m, tiles_n, device_cus());
  const dim3 grid(tiles_n * (g.tiles_m / tpb)), block(256);
  hipLaunchKernelGGL((conv3x3_halo_rw_kernel<TM, TN, WGM, WGN, PROWS, NPB, WROWS>), grid, block, 0, s, x, w, y, bias, g,
                     act, tpb);
}

int conv_halo_tiles_s(int v, int N, int H, int W, int C, int K, int S) {
  if (v < 0 || v >= kNumHalo) return -1;
  int TH, G;
  if (!halo_geom(v, N, H, W, C, S, TH, G)) return -1;
  const int P = (H - 1) / S + 1;
  return ((N + G - 1) / G) * ((P + TH - 1) / TH) * ((K + kHaloBN[v] - 1) / kHaloBN[v]);
}
int conv_halo_tiles(int v, int N, int H, int W, int C, int K) { return conv_halo_tiles_s(v, N, H, W, C, K, 1); }

// Splits that actually run for `splits` requested over C / 64 channel blocks (every split non-empty).
static int halo_eff_splits(int C, int splits, int& cpb) {
  const int ncb = C / 64;
  cpb = splits > 1 ? (ncb + splits - 1) / splits : ncb;
  return (ncb + cpb - 1) / cpb;
}

// Workspace bytes a split-K halo launch needs (0: the tile does not split / runs unsplit).
size_t conv_halo_ws_bytes(int v, int N, int H, int W, int C, int K, int splits, int S) {
  const int tiles = conv_halo_tiles_s(v, N, H, W, C, K, S);
  if (tiles <= 0 || splits < 2 || !halo_splittable(v)) return 0;
  int cpb;
  const int eff = halo_eff_splits(C, splits, cpb);
  if (eff < 2) return 0;
  return kSplitKHeader + (size_t)tiles * eff * kHaloBM[v] * kHaloBN[v] * sizeof(float);
}

void conv3x3_halo(int v, const void* x, const void* w, void* y, const void* bias, const void* res, int N, int H, int W,
                  int C, int K, int stride, int act, hipStream_t s, int splits, void* ws, size_t ws_bytes) {
  if (v < 0 || v >= kNumHalo) throw std::invalid_argument("conv2d_nhwc: unknown halo conv tile");
  if (C % 64 != 0 || K % 8 != 0 || bias == nullptr)
    throw std::invalid_argument("conv2d_nhwc: halo conv tiles need C % 64 == 0, K % 8 == 0 and a bias");
  if ((reinterpret_cast<uintptr_t>(y) | reinterpret_cast<uintptr_t>(res)) & 15)
    throw std::invalid_argument("conv2d_nhwc: halo conv tiles need 16-B aligned y / residual");
  if ((size_t)N * H * W * C * 2 >= (size_t(1) << 31) || (size_t)K * 9 * C * 2 >= (size_t(1) << 31))
    throw std::invalid_argument("conv2d_nhwc: halo conv operands must stay under 2 GiB");
  if (kHaloWR[v] && (res != nullptr || (act != ACT_NONE && act != ACT_RELU)))
    throw std::invalid_argument("conv2d_nhwc: resident-weight halo tiles: no residual, ReLU or no activation");
  HaloGeom g{N, H, W, C, K, 0, 1, 0, 0, 0, C / 64, (H - 1) / stride + 1, (W - 1) / stride + 1, stride, 0};
  if (!halo_geom(v, N, H, W, C, stride, g.TH, g.G))
    throw std::invalid_argument("conv2d_nhwc: halo conv tile " + std::to_string(v) + " does not fit this conv");
  g.Wp = stride * (g.Q - 1) + 3;
  g.THp = stride * (g.TH - 1) + 3;
  g.PR = g.G * g.THp * g.Wp;
  g.tiles_m = ((N + g.G - 1) / g.G) * ((g.P + g.TH - 1) / g.TH);
  // split-K: only when the workspace holds every split's partial tiles, else unsplit
  int eff = 1;
  float* part = nullptr;
  int* cnt = nullptr;
  if (splits > 1) {
    if (!halo_splittable(v)) throw std::invalid_argument("conv2d_nhwc: halo conv tile " + std::to_string(v) + " has no split-K");
    const size_t need = conv_halo_ws_bytes(v, N, H, W, C, K, splits, stride);
    const int tiles = conv_halo_tiles_s(v, N, H, W, C, K, stride);
    int cpb;
    const int e = halo_eff_splits(C, splits, cpb);
    if (need > 0 && ws != nullptr && need <= ws_bytes && tiles <= kSplitKMaxTiles &&
        need - kSplitKHeader <= (size_t(1) << 31)) {
      eff = e;
      g.cpb = cpb;
      cnt = static_cast<int*>(ws);
      part = reinterpret_cast<float*>(static_cast<char*>(ws) + kSplitKHeader);
    }
  }
  const f16 *xp = (const f16*)x, *wp = (const f16*)w, *bp = (const f16*)bias, *rp = (const f16*)res;
  f16* yp = (f16*)y;
  switch (v) {
    case 0: launch_halo<4, 4, 4, 1, 352, 1, 4, 2>(g, xp, wp, yp, bp, rp, act, s, 1, part, cnt); break;
    case 1: launch_halo<7, 1, 1, 4, 256, 1, 4, 2>(g, xp, wp, yp, bp, rp, act, s, 1, part, cnt); break;
    case 2: launch_halo<7, 1, 1, 4, 192, 2, 3, 2>(g, xp, wp, yp, bp, rp, act, s, eff, part, cnt); break;
    case 3: launch_halo<4, 1, 1, 4, 96, 2, 4, 2>(g, xp, wp, yp, bp, rp, act, s, eff, part, cnt); break;
    case 4: launch_halo<7, 2, 2, 2, 288, 2, 3, 1>(g, xp, wp, yp, bp, rp, act, s, eff, part, cnt); break;
    case 5: launch_halo<7, 4, 2, 2, 288, 2, 3, 1>(g, xp, wp, yp, bp, rp, act, s, eff, part, cnt); break;
    case 9: launch_halo<4, 4, 4, 1, 352, 2, 4, 1>(g, xp, wp, yp, bp, rp, act, s, eff, part, cnt); break;
    case 10: launch_halo<4, 2, 1, 4, 288, 2, 3, 1>(g, xp, wp, yp, bp, rp, act, s, eff, part, cnt); break;
    case 11: launch_halo<4, 1, 1, 4, 288, 2, 4, 1>(g, xp, wp, yp, bp, rp, act, s, eff, part, cnt); break;
    case 6: launch_halo_rw<2, 2, 2, 2, 192, 3, 576>(g, xp, wp, yp, bp, act, s); break;
    case 7: launch_halo_rw<2, 2, 4, 1, 192, 3, 576>(g, xp, wp, yp, bp, act, s); break;
    default: launch_halo_rw<4, 4, 4, 1, 352, 2, 576>(g, xp, wp, yp, bp, act, s); break;
  }
  RDB_HIP_CHECK(hipGetLastError());
}

}  // namespace rdb
