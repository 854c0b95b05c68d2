// Fused QKV projection + attention for short sequences (S <= 128, head dim 64):
// BERT-base / -large serving at seq 128 (reference: the HF BertSelfAttention
// the reference's BERT deployments run, SURVEY.md §2.7 -- there it is three
// GEMMs, a transpose and an SDPA kernel).
//
//   ctx[b, s, h, :] = softmax(Q_bh K_bh^T * scale + mask) V_bh,
//   [Q_bh | K_bh | V_bh] = X[b] @ Wp[h]^T + bp[h]
//
// One workgroup = one (sequence b, head h).  At S <= 128 the projection tile
// [128 tokens] x [q_h | k_h | v_h] = 128 x 192 holds EVERYTHING head h of
// sequence b needs, so the block
//   1. runs the MFMA GEMM main loop of gemm_core.h (LDS-DMA staging, 2 or 3
//      stages, counted vmcnt) over K = hidden with the head-major packed weight
//      Wp [H * 192, hidden] (rows h*192 + [0,64) = q_h, [64,128) = k_h,
//      [128,192) = v_h; ops.pack_qkv_heads builds it once);
//   2. parks Q, K (row-major, XOR-swizzled) and V^T in the now idle staging LDS
//      as bf16/f16 -- the same layouts and rounding point as the unfused path
//      (the projection output is rounded to the activation dtype there too);
//   3. runs the attention of attention.hip's single-key-block case on them
//      (S^T = K Q^T with lane-local softmax, O^T += V^T P^T) and stores ctx.
// The [B*S, 3*H*64] QKV activation is never written or re-read (19 MB per
// BERT-base layer at B = 32) and one kernel per layer disappears.
//
// Grid: B * H blocks, XCD-remapped so the H heads of one sequence (which share
// its 128 x hidden A panel) run on one XCD's L2.
//
// LNA = true: X holds RAW rows whose LayerNorm is folded into the weight
// (Wp = W * gamma, colsum = rowsum(Wp), bias_f = b + W beta; gemm_core.h
// "deferred-LayerNorm"): the block computes each token's (sum, sum of squares)
// from the A fragments of its own main loop (frag_stats) and corrects
//   P = rstd * (X Wp^T - mean * colsum) + bias_f;
// head 0's block stores the statistics to stats_out for the o-projection's
// LayerNorm-on-load of the same rows (the residual).  No LayerNorm kernel runs.
#include "gemm_core.h"
#include <stdexcept>

namespace rdb {

struct QkvLn {
  const float* colsum;   // [H*192], packed order
  const float* bias_f;   // [H*192]
  float* stats_out;      // [B*S, 2] (sum, sum of squares) of X's rows, row stride 2; may be null
  float inv_d, eps;
  const float* a_stats;  // LNA == 2: X's row statistics as partials [B*S][parts][2] (row stride a_ld floats)
  int a_ld, a_parts;
};

// SEQ = 2 (S == 128 only): one block = TWO consecutive sequences of one head, a
// 256 x 192 projection tile -- the head's W tile (192 x hidden) is staged once
// for two sequences, 30 % fewer bytes per FLOP through the per-CU L2 -> LDS
// path that bounds the projection; B*H/2 blocks.  Waves 0..3 then run the
// attention of the first sequence, 4..7 of the second.
// OCC (> 0) overrides the waves-per-SIMD register budget (4 = two co-resident
// 8-wave blocks per CU).
// LNA: 0 = plain; 1 = folded LayerNorm, X's row statistics computed in the main
// loop (frag_stats); 2 = folded LayerNorm, statistics given as the producer's
// per-N-tile partials (ln.a_stats; gemm_core.h EPI_STG | EPI_STATS) -- no
// statistics work in the main loop.
template <typename T, int NW, int STAGES, int LNA, int WGM_ = (NW == 8 ? 4 : 2), int SEQ = 1, int OCC = 0>
__global__ void __launch_bounds__(64 * NW, OCC > 0 ? OCC : (NW == 8 && (STAGES == 3 || SEQ == 2) ? 1 : 2))
qkv_attn_kernel(DenseParams ap, const T* __restrict__ W, const T* __restrict__ bias, int S, int H,
                const int* __restrict__ lens, T* __restrict__ out, int ld_out, float scale_log2e, QkvLn ln,
                const int* __restrict__ kids, int pad) {
  constexpr int BM = 128 * SEQ, BN = 192, BK = 64, D = 64;
  static_assert(SEQ == 1 || (SEQ == 2 && NW == 8), "two sequences per block: 8 waves");
  constexpr int WGM = WGM_, WGN = NW / WGM_;
  constexpr int NT = 64 * NW;
  constexpr int WM = BM / WGM, WN = BN / WGN;       // 32|64 x 96
  constexpr int TM = WM / 16, TN = WN / 16;
  constexpr int A_CH = BM * 8 / NT;                 // 16-B DMA pieces per thread per A tile
  constexpr int W_CH = BN / (8 * NW);               // ... per W tile (192 = 24 pieces)
  static_assert(BN % (8 * NW) == 0 && BM % (8 * NW) == 0, "DMA split");
  constexpr int kStage = (BM + BN) * BK * 2;        // 40 KiB
  constexpr int QT = BM / (16 * NW);                // 16-query tiles per wave in the attention phase
  constexpr int VT_LD = BM + 8;                     // V^T row (elements), +8: conflict-free 8-B reads
  constexpr int Q_OFF = 0, K_OFF = BM * D * 2, V_OFF = 2 * BM * D * 2;
  static_assert(V_OFF + D * VT_LD * 2 <= STAGES * kStage, "attention operands must fit the staging LDS");
  typedef typename MfmaOp<T>::frag frag;
  typedef T frag4 __attribute__((ext_vector_type(4)));

  __shared__ __attribute__((aligned(16))) char smem[STAGES * kStage];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WGN, wn = wid % WGN;
  const int fr = lane & 15, fg = lane >> 4;
  const int t = xcd_remap(blockIdx.x, gridDim.x);
  const int b = t / H, h = t - b * H;            // b: the block's first sequence / SEQ
  const int m0 = b * SEQ * S, n0 = h * BN;
  const int K = ap.K;

  // ---- 1. projection main loop (gemm_core.h's, fixed 128 x 192 tile) ----
  DenseLoader<T, A_CH> la;
  la.init(ap, tid, m0);
  const int N = H * BN;
  const __amdgpu_buffer_rsrc_t wsrc = make_rsrc(W, (uint32_t)((size_t)(N - 1) * K * sizeof(T) + (size_t)K * sizeof(T)));
  uint32_t woff[W_CH];
  int wch[W_CH];
#pragma unroll
  for (int i = 0; i < W_CH; ++i) {
    const int row = dma_row(tid, W_CH, i);
    wch[i] = dma_chunk(tid, row);
    woff[i] = (uint32_t)((size_t)(n0 + row) * K * sizeof(T));
  }
  const int wid_u = __builtin_amdgcn_readfirstlane(wid);
  auto stage = [&](int buf, int k0) {
    char* base = smem + buf * kStage;
#pragma unroll
    for (int i = 0; i < A_CH; ++i) dma16(la.rsrc, base + (wid_u * A_CH + i) * 1024, la.offset(i, k0));
#pragma unroll
    for (int i = 0; i < W_CH; ++i) {
      const int gk = k0 + wch[i] * 8;
      dma16(wsrc, base + BM * BK * 2 + (wid_u * W_CH + i) * 1024, gk < K ? woff[i] + (uint32_t)(gk * sizeof(T)) : kOOB);
    }
  };

  f32x4 acc[TN][TM];
#pragma unroll
  for (int i = 0; i < TN; ++i)
#pragma unroll
    for (int j = 0; j < TM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float st1[LNA ? TM : 1], st2[LNA ? TM : 1];
#pragma unroll
  for (int j = 0; j < (LNA ? TM : 1); ++j) st1[j] = st2[j] = 0.f;
  // LNA == 2: this lane's rows' partials, issued before the first DMA and summed
  // behind it (the wait for them is the one the first stage needs anyway)
  float2 xp[LNA == 2 ? TM * 8 : 1];
  if constexpr (LNA == 2) {
#pragma unroll
    for (int j = 0; j < TM; ++j) {
      const int m = m0 + wm * WM + j * 16 + fr;
      const float* row = ln.a_stats + (size_t)(m < ap.M ? m : ap.M - 1) * ln.a_ld;
#pragma unroll
      for (int p = 0; p < 8; ++p)
        xp[j * 8 + p] = p < ln.a_parts ? *reinterpret_cast<const float2*>(row + 2 * p) : float2{0.f, 0.f};
    }
  }
  auto sum_partials = [&] {
    if constexpr (LNA == 2) {
#pragma unroll
      for (int j = 0; j < TM; ++j)
#pragma unroll
        for (int p = 0; p < 8; ++p) {
          st1[j] += xp[j * 8 + p].x;
          st2[j] += xp[j * 8 + p].y;
        }
    }
  };
  auto compute = [&](int buf) {
    const char* sa = smem + buf * kStage;
    const char* sw = sa + BM * BK * 2;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      frag wf[TN], af[TM];
      const int chunk = ks * 4 + fg;
#pragma unroll
      for (int i = 0; i < TN; ++i) wf[i] = *reinterpret_cast<const frag*>(sw + swz_off(wn * WN + i * 16 + fr, chunk));
#pragma unroll
      for (int j = 0; j < TM; ++j) af[j] = *reinterpret_cast<const frag*>(sa + swz_off(wm * WM + j * 16 + fr, chunk));
      if constexpr (LNA == 1) {
#pragma unroll
        for (int j = 0; j < TM; ++j) frag_stats<T>(af[j], st1[j], st2[j]);   // k >= K reads as 0
      }
#pragma unroll
      for (int i = 0; i < TN; ++i)
#pragma unroll
        for (int j = 0; j < TM; ++j) acc[i][j] = MfmaOp<T>::mma(wf[i], af[j], acc[i][j]);
      if constexpr (TM * TN >= 16) __builtin_amdgcn_sched_barrier(0);
    }
  };

  // key length of this sequence: fetched before the main loop, used after it --
  // either a precomputed lens[b] or, with kids (the [B, S] token ids), counted
  // here from the ids (non-pad tokens, right padding): no separate lengths kernel
  // (SEQ = 2: S == 128, tokens [128*sq, 128*sq + 128) of the tile are sequence b*2 + sq;
  // wave w's attention queries lie in sequence w / 4)
  const int nseq = ap.M / S;
  const int my_seq = SEQ == 1 ? 0 : wid / (NW / SEQ);
  const int gseq = b * SEQ + my_seq < nseq ? b * SEQ + my_seq : nseq - 1;
  int kv_len = lens ? lens[gseq] : S;
  const int kid = (kids != nullptr && tid < SEQ * S && b * SEQ + tid / S < nseq) ? kids[(size_t)b * SEQ * S + tid] : pad;
  const int nk = (K + BK - 1) / BK;
  if constexpr (STAGES == 2) {
    stage(0, 0);
    sum_partials();
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
      if (kt + 1 < nk) stage((kt + 1) & 1, (kt + 1) * BK);
      compute(kt & 1);
      __syncthreads();
    }
  } else {
    constexpr int kLoads = A_CH + W_CH;
    constexpr int kWaitOne = (kLoads & 15) | ((kLoads >> 4) << 14) | 0x70 | 0xF00;
    constexpr int kWaitAll = 0x70 | 0xF00;
    static_assert(kLoads < 64, "vmcnt field");
    stage(0, 0);
    if (nk > 1) stage(1, BK);
    sum_partials();
    int buf = 0;
    for (int kt = 0; kt < nk; ++kt) {
      if (kt + 1 < nk) __builtin_amdgcn_s_waitcnt(kWaitOne);
      else __builtin_amdgcn_s_waitcnt(kWaitAll);
      asm volatile("" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (kt + 2 < nk) stage(buf == 0 ? 2 : buf - 1, (kt + 2) * BK);
      compute(buf);
      buf = buf == 2 ? 0 : buf + 1;
    }
    __syncthreads();
  }
  if (kids != nullptr) {
    // the per-wave key counts live in the idle tail of the staging LDS (past the
    // attention operands): a separate __shared__ array would push the 2-stage
    // block to 81,952 B, just over the 80 KiB that lets two blocks share a CU
    int* s_cnt = reinterpret_cast<int*>(smem + STAGES * kStage - 64);
    static_assert(V_OFF + D * VT_LD * 2 <= STAGES * kStage - 64 && NW * 4 <= 64, "key-count slot");
    const unsigned long long bal = __ballot(kid != pad);
    if (lane == 0) s_cnt[wid] = __popcll(bal);
    __syncthreads();
    kv_len = 0;
    if constexpr (SEQ == 1) {
#pragma unroll
      for (int w = 0; w < NW; ++w) kv_len += s_cnt[w];
    } else {                  // ids of sequence sq were read by waves 2*sq, 2*sq + 1 (S == 128)
      kv_len = s_cnt[2 * my_seq] + s_cnt[2 * my_seq + 1];
    }
  }
  kv_len = kv_len < S ? (kv_len < 1 ? 1 : kv_len) : S;
  // LNA: per-row (mean, rstd) of this lane's rows; head 0 publishes the sums
  float mu[LNA ? TM : 1], rs[LNA ? TM : 1];
  if constexpr (LNA) {
#pragma unroll
    for (int j = 0; j < TM; ++j) {
      float a = st1[j], q = st2[j];
      if constexpr (LNA == 1) {   // the 4 lanes of a row each saw a quarter of its k
        a += __shfl_xor(a, 16, 64);
        q += __shfl_xor(q, 16, 64);
        a += __shfl_xor(a, 32, 64);
        q += __shfl_xor(q, 32, 64);
      }
      ln_row_stats(float2{a, q}, ln.inv_d, ln.eps, mu[j], rs[j]);
      const int tok = wm * WM + j * 16 + fr;
      if (LNA == 1 && ln.stats_out != nullptr && h == 0 && wn == 0 && fg == 0 && tok % 128 < S && m0 + tok < ap.M)
        *reinterpret_cast<float2*>(ln.stats_out + (size_t)(m0 + tok) * 2) = float2{a, q};
    }
  }

  // ---- 2. + bias, round to T, park Q / K / V^T in LDS ----
  // lane holds P[token = wm*WM + j*16 + fr][col = wn*WN + i*16 + fg*4 .. +3];
  // a 16-column fragment never straddles the q / k / v boundaries (64, 128)
  char* Qs = smem + Q_OFF;
  char* Ks = smem + K_OFF;
  T* Vt = reinterpret_cast<T*>(smem + V_OFF);
#pragma unroll
  for (int i = 0; i < TN; ++i) {
    const int c0 = wn * WN + i * 16;                  // wave-uniform
    const int c = c0 + fg * 4;
    f32x4 bv, cs;
    if constexpr (LNA) {
      bv = *reinterpret_cast<const f32x4*>(ln.bias_f + n0 + c);
      cs = *reinterpret_cast<const f32x4*>(ln.colsum + n0 + c);
    } else {
      const u32x2 braw = *reinterpret_cast<const u32x2*>(bias + n0 + c);
      const T* be = reinterpret_cast<const T*>(&braw);
      bv = f32x4{(float)be[0], (float)be[1], (float)be[2], (float)be[3]};
    }
#pragma unroll
    for (int j = 0; j < TM; ++j) {
      const int tok = wm * WM + j * 16 + fr;
      f32x4 v = acc[i][j];
      if constexpr (LNA) v = (v - mu[j] * cs) * rs[j];
      v += bv;
      const frag4 y = {(T)v[0], (T)v[1], (T)v[2], (T)v[3]};
      if (c0 < 128) {        // Q or K: row-major [tok][d], 16-B chunks XOR-swizzled
        const int d = c0 < 64 ? c : c - 64;
        *reinterpret_cast<frag4*>((c0 < 64 ? Qs : Ks) + swz_off(tok, d >> 3) + (d & 7) * 2) = y;
      } else {               // V^T [d][tok]
        const int d = c - 128;
#pragma unroll
        for (int e = 0; e < 4; ++e) Vt[(d + e) * VT_LD + tok] = y[e];
      }
    }
  }
  __syncthreads();

  // ---- 3. attention: wave w owns queries [w*16*QT, (w+1)*16*QT) ----
  const int q0 = wid * 16 * QT;                      // token index in the tile
  const int kbase = my_seq * 128;                    // this wave's sequence's keys in the tile
  frag qf[QT][2];
#pragma unroll
  for (int qt = 0; qt < QT; ++qt)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
      qf[qt][ks] = *reinterpret_cast<const frag*>(Qs + swz_off(q0 + qt * 16 + fr, ks * 4 + fg));
  // S^T = K . Q^T: lane holds scores of keys kt*16 + fg*4 + e for query q0 + qt*16 + fr
  f32x4 s[8][QT];
#pragma unroll
  for (int kt = 0; kt < 8; ++kt) {
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) s[kt][qt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const frag kf = *reinterpret_cast<const frag*>(Ks + swz_off(kbase + kt * 16 + fr, ks * 4 + fg));
#pragma unroll
      for (int qt = 0; qt < QT; ++qt) s[kt][qt] = MfmaOp<T>::mma(kf, qf[qt][ks], s[kt][qt]);
    }
  }
  float l_run[QT];
  const bool need_mask = kv_len < 128;
#pragma unroll
  for (int qt = 0; qt < QT; ++qt) {
    float mx = -INFINITY;
#pragma unroll
    for (int kt = 0; kt < 8; ++kt)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if (need_mask && kt * 16 + fg * 4 + e >= kv_len) s[kt][qt][e] = -INFINITY;
        mx = fmaxf(mx, s[kt][qt][e]);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float m_use = mx * scale_log2e;            // kv_len >= 1: finite
    float ls = 0.f;
#pragma unroll
    for (int kt = 0; kt < 8; ++kt)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float p = exp2f(fmaf(s[kt][qt][e], scale_log2e, -m_use));
        s[kt][qt][e] = p;
        ls += p;
      }
    l_run[qt] = ls;
  }
  // O^T += V^T . P^T over 4 chunks of 32 keys (P from the S^T registers, permuted k order)
  f32x4 o[4][QT];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) o[dt][qt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    frag pf[QT];
#pragma unroll
    for (int qt = 0; qt < QT; ++qt)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        pf[qt][e] = (T)s[2 * c][qt][e];
        pf[qt][4 + e] = (T)s[2 * c + 1][qt][e];
      }
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const T* vr = Vt + (dt * 16 + fr) * VT_LD + kbase + c * 32 + fg * 4;
      const frag4 lo = *reinterpret_cast<const frag4*>(vr);
      const frag4 hi = *reinterpret_cast<const frag4*>(vr + 16);
      const frag vf = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
      for (int qt = 0; qt < QT; ++qt) o[dt][qt] = MfmaOp<T>::mma(vf, pf[qt], o[dt][qt]);
    }
  }
  // normalise and store: lane holds ctx[q][dt*16 + 4*fg + e]
#pragma unroll
  for (int qt = 0; qt < QT; ++qt) {
    float l = l_run[qt];
    l += __shfl_xor(l, 16, 64);
    l += __shfl_xor(l, 32, 64);
    const float inv = 1.f / l;
    const int q = q0 + qt * 16 + fr;
    if (q - kbase >= S || m0 + q >= ap.M) continue;
    T* op = out + (size_t)(m0 + q) * ld_out + h * D;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const frag4 v = {(T)(o[dt][qt][0] * inv), (T)(o[dt][qt][1] * inv), (T)(o[dt][qt][2] * inv),
                       (T)(o[dt][qt][3] * inv)};
      *reinterpret_cast<frag4*>(op + dt * 16 + fg * 4) = v;
    }
  }
}

// cfg: 0 = 8 waves (4x2) / 3 stages (1 block per CU), 1 = 8 waves (4x2) / 2 stages, 2 = 4 waves / 2 stages,
//      3 = 8 waves (2x4: 64x48 wave tiles, fewer LDS fragment reads per MFMA) / 2 stages,
//      4 = two sequences per block (256 x 192 tile, 8 waves 4x2, 2 stages; S == 128 only, else cfg 3)
// The 2-stage configs (1, 3) take exactly 80 KiB of LDS and <= 128 VGPRs: two
// blocks share a CU, one block's softmax beside the other's projection MFMAs.
constexpr int kNumQkvAttnCfgs = 5;

template <typename T, int LNA>
static void launch_qkv_attn(int cfg, const DenseParams& p, const T* W, const T* bias, int B, int S, int H,
                            const int* lens, T* out, int ld_out, float sl2e, const QkvLn& ln, hipStream_t s,
                            const int* kids, int pad) {
  const dim3 grid(B * H);
  switch (cfg) {
    case 0:
      hipLaunchKernelGGL((qkv_attn_kernel<T, 8, 3, LNA>), grid, dim3(512), 0, s, p, W, bias, S, H, lens, out, ld_out,
                         sl2e, ln, kids, pad);
      break;
    case 1:
      hipLaunchKernelGGL((qkv_attn_kernel<T, 8, 2, LNA>), grid, dim3(512), 0, s, p, W, bias, S, H, lens, out, ld_out,
                         sl2e, ln, kids, pad);
      break;
    case 3:
      hipLaunchKernelGGL((qkv_attn_kernel<T, 8, 2, LNA, 2>), grid, dim3(512), 0, s, p, W, bias, S, H, lens, out,
                         ld_out, sl2e, ln, kids, pad);
      break;
    case 4:   // two sequences per block (S == 128, host-checked)
      hipLaunchKernelGGL((qkv_attn_kernel<T, 8, 2, LNA, 4, 2>), dim3((B + 1) / 2 * H), dim3(512), 0, s, p, W, bias, S,
                         H, lens, out, ld_out, sl2e, ln, kids, pad);
      break;
    default:
      hipLaunchKernelGGL((qkv_attn_kernel<T, 4, 2, LNA>), grid, dim3(256), 0, s, p, W, bias, S, H, lens, out, ld_out,
                         sl2e, ln, kids, pad);
      break;
  }
}

// X [B*S, hidden] (row stride ldx), Wp [H*192, hidden] head-major packed, bp [H*192],
// out [B*S, H*64] (row stride ld_out).  dtype 0 = bf16, 1 = f16.
// colsum != 0 selects the LayerNorm-folded form: bp is unused, colsum / bias_f
// are f32 [H*192] (packed order), stats_out (optional) f32 [B*S, 2].
void qkv_attn_fwd(int dtype, uintptr_t X, int ldx, uintptr_t Wp, uintptr_t bp, int B, int S, int H, int hidden,
                  uintptr_t lens, uintptr_t out, int ld_out, float scale, int cfg, uintptr_t stream,
                  uintptr_t colsum, uintptr_t bias_f, uintptr_t stats_out, float eps, uintptr_t key_ids, int pad,
                  uintptr_t a_stats, int a_ld, int a_parts) {
  if (S < 1 || S > 128) throw std::invalid_argument("qkv_attn: 1 <= S <= 128");
  if (hidden % 8 || ldx % 8 || ld_out % 4) throw std::invalid_argument("qkv_attn: hidden / ldx % 8, ld_out % 4");
  const bool lna = colsum != 0;
  if ((X | Wp | out) & 15 || (!lna && (bp & 7)) || (lna && ((colsum | bias_f) & 15 || !bias_f)) || stats_out & 7)
    throw std::invalid_argument("qkv_attn: alignment / folded-LayerNorm operands");
  if (cfg < 0 || cfg >= kNumQkvAttnCfgs) cfg = 1;
  if (cfg == 4 && S != 128) cfg = 3;
  if (key_ids && lens) throw std::invalid_argument("qkv_attn: pass lens or key_ids, not both");
  if (key_ids & 3) throw std::invalid_argument("qkv_attn: key_ids must be int32-aligned");
  if (a_stats && (!lna || stats_out || (a_stats & 7) || a_parts < 1 || a_parts > 8 || a_ld < 2 * a_parts))
    throw std::invalid_argument("qkv_attn: partial statistics need the folded form, 1..8 parts, no stats_out");
  if (B <= 0 || H <= 0) return;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const DenseParams p{reinterpret_cast<const void*>(X), ldx, B * S, hidden};
  const float sl2e = scale * 1.4426950408889634f;
  const QkvLn ln{reinterpret_cast<const float*>(colsum), reinterpret_cast<const float*>(bias_f),
                 reinterpret_cast<float*>(stats_out), 1.0f / hidden, eps, reinterpret_cast<const float*>(a_stats),
                 a_ld, a_parts};
#define RDB_QA(T, L)                                                                                            \
  launch_qkv_attn<T, L>(cfg, p, reinterpret_cast<const T*>(Wp), reinterpret_cast<const T*>(bp), B, S, H,        \
                        reinterpret_cast<const int*>(lens), reinterpret_cast<T*>(out), ld_out, sl2e, ln, s,   \
                        reinterpret_cast<const int*>(key_ids), pad)
  if (dtype == 0) {
    if (lna && a_stats) RDB_QA(bf16, 2); else if (lna) RDB_QA(bf16, 1); else RDB_QA(bf16, 0);
  } else if (dtype == 1) {
    if (lna) RDB_QA(f16, 1); else RDB_QA(f16, 0);
  } else {
    throw std::invalid_argument("qkv_attn: dtype must be bf16 or f16");
  }
#undef RDB_QA
  RDB_HIP_CHECK(hipGetLastError());
}

}  // namespace rdb
