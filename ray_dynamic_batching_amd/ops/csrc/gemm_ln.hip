// Dense bf16 MFMA GEMM with the deferred-LayerNorm epilogues (gemm_core.h
// LnEpi): the GEMMs of a post-LN transformer layer run with no LayerNorm
// kernel between them.
//
//   mode LNA          y = act(rstd_A[m] (A W'^T - mean_A[m] colsum[n]) + bias'[n])   (W' = W * gamma)
//   mode STATS        y = A W^T + bias + R,                 stats[m] += (sum y, sum y^2)
//   mode LNR | STATS  y = A W^T + bias + LN(R) (normalised on load), stats[m] += ...
//   mode LNR          y = A W^T + bias + LN(R)
//   mode LNOUT        y = LN(A W^T + bias + R) (gamma r_g, beta r_b): the row
//                     panel reduces statistics through o_stats (zeroed [M, 2])
//                     and the panel counters (zeroed int [tiles_m])
//   mode LNA | SELF   as LNA, but A's row statistics are computed by this GEMM
//                     from the A tiles of its own main loop; the first N-tile's
//                     blocks store them to o_stats (for a later LNR of A)
//
// Used by models/bert.py (fold_ln): QKV and FFN-up take LNA, o-proj and
// FFN-down take (LNR |) STATS.  Reference behaviour being preserved: the
// BertLayer LayerNorms of the served models.
#include "gemm_core.h"
#include <stdexcept>
#include <string>

namespace rdb {

void gemm_tn_ln(uintptr_t A, int lda, uintptr_t W, int ldw, uintptr_t C, int ldc, uintptr_t bias, uintptr_t R,
                int ldr, int M, int N, int K, float alpha, int act, int mode, uintptr_t a_stats, int a_ld,
                uintptr_t a_colsum, uintptr_t a_bias, uintptr_t r_stats, int r_ld, uintptr_t r_g, uintptr_t r_b,
                uintptr_t o_stats, int o_ld, float a_inv_d, float r_inv_d, float eps, uintptr_t stream, int cfg,
                uintptr_t panel, uintptr_t err, int a_parts, int r_parts) {
  if (K % 8 != 0 || lda % 8 != 0 || ldw % 8 != 0) throw std::invalid_argument("gemm_tn_ln: K/lda/ldw % 8");
  if ((A | W) & 15) throw std::invalid_argument("gemm_tn_ln: A/W must be 16-byte aligned");
  if (N % 4 != 0 || ldc % 4 != 0) throw std::invalid_argument("gemm_tn_ln: N and ldc must be multiples of 4");
  if (act == ACT_SWIGLU) throw std::invalid_argument("gemm_tn_ln: no SWIGLU");
  if (M <= 0 || N <= 0 || K <= 0) return;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  LnEpi ln{};
  ln.a_stats = reinterpret_cast<const float*>(a_stats);
  ln.a_colsum = reinterpret_cast<const float*>(a_colsum);
  ln.a_bias = reinterpret_cast<const float*>(a_bias);
  ln.r_stats = reinterpret_cast<const float*>(r_stats);
  ln.r_g = reinterpret_cast<const void*>(r_g);
  ln.r_b = reinterpret_cast<const void*>(r_b);
  ln.o_stats = reinterpret_cast<float*>(o_stats);
  ln.a_ld = a_ld; ln.r_ld = r_ld; ln.o_ld = o_ld;
  ln.a_inv_d = a_inv_d; ln.r_inv_d = r_inv_d; ln.eps = eps;
  ln.panel = reinterpret_cast<int*>(panel);
  ln.err = reinterpret_cast<int*>(err);
  ln.a_parts = a_parts;
  ln.r_parts = r_parts;
  DenseParams p{reinterpret_cast<const void*>(A), lda, M, K};
  auto w = reinterpret_cast<const bf16*>(W);
  auto b = reinterpret_cast<const bf16*>(bias);
  auto r = reinterpret_cast<const bf16*>(R);
  auto c = reinterpret_cast<bf16*>(C);
  if (cfg < 0 || cfg >= kNumTiles) cfg = pick_tile_cfg(M, N, true);
  auto need = [](bool ok, const char* what) {
    if (!ok) throw std::invalid_argument(what);
  };
  if (mode & EPI_STG) {
    // the staged epilogue's requirements (16-B rows, no SwiGLU) and the partial layouts
    cfg = stg_tile_cfg(cfg);
    need(N % 8 == 0 && ldc % 8 == 0 && (C & 15) == 0 && (!R || (ldr % 8 == 0 && (R & 15) == 0)),
         "gemm_tn_ln: staged LN modes need N, ldc, ldr % 8 and 16-byte aligned C / residual");
    need((a_stats & 7) == 0 && (r_stats & 7) == 0 && (o_stats & 7) == 0 && a_parts >= 1 && r_parts >= 1,
         "gemm_tn_ln: staged LN statistics: 8-byte aligned, parts >= 1");
    if (mode & EPI_STATS) {
      const int parts = (N + kTileBN[cfg] - 1) / kTileBN[cfg];
      need(o_ld >= 2 * parts, "gemm_tn_ln: out statistics row stride < 2 x N-tiles of the tile");
    }
  }
  switch (mode) {
    case EPI_LNA:
      need(a_stats && a_colsum && a_bias && !bias && !R, "gemm_tn_ln: LNA needs a_stats/a_colsum/a_bias, no bias/R");
      launch_mfma_gemm_t<bf16, bf16, DenseLoader, false, false, EPI_LNA>(p, w, ldw, c, ldc, b, r, ldr, M, N, K,
                                                                         alpha, act, s, cfg, ln);
      break;
    case EPI_STATS:
      need(o_stats && bias && R, "gemm_tn_ln: STATS needs o_stats, bias and R");
      launch_mfma_gemm_t<bf16, bf16, DenseLoader, true, true, EPI_STATS>(p, w, ldw, c, ldc, b, r, ldr, M, N, K,
                                                                         alpha, act, s, cfg, ln);
      break;
    case EPI_LNR | EPI_STATS:
      need(o_stats && bias && R && r_stats && r_g && r_b, "gemm_tn_ln: LNR|STATS needs o_stats, bias, R, r_*");
      launch_mfma_gemm_t<bf16, bf16, DenseLoader, true, true, EPI_LNR | EPI_STATS>(p, w, ldw, c, ldc, b, r, ldr, M,
                                                                                   N, K, alpha, act, s, cfg, ln);
      break;
    case EPI_LNR:
      need(bias && R && r_stats && r_g && r_b, "gemm_tn_ln: LNR needs bias, R, r_*");
      launch_mfma_gemm_t<bf16, bf16, DenseLoader, true, true, EPI_LNR>(p, w, ldw, c, ldc, b, r, ldr, M, N, K, alpha,
                                                                       act, s, cfg, ln);
      break;
#if RDB_EXPERIMENTAL
    case EPI_LNOUT: {
      need(bias && R && r_g && r_b && o_stats && panel && act == ACT_NONE,
           "gemm_tn_ln: LNOUT needs bias, R, r_g/r_b, o_stats, panel workspaces and no activation");
      need(N % 8 == 0 && ldc % 8 == 0 && ldr % 8 == 0 && ((C | R | r_g | r_b) & 15) == 0,
           "gemm_tn_ln: LNOUT needs N, ldc, ldr % 8 and 16-byte aligned C, R, gamma, beta");
      if (!ln_out_tile_ok(cfg)) cfg = -1;
      if (cfg >= 0) {   // every block of a row panel must be able to be resident at once
        const long tiles = (long)((M + kTileBM[cfg] - 1) / kTileBM[cfg]) * ((N + kTileBN[cfg] - 1) / kTileBN[cfg]);
        if (tiles > 256L * tile_blocks_per_cu(cfg)) cfg = -1;
      }
      if (cfg < 0) {
        for (int t = 0; t < 19 && cfg < 0; ++t) {
          const long tiles = (long)((M + kTileBM[t] - 1) / kTileBM[t]) * ((N + kTileBN[t] - 1) / kTileBN[t]);
          if (ln_out_tile_ok(t) && tiles <= 256L * tile_blocks_per_cu(t)) cfg = t;
        }
        need(cfg >= 0, "gemm_tn_ln: LNOUT: no tile keeps every row panel resident at this M, N");
      }
      launch_mfma_gemm_t<bf16, bf16, DenseLoader, true, true, EPI_LNOUT>(p, w, ldw, c, ldc, b, r, ldr, M, N, K, alpha,
                                                                         act, s, cfg, ln);
      break;
    }
#endif
    case EPI_LNA | EPI_SELF:
      need(a_colsum && a_bias && !bias && !R, "gemm_tn_ln: LNA|SELF needs a_colsum/a_bias, no bias/R");
      launch_mfma_gemm_t<bf16, bf16, DenseLoader, false, false, EPI_LNA | EPI_SELF>(p, w, ldw, c, ldc, b, r, ldr, M, N,
                                                                                    K, alpha, act, s, cfg, ln);
      break;
#if RDB_EXPERIMENTAL
    case EPI_STG | EPI_LNA:
      need(a_stats && a_colsum && a_bias && !bias && !R, "gemm_tn_ln: STG|LNA needs a_stats/a_colsum/a_bias, no bias/R");
      launch_mfma_gemm_t<bf16, bf16, DenseLoader, false, false, EPI_STG | EPI_LNA>(p, w, ldw, c, ldc, b, r, ldr, M, N,
                                                                                   K, alpha, act, s, cfg, ln);
      break;
    case EPI_STG | EPI_STATS:
      need(o_stats && bias && R, "gemm_tn_ln: STG|STATS needs o_stats, bias and R");
      launch_mfma_gemm_t<bf16, bf16, DenseLoader, true, true, EPI_STG | EPI_STATS>(p, w, ldw, c, ldc, b, r, ldr, M, N,
                                                                                   K, alpha, act, s, cfg, ln);
      break;
    case EPI_STG | EPI_LNR | EPI_STATS:
      need(o_stats && bias && R && r_stats && r_g && r_b, "gemm_tn_ln: STG|LNR|STATS needs o_stats, bias, R, r_*");
      launch_mfma_gemm_t<bf16, bf16, DenseLoader, true, true, EPI_STG | EPI_LNR | EPI_STATS>(
          p, w, ldw, c, ldc, b, r, ldr, M, N, K, alpha, act, s, cfg, ln);
      break;
    case EPI_STG | EPI_LNR:
      need(bias && R && r_stats && r_g && r_b, "gemm_tn_ln: STG|LNR needs bias, R, r_*");
      launch_mfma_gemm_t<bf16, bf16, DenseLoader, true, true, EPI_STG | EPI_LNR>(p, w, ldw, c, ldc, b, r, ldr, M, N,
                                                                                 K, alpha, act, s, cfg, ln);
      break;
#else
    case EPI_LNOUT:
    case EPI_STG | EPI_LNA:
    case EPI_STG | EPI_STATS:
    case EPI_STG | EPI_LNR | EPI_STATS:
    case EPI_STG | EPI_LNR:
      RDB_EXPERIMENTAL_MISSING("gemm_tn_ln (LNOUT / staged modes)");
#endif
    default:
      throw std::invalid_argument(
          "gemm_tn_ln: mode must be LNA (1), STATS (4), LNR|STATS (6), LNR (2), LNA|SELF (9), LNOUT (16) or a "
          "staged mode STG (32) | LNA, STATS, LNR|STATS, LNR");
  }
  RDB_HIP_CHECK(hipGetLastError());
}

int gemm_stg_cfg(int cfg) { return stg_tile_cfg(cfg); }
int gemm_tile_bn(int cfg) { return cfg >= 0 && cfg < kNumTiles ? kTileBN[cfg] : -1; }

}  // namespace rdb
