// Full-row GEMM + bias + residual + LayerNorm for gfx950: the post-LN
// transformer's o-proj -> LN1 and FFN-down -> LN2 (BERT / ViT hidden 768) in
// ONE kernel, with the row statistics block-local -- no LayerNorm launch, no
// pre-LN activation round trip, no cross-block wait.
//
//   C[m, :] = LayerNorm(A[m, :] W^T + bias + R[m, :]) * gamma + beta,  N = NFULL
//
// Geometry: a 512-thread block owns BM = 64 WHOLE rows (all NFULL columns), so
// M = 4096 (BERT-base batch 32) is 64 blocks -- a quarter of the chip, which the
// replica's second compute stream fills.  Wave w owns columns [w*WN, w*WN+WN)
// (WN = NFULL / 8 = 96 -> 4 x 6 fragments of v_mfma_f32_16x16x32_bf16, 96 f32
// accumulator VGPRs).  Why this is cheaper in CU-time than a tiled GEMM plus a
// LayerNorm kernel: the tiles that fill 256 CUs with N = 768 are small (128 x
// 96: ~0.5 KiB of LDS traffic per MFMA, 27 % of the MFMA peak in two-stream
// serving), while a 64 x 768 panel re-uses every A element 768 times and every
// W element 64 times.
//
// Operand paths (per BK = 32 step):
//   * W (the weight, L2-resident and read by every block): each wave loads ITS
//     96 rows x 32 k straight into fragment registers (16 B per lane, no LDS:
//     no other wave needs them), three register buffers = two steps of prefetch.
//     W is PACKED k-tile-major, Wp[K/32][NFULL][32] (ops.pack_rowln_weight, once
//     at load): a step's slice is one contiguous 48 KiB run and every wave
//     instruction reads 1 KiB contiguously.  Row-major [N, K] made each step
//     touch all 768 rows -- the whole matrix's pages, every step -- and ran 4-5x
//     slower (measured: o-proj 49 us, FFN-down 148 us on MI355X).
//   * A (64 rows x 32 k, shared by all 8 waves): one 8-B buffer load per thread,
//     two steps ahead in registers, ds_write into one of three LDS buffers
//     (XOR-swizzled 16-B chunks), 4 ds_read_b128 per wave per step.
//   The step ends with lgkmcnt(0) + a raw s_barrier (no __syncthreads: its
//   fence would drain the in-flight W / A prefetch every step).
//
// Epilogue (all in registers + 4 KiB of LDS): v = acc + bias + R (f32), row
// partial sums over a lane's 24 values, a 4-lane shuffle reduction, the 8
// waves' partials through LDS, then the same for sum((v - mean)^2) (two-pass,
// the statistics of the f32 values), y = (v - mean) * rstd * gamma + beta,
// 8-B bf16x4 stores.
//
// The fp32 reference is ops.linear_residual_ln_ref (tests/test_ops_gpu.py).
#include <hip/hip_runtime.h>

#include <stdexcept>
#include <string>

#include "gemm_core.h"

namespace rdb {

#if RDB_EXPERIMENTAL
template <int NFULL>
__global__ void __launch_bounds__(512, 2)
gemm_rowln_kernel(const bf16* __restrict__ A, int lda, const bf16* __restrict__ W,
                  const bf16* __restrict__ bias, const bf16* __restrict__ R, int ldr, const bf16* __restrict__ gamma,
                  const bf16* __restrict__ beta, bf16* __restrict__ C, int ldc, int M, int K, float eps) {
  constexpr int BM = 64, BK = 32, NW = 8, WN = NFULL / NW, TN = WN / 16, TM = BM / 16;
  constexpr int ABUF = BM * BK * 2;  // 4 KiB per A stage
  static_assert(WN % 16 == 0, "NFULL must split into 16-column fragments per wave");
  typedef bf16x8 frag;
  __shared__ __attribute__((aligned(16))) char sa[3 * ABUF];
  __shared__ __attribute__((aligned(16))) float red[2][BM][NW];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int m0 = blockIdx.x * BM;
  const int nk = K / BK;

  // ---- A staging: thread t -> row t/8, 4 k-elements (t%8)*4 ----
  const __amdgpu_buffer_rsrc_t asrc = make_rsrc(A, (uint32_t)((size_t)(M - 1) * lda * 2 + (size_t)K * 2));
  const int arow = tid >> 3, akq = tid & 7;
  const uint32_t aoff = (m0 + arow < M) ? (uint32_t)((size_t)(m0 + arow) * lda * 2 + akq * 8) : kOOB;
  const int awr = arow * 64 + (((akq >> 1) ^ ((arow >> 2) & 3)) << 4) + (akq & 1) * 8;
  // a step past the end issues its loads anyway, as out-of-range buffer loads
  // (zero, no memory traffic): every step then has the same loads in flight and
  // hipcc's waitcnt pass keeps a counted vmcnt instead of draining to 0
  auto gA = [&](int kt) -> u32x2 {
    return bload8(asrc, (aoff == kOOB || kt >= nk) ? kOOB : aoff + (uint32_t)(kt * BK * 2));
  };

  // ---- W fragments (packed Wp[kt][n][32]): lane -> row wid*WN + nf*16 + lane%16, k-chunk lane/16 ----
  const __amdgpu_buffer_rsrc_t wsrc = make_rsrc(W, (uint32_t)((size_t)K * NFULL * 2));
  const uint32_t woff0 = (uint32_t)((wid * WN + (lane & 15)) * BK * 2 + (lane >> 4) * 16);
  constexpr uint32_t wstep = 16 * BK * 2, wkt = NFULL * BK * 2;
  auto gW = [&](frag (&wf)[TN], int kt) {
#pragma unroll
    for (int nf = 0; nf < TN; ++nf) {
      const u32x4 raw = bload16(wsrc, kt >= nk ? kOOB : woff0 + nf * wstep + (uint32_t)kt * wkt);
      wf[nf] = __builtin_bit_cast(frag, raw);
    }
  };
  auto rA = [&](frag (&af)[TM], int buf) {
#pragma unroll
    for (int mf = 0; mf < TM; ++mf) {
      const int row = mf * 16 + (lane & 15), ch = lane >> 4;
      af[mf] = *reinterpret_cast<const frag*>(sa + buf * ABUF + row * 64 + ((ch ^ ((row >> 2) & 3)) << 4));
    }
  };
  auto barrier = [] {
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's LDS writes / reads are done
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  frag w[3][TN];
  u32x2 areg[3];
  // prologue: A(0) in LDS buffer 0, A(1) / W(0) / W(1) in flight
  areg[0] = gA(0);
  areg[1] = gA(1);
  gW(w[0], 0);
  gW(w[1], 1);
  *reinterpret_cast<u32x2*>(sa + awr) = areg[0];
  barrier();

  // step kt (p = kt % 3): issue A(kt+2) then W(kt+2) (A first, so the ds_write
  // that needs A(kt+2) one step later leaves W(kt+2) in flight), MFMAs on
  // W(kt) x A(kt), stage A(kt+1) into the next LDS buffer, barrier.
  auto step = [&](auto P, int kt) {
    constexpr int p = decltype(P)::value;
    constexpr int p1 = (p + 1) % 3, p2 = (p + 2) % 3;
    areg[p2] = gA(kt + 2);
    gW(w[p2], kt + 2);
    frag af[TM];
    rA(af, p);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int nf = 0; nf < TN; ++nf)
#pragma unroll
      for (int mf = 0; mf < TM; ++mf) acc[mf][nf] = MfmaOp<bf16>::mma(w[p][nf], af[mf], acc[mf][nf]);
    __builtin_amdgcn_s_setprio(0);
    // unconditional: past the end it stages the zeros of an out-of-range load
    // into a buffer no later step reads (a conditional store lets hipcc sink
    // the A load into the branch and drain vmcnt to 0 there)
    *reinterpret_cast<u32x2*>(sa + p1 * ABUF + awr) = areg[p1];
    barrier();
  };
  int kt = 0;
  for (; kt + 3 <= nk; kt += 3) {
    step(std::integral_constant<int, 0>{}, kt);
    step(std::integral_constant<int, 1>{}, kt + 1);
    step(std::integral_constant<int, 2>{}, kt + 2);
  }
  if (kt < nk) step(std::integral_constant<int, 0>{}, kt);
  if (kt + 1 < nk) step(std::integral_constant<int, 1>{}, kt + 1);

  // ---- epilogue: lane holds rows mf*16 + lane%16, columns wid*WN + nf*16 + 4*(lane/16) + r ----
  const int cq = wid * WN + 4 * (lane >> 4);
  const __amdgpu_buffer_rsrc_t vsrc_b = make_rsrc(bias, NFULL * 2);
  const __amdgpu_buffer_rsrc_t vsrc_g = make_rsrc(gamma, NFULL * 2);
  const __amdgpu_buffer_rsrc_t vsrc_e = make_rsrc(beta, NFULL * 2);
  const __amdgpu_buffer_rsrc_t rsrc = make_rsrc(R, (uint32_t)((size_t)(M - 1) * ldr * 2 + NFULL * 2));
  auto unpack = [](u32x2 raw, float (&o)[4]) {
    o[0] = __uint_as_float(raw.x << 16);
    o[1] = __uint_as_float(raw.x & 0xFFFF0000u);
    o[2] = __uint_as_float(raw.y << 16);
    o[3] = __uint_as_float(raw.y & 0xFFFF0000u);
  };
  // residual loads first (the long-latency ones), then the per-column vectors
  u32x2 rraw[TM][TN];
#pragma unroll
  for (int mf = 0; mf < TM; ++mf) {
    const int gm = m0 + mf * 16 + (lane & 15);
    const uint32_t ro = gm < M ? (uint32_t)((size_t)gm * ldr * 2) : kOOB;
#pragma unroll
    for (int nf = 0; nf < TN; ++nf)
      rraw[mf][nf] = bload8(rsrc, ro == kOOB ? kOOB : ro + (uint32_t)((cq + nf * 16) * 2));
  }
  float bv[TN][4];
#pragma unroll
  for (int nf = 0; nf < TN; ++nf) unpack(bload8(vsrc_b, (uint32_t)((cq + nf * 16) * 2)), bv[nf]);

  float mean[TM], rstd[TM];
#pragma unroll
  for (int mf = 0; mf < TM; ++mf) {
    float s = 0.f;
#pragma unroll
    for (int nf = 0; nf < TN; ++nf) {
      float rv[4];
      unpack(rraw[mf][nf], rv);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        acc[mf][nf][r] += bv[nf][r] + rv[r];
        s += acc[mf][nf][r];
      }
    }
    s += __shfl_xor(s, 16, 64);
    s += __shfl_xor(s, 32, 64);
    if (lane < 16) red[0][mf * 16 + lane][wid] = s;
  }
  __syncthreads();
  constexpr float inv_n = 1.0f / NFULL;
#pragma unroll
  for (int mf = 0; mf < TM; ++mf) {
    const f32x4* pr = reinterpret_cast<const f32x4*>(&red[0][mf * 16 + (lane & 15)][0]);
    const f32x4 a = pr[0], b = pr[1];
    mean[mf] = (a.x + a.y + a.z + a.w + b.x + b.y + b.z + b.w) * inv_n;
    float q = 0.f;
#pragma unroll
    for (int nf = 0; nf < TN; ++nf)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float d = acc[mf][nf][r] - mean[mf];
        q += d * d;
      }
    q += __shfl_xor(q, 16, 64);
    q += __shfl_xor(q, 32, 64);
    if (lane < 16) red[1][mf * 16 + lane][wid] = q;
  }
  float gv[TN][4], ev[TN][4];
#pragma unroll
  for (int nf = 0; nf < TN; ++nf) {
    unpack(bload8(vsrc_g, (uint32_t)((cq + nf * 16) * 2)), gv[nf]);
    unpack(bload8(vsrc_e, (uint32_t)((cq + nf * 16) * 2)), ev[nf]);
  }
  __syncthreads();
#pragma unroll
  for (int mf = 0; mf < TM; ++mf) {
    const f32x4* pr = reinterpret_cast<const f32x4*>(&red[1][mf * 16 + (lane & 15)][0]);
    const f32x4 a = pr[0], b = pr[1];
    rstd[mf] = rsqrtf((a.x + a.y + a.z + a.w + b.x + b.y + b.z + b.w) * inv_n + eps);
  }
#pragma unroll
  for (int mf = 0; mf < TM; ++mf) {
    const int gm = m0 + mf * 16 + (lane & 15);
    if (gm >= M) continue;
    bf16* crow = C + (size_t)gm * ldc + cq;
#pragma unroll
    for (int nf = 0; nf < TN; ++nf) {
      float o[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) o[r] = (acc[mf][nf][r] - mean[mf]) * rstd[mf] * gv[nf][r] + ev[nf][r];
      store4<bf16>(crow + nf * 16, o[0], o[1], o[2], o[3]);
    }
  }
}

// Host launcher (bindings.cpp: ``gemm_rowln``).  Requirements (checked by
// ops.linear_rowln as well): N == 768, K % 32 == 0, lda % 4 == 0, W packed
// [K/32][N][32], 16-B aligned A / W, 8-B aligned bias / R / gamma / beta / C with
// ldr, ldc % 4 == 0.
void gemm_rowln(uintptr_t A, int lda, uintptr_t W, uintptr_t bias, uintptr_t R, int ldr, uintptr_t gamma,
                uintptr_t beta, uintptr_t C, int ldc, int M, int N, int K, float eps, uintptr_t stream) {
  if (N != 768) throw std::invalid_argument("gemm_rowln: N must be 768 (got " + std::to_string(N) + ")");
  if (K <= 0 || K % 32 != 0) throw std::invalid_argument("gemm_rowln: K must be a positive multiple of 32");
  if (lda % 4 != 0 || ldr % 4 != 0 || ldc % 4 != 0) throw std::invalid_argument("gemm_rowln: lda/ldr/ldc % 4");
  if (((A | W) & 15) || ((bias | R | gamma | beta | C) & 7)) throw std::invalid_argument("gemm_rowln: alignment");
  if ((size_t)M * lda * 2 >= 0x80000000ull || (size_t)M * ldr * 2 >= 0x80000000ull)
    throw std::invalid_argument("gemm_rowln: operand exceeds the 2 GiB buffer-offset range");
  if (M <= 0) return;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(gemm_rowln_kernel<768>, dim3((M + 63) / 64), dim3(512), 0, s, reinterpret_cast<const bf16*>(A),
                     lda, reinterpret_cast<const bf16*>(W), reinterpret_cast<const bf16*>(bias),
                     reinterpret_cast<const bf16*>(R), ldr, reinterpret_cast<const bf16*>(gamma),
                     reinterpret_cast<const bf16*>(beta), reinterpret_cast<bf16*>(C), ldc, M, K, eps);
  RDB_HIP_CHECK(hipGetLastError());
}
#else
void gemm_rowln(uintptr_t, int, uintptr_t, uintptr_t, uintptr_t, int, uintptr_t, uintptr_t, uintptr_t, int, int, int,
                int, float, uintptr_t) {
  RDB_EXPERIMENTAL_MISSING("gemm_rowln");
}
#endif

}  // namespace rdb
