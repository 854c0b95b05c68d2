// Fused multi-head attention forward for gfx950 (flash-style, online softmax).
//
// Reads Q/K/V straight out of the packed projection output [T, (H+2*Hkv)*D]
// (no transpose kernels), supports a per-sequence key length (padding mask),
// causal masking and GQA (Hkv divides H).  Used by BERT-base (S=128, D=64,
// bidirectional) and Llama-3 prefill (D=128, causal, GQA).
//
// One workgroup = 4 waves = 64 * QT query rows of one (batch, head); each wave
// owns 16 * QT query rows.  QT = 1 when the QT = 2 grid would not give every CU
// two blocks (BERT: B32 x H12 x S128 is 384 blocks at QT = 2, i.e. 1.5 per CU
// and no overlap of one block's K/V load latency with another's math; 768 at
// QT = 1, at the price of staging each K/V block twice).  K/V blocks of 128 keys are staged in LDS:
//   * K row-major [key][D] with the 16-B chunk XOR swizzle (ds_read_b128 frags);
//   * V transposed [D][128 + 8] (the +8 element pad makes the 8-byte fragment
//     reads of 16 d-rows x 2 key groups conflict-free).
// Swapped products keep softmax lane-local (cdna_hip_programming.md T12 idea):
//   S^T = K . Q^T   (A = K frag from LDS, B = Q frag in registers)
//        -> each lane holds 4 keys x (key tiles) for ONE query, so the row
//           max / sum need only 2 cross-lane steps (xor 16, xor 32);
//   O^T += V^T . P^T (A = V^T frag from LDS, B = P taken from the S^T
//        accumulator registers with a permuted-but-consistent k order, §3)
//        -> each lane holds 4 consecutive d of one query: 8-byte stores.
#include "common.h"
#include <cstdlib>
#include <stdexcept>

namespace rdb {

template <int D>
struct AttnCfg {
  // keys per LDS block: 64 at D = 128 keeps S^T (and the K/V staging) within
  // the register budget next to the 128-wide O accumulator (KB = 128 spilled)
  static constexpr int KB = D == 128 ? 64 : 128;
  static constexpr int ROWB = D * 2;             // bytes per K row
  static constexpr int CPR = ROWB / 16;          // 16-B chunks per K row (8 or 16)
  static constexpr int VT_LD = KB + 8;           // V^T row length (elements)
  static constexpr int K_BYTES = KB * ROWB;
  static constexpr int V_BYTES = D * VT_LD * 2;
};

template <typename T>
__device__ __forceinline__ f32x4 mma16(
    T __attribute__((ext_vector_type(8))) a, T __attribute__((ext_vector_type(8))) b, f32x4 c);
template <>
__device__ __forceinline__ f32x4 mma16<bf16>(bf16x8 a, bf16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
template <>
__device__ __forceinline__ f32x4 mma16<f16>(f16x8 a, f16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
}

template <int CPR>
__device__ __forceinline__ int kswz(int row, int chunk) {
  if constexpr (CPR == 8) return row * 128 + ((chunk ^ ((row >> 1) & 7)) << 4);
  else return row * (CPR * 16) + ((chunk ^ (row & 15)) << 4);
}

template <typename T, int D, int QT>
__global__ void __launch_bounds__(256, QT == 1 ? 3 : 2)
attn_fwd_kernel(const T* __restrict__ qkv, int ld_qkv, int q_off, int k_off, int v_off,
                int H, int Hkv, int S, const int* __restrict__ lens, int causal,
                T* __restrict__ out, int ld_out, float scale_log2e) {
  typedef AttnCfg<D> C;
  typedef T frag8 __attribute__((ext_vector_type(8)));
  typedef T frag4 __attribute__((ext_vector_type(4)));
  constexpr int KB = C::KB;
  constexpr int NKT = KB / 16;       // key tiles per block
  constexpr int NKS = D / 32;        // k-steps for S = K.Q^T
  constexpr int NDT = D / 16;        // d tiles of O^T
  __shared__ __attribute__((aligned(16))) char smem[C::K_BYTES + C::V_BYTES];
  char* Ks = smem;
  T* Vt = reinterpret_cast<T*>(smem + C::K_BYTES);

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const int b = blockIdx.z, h = blockIdx.y;
  const int hk = h / (H / Hkv);
  constexpr int QROWS = 64 * QT;                 // query rows per block
  const int q0 = blockIdx.x * QROWS + wid * 16 * QT;  // this wave's first query row
  const size_t tok0 = (size_t)b * S;

  // K/V staging: EVERY load of a block is issued before the first LDS write
  // (one memory round trip per block); rows past S clamp to a valid row, their
  // scores are masked below.  Block 0 is always needed, so its loads go out
  // before anything else -- in particular before the key length arrives.
  // D = 128 stages in two halves so the staging registers stay at 32 VGPRs
  // (holding all 16 K/V vectors spilled at D = 128).
  constexpr int NST = KB * C::CPR / 256;          // 16-B K (and V) vectors per thread per block
  constexpr int NCH = NST > 4 ? 4 : NST;          // ... held in registers at a time
  constexpr int NPART = NST / NCH;
  u32x4 kreg[NCH];
  frag8 vreg[NCH];
  auto load_kv = [&](int key0, int part) {
#pragma unroll
    for (int j = 0; j < NCH; ++j) {
      const int qd = tid + 256 * (part * NCH + j);
      const int krow = min(key0 + qd / C::CPR, S - 1), kc = qd % C::CPR;
      kreg[j] = *reinterpret_cast<const u32x4*>(qkv + (tok0 + krow) * ld_qkv + k_off + hk * D + kc * 8);
      const int vrow = min(key0 + (qd & (KB - 1)), S - 1), vc = qd / KB;
      vreg[j] = *reinterpret_cast<const frag8*>(qkv + (tok0 + vrow) * ld_qkv + v_off + hk * D + vc * 8);
    }
  };
  auto store_kv = [&](int part) {
#pragma unroll
    for (int j = 0; j < NCH; ++j) {   // K row-major, swizzled
      const int qd = tid + 256 * (part * NCH + j), row = qd / C::CPR, c = qd % C::CPR;
      *reinterpret_cast<u32x4*>(Ks + kswz<C::CPR>(row, c)) = kreg[j];
    }
#pragma unroll
    for (int j = 0; j < NCH; ++j) {
      // V transposed: lanes of a wave take consecutive keys, so lanes 2p / 2p+1
      // hold keys (k, k+1).  They swap half their 8 d-values, then each writes
      // 4 key PAIRS as dwords (the even lane d 0..3, the odd lane d 4..7): 4
      // ds_write_b32 instead of 8 ds_write_b16, and every 32-lane group hits
      // 32 distinct banks (VT_LD = KB + 8 puts d-row +4 at bank offset 16).
      const int qd = tid + 256 * (part * NCH + j), row = qd & (KB - 1), c = qd / KB;
      const u32x4 mine = __builtin_bit_cast(u32x4, vreg[j]);
      const bool odd = row & 1;
      const uint32_t s0 = odd ? mine[0] : mine[2], s1 = odd ? mine[1] : mine[3];
      const uint32_t r0 = __shfl_xor(s0, 1, 64), r1 = __shfl_xor(s1, 1, 64);
      const uint32_t m0 = odd ? mine[2] : mine[0], m1 = odd ? mine[3] : mine[1];  // my d-values to write
      const uint32_t mv[4] = {m0 & 0xffffu, m0 >> 16, m1 & 0xffffu, m1 >> 16};
      const uint32_t pv[4] = {r0 & 0xffffu, r0 >> 16, r1 & 0xffffu, r1 >> 16};
      const int d0 = c * 8 + (odd ? 4 : 0), k0 = row & ~1;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const uint32_t w = odd ? (pv[e] | (mv[e] << 16)) : (mv[e] | (pv[e] << 16));
        *reinterpret_cast<uint32_t*>(Vt + (d0 + e) * C::VT_LD + k0) = w;
      }
    }
  };
  load_kv(0, 0);

  // Q fragments (B operand): lane holds Q[q][ks*32 + 8*fg + j].
  frag8 qf[QT][NKS];
#pragma unroll
  for (int qt = 0; qt < QT; ++qt) {
    const int q = min(q0 + qt * 16 + fr, S - 1);  // rows past S are computed, never stored
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks)
      qf[qt][ks] = *reinterpret_cast<const frag8*>(qkv + (tok0 + q) * ld_qkv + q_off + h * D + ks * 32 + fg * 8);
  }
  int kv_len = lens ? lens[b] : S;
  kv_len = kv_len > S ? S : kv_len;

  f32x4 o[NDT][QT];
#pragma unroll
  for (int i = 0; i < NDT; ++i)
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) o[i][qt] = f32x4{0.f, 0.f, 0.f, 0.f};
  // running max in the SCALED (log2) domain; raw scores are scaled inside exp2's FMA
  float m_run[QT], l_run[QT];
#pragma unroll
  for (int qt = 0; qt < QT; ++qt) { m_run[qt] = -INFINITY; l_run[qt] = 0.f; }

  // Causal: keys beyond the block's last query are never needed.
  int key_end = kv_len;
  if (causal) {
    const int qlast = blockIdx.x * QROWS + QROWS - 1;
    key_end = key_end < qlast + 1 ? key_end : qlast + 1;
  }
  const int nblk = (key_end + KB - 1) / KB;

  for (int kb = 0; kb < nblk; ++kb) {
    const int key0 = kb * KB;
    if (kb > 0) load_kv(key0, 0);
    __syncthreads();  // previous block's LDS reads are done
#pragma unroll
    for (int part = 0; part < NPART; ++part) {
      if (part > 0) load_kv(key0, part);
      store_kv(part);
    }
    __syncthreads();

    // ---- S^T = K . Q^T ----
    f32x4 s[NKT][QT];
#pragma unroll
    for (int kt = 0; kt < NKT; ++kt) {
#pragma unroll
      for (int qt = 0; qt < QT; ++qt) s[kt][qt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) {
        const frag8 kf = *reinterpret_cast<const frag8*>(Ks + kswz<C::CPR>(kt * 16 + fr, ks * 4 + fg));
#pragma unroll
        for (int qt = 0; qt < QT; ++qt) s[kt][qt] = mma16<T>(kf, qf[qt][ks], s[kt][qt]);
      }
    }

    // ---- mask (only blocks that need it: wave-uniform test), online softmax
    // (lane-local query q = q0 + qt*16 + fr) ----
    const bool need_mask = key0 + KB > kv_len || (causal && key0 + KB - 1 > q0);
#pragma unroll
    for (int qt = 0; qt < QT; ++qt) {
      const int q = q0 + qt * 16 + fr;
      float mx = -INFINITY;
      if (need_mask) {
#pragma unroll
        for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int key = key0 + kt * 16 + fg * 4 + e;
            const bool masked = (key >= kv_len) || (causal && key > q);
            s[kt][qt][e] = masked ? -INFINITY : s[kt][qt][e];
            mx = fmaxf(mx, s[kt][qt][e]);
          }
      } else {
#pragma unroll
        for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
          for (int e = 0; e < 4; ++e) mx = fmaxf(mx, s[kt][qt][e]);
      }
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float m_new = fmaxf(m_run[qt], mx * scale_log2e);   // scale > 0: max commutes
      const float m_use = (m_new == -INFINITY) ? 0.f : m_new;
      if (kb > 0) {  // the first block has nothing to rescale
        const float alpha = exp2f(m_run[qt] - m_use);
        l_run[qt] *= alpha;
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt) o[dt][qt] *= alpha;
      }
      m_run[qt] = m_new;
      float ls = 0.f;
#pragma unroll
      for (int kt = 0; kt < NKT; ++kt)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float p = exp2f(fmaf(s[kt][qt][e], scale_log2e, -m_use));
          s[kt][qt][e] = p;
          ls += p;
        }
      l_run[qt] += ls;  // partial over this lane's keys; reduced across fg at the end
    }

    // ---- O^T += V^T . P^T over 4 chunks of 32 keys ----
#pragma unroll
    for (int c = 0; c < KB / 32; ++c) {
      frag8 pf[QT];
#pragma unroll
      for (int qt = 0; qt < QT; ++qt) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          pf[qt][e] = (T)s[2 * c][qt][e];
          pf[qt][4 + e] = (T)s[2 * c + 1][qt][e];
        }
      }
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) {
        const T* vr = Vt + (dt * 16 + fr) * C::VT_LD + c * 32 + fg * 4;
        const frag4 lo = *reinterpret_cast<const frag4*>(vr);
        const frag4 hi = *reinterpret_cast<const frag4*>(vr + 16);
        const frag8 vf = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
        for (int qt = 0; qt < QT; ++qt) o[dt][qt] = mma16<T>(vf, pf[qt], o[dt][qt]);
      }
    }
  }

  // ---- normalise and store: lane holds O[q][dt*16 + 4*fg + e] ----
#pragma unroll
  for (int qt = 0; qt < QT; ++qt) {
    float l = l_run[qt];
    l += __shfl_xor(l, 16, 64);
    l += __shfl_xor(l, 32, 64);
    const float inv = l > 0.f ? 1.f / l : 0.f;
    const int q = q0 + qt * 16 + fr;
    if (q >= S) continue;
    T* op = out + (tok0 + q) * ld_out + h * D;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) {
      const frag4 v = {(T)(o[dt][qt][0] * inv), (T)(o[dt][qt][1] * inv),
                       (T)(o[dt][qt][2] * inv), (T)(o[dt][qt][3] * inv)};
      *reinterpret_cast<frag4*>(op + dt * 16 + fg * 4) = v;
    }
  }
}

void attn_fwd(int dtype, uintptr_t qkv, int ld_qkv, int q_off, int k_off, int v_off, int B, int H, int Hkv,
              int S, int D, uintptr_t lens, int causal, uintptr_t out, int ld_out, float scale,
              uintptr_t stream) {
  if (H % Hkv != 0) throw std::invalid_argument("attn: H must be a multiple of Hkv");
  if (ld_qkv % 8 || q_off % 8 || k_off % 8 || v_off % 8 || ld_out % 4)
    throw std::invalid_argument("attn: strides/offsets must be 16-byte aligned");
  if (B <= 0 || S <= 0) return;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  // QT = 2 (128 query rows per block) unless that leaves fewer than 2 blocks per CU
  const long blocks2 = (long)((S + 127) / 128) * H * B;
  int qt = blocks2 < 512 ? 1 : 2;
  if (const char* e = getenv("RDB_ATTN_QT")) qt = atoi(e) == 1 ? 1 : 2;   // A/B override
  dim3 grid((S + 64 * qt - 1) / (64 * qt), H, B), blk(256);
  const float sl2e = scale * 1.4426950408889634f;
#define RDB_ATTN(T, DD)                                                                              \
  if (qt == 1)                                                                                       \
    hipLaunchKernelGGL((attn_fwd_kernel<T, DD, 1>), grid, blk, 0, s, (const T*)qkv, ld_qkv, q_off, k_off, \
                       v_off, H, Hkv, S, (const int*)lens, causal, (T*)out, ld_out, sl2e);             \
  else                                                                                               \
    hipLaunchKernelGGL((attn_fwd_kernel<T, DD, 2>), grid, blk, 0, s, (const T*)qkv, ld_qkv, q_off, k_off, \
                       v_off, H, Hkv, S, (const int*)lens, causal, (T*)out, ld_out, sl2e)
  if (D != 64 && D != 128) throw std::invalid_argument("attn: head dim must be 64 or 128");
  if (dtype == 0) { if (D == 64) RDB_ATTN(bf16, 64); else RDB_ATTN(bf16, 128); }
  else if (dtype == 1) { if (D == 64) RDB_ATTN(f16, 64); else RDB_ATTN(f16, 128); }
  else throw std::invalid_argument("attn: dtype must be bf16 or f16");
#undef RDB_ATTN
  RDB_HIP_CHECK(hipGetLastError());
}

}  // namespace rdb
