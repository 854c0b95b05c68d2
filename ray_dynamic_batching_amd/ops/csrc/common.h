// Shared device helpers for the gfx950 (CDNA4) kernels of ray_dynamic_batching_amd.
//
// Everything here is written for a 64-lane wavefront and the gfx950 MFMA
// instruction set; there is no portability layer.
#pragma once
#include <stdexcept>
#include <string>
// RDB_EXPERIMENTAL_KERNELS: kernel variants that lost their A/Bs (stream-K,
// the full-row GEMM+LayerNorm, the LNOUT / staged-partial-statistics LayerNorm
// epilogues) are only compiled into an opt-in build:
//   python -m ray_dynamic_batching_amd._build --variant experimental -D RDB_EXPERIMENTAL_KERNELS
// (loaded with RDB_OPS_SO=<that .so>).  The default library's entry points
// for them throw.
#ifdef RDB_EXPERIMENTAL_KERNELS
#define RDB_EXPERIMENTAL 1
#else
#define RDB_EXPERIMENTAL 0
#endif
#define RDB_EXPERIMENTAL_MISSING(WHAT)                                                                 \
  throw std::runtime_error(std::string(WHAT) +                                                          \
                           ": experimental kernel not in this build (python -m ray_dynamic_batching_amd._build " \
                           "--variant experimental -D RDB_EXPERIMENTAL_KERNELS, then RDB_OPS_SO=<that .so>)")
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

namespace rdb {

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16;
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

constexpr int kWave = 64;

__device__ __forceinline__ float bf2f(bf16 x) { return (float)x; }
__device__ __forceinline__ bf16 f2bf(float x) { return (bf16)x; }  // RNE, NaN-preserving (v_cvt_pk_bf16_f32)

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Epilogue activations shared by GEMM / conv kernels.
// ACT_SWIGLU is a GEMM-only pairing epilogue: W rows are interleaved (gate_j, up_j),
// the output has N/2 columns and holds silu(gate_j) * up_j.
enum Act : int { ACT_NONE = 0, ACT_GELU = 1, ACT_RELU = 2, ACT_TANH = 3, ACT_SILU = 4, ACT_GELU_TANH = 5, ACT_SWIGLU = 6, ACT_SIGMOID = 7 };

// erf with |error| <= 1.5e-7 (Abramowitz & Stegun 7.1.26): one exp, one rcp,
// five FMAs and no branches -- ocml's erff is a branchy piecewise polynomial
// that dominated the GELU epilogue of the FFN-up GEMM.
__device__ __forceinline__ float fast_erf(float x) {
  const float a = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, a, 1.0f));
  float p = fmaf(1.061405429f, t, -1.453152027f);
  p = fmaf(p, t, 1.421413741f);
  p = fmaf(p, t, -0.284496736f);
  p = fmaf(p, t, 0.254829592f);
  const float y = 1.0f - p * t * __expf(-a * a);
  return copysignf(y, x);
}

template <int ACT>
__device__ __forceinline__ float apply_act(float x) {
  if constexpr (ACT == ACT_GELU) {
#ifdef RDB_GELU_OLD   // A/B build: the previous formulation
    return 0.5f * x * (1.0f + fast_erf(x * 0.70710678118654752f));
#endif
    // exact-erf GELU, rewritten so adjacent calls pack into v_pk_*_f32 (no
    // copysign, the 1/sqrt2 folded into the constants):
    //   0.5 x (1 + erf(x/sqrt2)) = 0.5 x + 0.5 |x| erf(|x|/sqrt2)
    // erf(a) = 1 - t P(t) exp(-a^2), t = 1 / (1 + p a)  (A&S 7.1.26, |err| <= 1.5e-7)
    // exp(-x^2/2) = exp2(-x^2 * log2(e) / 2) on v_exp_f32 (argument <= 0)
    const float ax = fabsf(x);
    const float t = __builtin_amdgcn_rcpf(fmaf(0.23164193f, ax, 1.0f));   // 0.3275911 / sqrt2
    float p = fmaf(1.061405429f, t, -1.453152027f);
    p = fmaf(p, t, 1.421413741f);
    p = fmaf(p, t, -0.284496736f);
    p = fmaf(p, t, 0.254829592f);
    const float e = __builtin_amdgcn_exp2f(x * x * -0.72134752044448170f);
    const float erfa = fmaf(-(p * t), e, 1.0f);
    return fmaf(0.5f * ax, erfa, 0.5f * x);
  } else if constexpr (ACT == ACT_RELU) {
    return fmaxf(x, 0.0f);
  } else if constexpr (ACT == ACT_TANH) {
    return tanhf(x);
  } else if constexpr (ACT == ACT_SILU) {
    // x * sigmoid(x) with v_exp_f32 + v_rcp_f32 (1 ulp) instead of an IEEE
    // division sequence (~10 VALU per element); exp2 overflow -> rcp(inf) = 0
    return x * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(x * -1.4426950408889634f));
  } else if constexpr (ACT == ACT_GELU_TANH) {
    // 0.5 x (1 + tanh(u)) == x * sigmoid(2u), u = sqrt(2/pi) (x + 0.044715 x^3):
    // the same function without ocml's branchy tanhf (which spilled the GEMM epilogue)
    const float u2 = x * fmaf(-0.10294324f, x * x, -2.3022082f);   // -2u * log2(e)
    return x * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(u2));
  } else if constexpr (ACT == ACT_SIGMOID) {
    return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(x * -1.4426950408889634f));
  } else {
    return x;
  }
}

// Bijective XCD-aware remap of a linear workgroup id (MI355X: 8 XCDs, blocks
// dealt round-robin).  Consecutive *logical* tiles land on the same XCD so
// they share that XCD's L2 (guide T1; bijective form for nwg % 8 != 0).
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int q = nwg >> 3, r = nwg & 7;
  const int xcd = orig & 7, idx = orig >> 3;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
}

}  // namespace rdb

#define RDB_HIP_CHECK(expr)                                                        \
  do {                                                                             \
    hipError_t _e = (expr);                                                        \
    if (_e != hipSuccess) throw std::runtime_error(std::string("HIP error: ") +    \
                                                   hipGetErrorString(_e) + " @ " + \
                                                   __FILE__ + ":" + std::to_string(__LINE__)); \
  } while (0)
