// Shared device/host helpers for the Pi0 MI355X (gfx950 / CDNA4) kernels.
// Written for gfx950 only: wave64, MFMA bf16 16x16x32, 160 KiB LDS per CU.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "../../include/pz_abi.h"

typedef unsigned short bf16_t;  // storage type for bf16 tensors
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef int i32x8 __attribute__((ext_vector_type(8)));  // 32 fp8 codes: one v_mfma_*_16x16x128_f8f6f4 operand
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float bf2f(bf16_t h) { return __uint_as_float(((unsigned)h) << 16); }
__device__ __forceinline__ bf16_t f2bf(float f) {
  __bf16 b = (__bf16)f;  // v_cvt_pk_bf16_f32: RNE, NaN preserved
  return __builtin_bit_cast(bf16_t, b);
}
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
// one v_cvt_pk_bf16_f32 (RNE, NaN preserved), lo in bits 0..15
__device__ __forceinline__ unsigned pack2bf(float lo, float hi) {
  return __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2_t{lo, hi}, bf16x2_t));
}

__device__ __forceinline__ float warp_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float warp_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// block-wide sum for blockDim.x == 64 * NW, result broadcast to all threads
template <int NW>
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = warp_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (NW == 1) return v;
  if (l == 0) red[w] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < NW; ++i) t += red[i];
  __syncthreads();
  return t;
}

// Activations with hardware v_exp_f32 / v_rcp_f32 (each ~1 ulp): a plain '/' or __fdividef compiles to the
// IEEE division sequence (v_div_scale / v_div_fmas / v_div_fixup, ~11 instructions) in this build, which made
// the per-element VALU work of every fused activation epilogue (GELU + aux, GeGLU, their backward) 23
// instructions instead of 8 for gelu_tanh.
__device__ __forceinline__ float fast_rcp(float x) { return __builtin_amdgcn_rcpf(x); }
// e^u as 2^(u log2 e) on v_exp_f32
__device__ __forceinline__ float fast_exp(float u) { return __builtin_amdgcn_exp2f(u * 1.4426950408889634f); }

// tanh(u) = 1 - 2 / (e^{2u} + 1): saturates cleanly to +-1
__device__ __forceinline__ float tanh_fast(float u) { return 1.f - 2.f * fast_rcp(fast_exp(2.f * u) + 1.f); }

// gelu(x, approximate="tanh") = 0.5 x (1 + tanh(u)) = x * sigmoid(2u), u = k0 (x + k1 x^3):
// one v_exp_f32, one v_rcp_f32 and 5 FMA / mul (fp32)
__device__ __forceinline__ float gelu_tanh(float x) {
  constexpr float c0 = -2.f * 0.7978845608028654f * 1.4426950408889634f, c1 = c0 * 0.044715f;
  const float e = __builtin_amdgcn_exp2f(x * __builtin_fmaf(c1, x * x, c0));  // e^{-2u}
  return x * fast_rcp(1.f + e);
}
// d/dx gelu_tanh = 0.5 (1 + t) + 0.5 x (1 - t^2) u', t = tanh(u), u' = k0 (1 + 3 k1 x^2).  With s = sigmoid(2u) =
// 0.5 (1 + t) (gelu_tanh's rcp(1 + e^{-2u})) and 1 - t^2 = 4 s (1 - s): grad = s + 2 x s (1 - s) u' -- the same
// exp / rcp as the forward value, so the DGEGLU epilogues get gelu and its derivative from ONE v_exp_f32 and ONE
// v_rcp_f32 (gelu_tanh_both): 12 VALU + 2 transcendental ops per element instead of 23 + 4 (the round-5 tanh form).
// s -> 1 for large x (grad -> 1), e -> inf, s -> 0 for very negative x (grad -> 0): no NaN.
__device__ __forceinline__ void gelu_tanh_both(float x, float& gl, float& gr) {
  constexpr float c0 = -2.f * 0.7978845608028654f * 1.4426950408889634f, c1 = c0 * 0.044715f;
  constexpr float k0 = 0.7978845608028654f, k3 = 3.f * 0.044715f * 0.7978845608028654f;
  const float x2 = x * x;
  const float s = fast_rcp(1.f + __builtin_amdgcn_exp2f(x * __builtin_fmaf(c1, x2, c0)));  // sigmoid(2u)
  gl = x * s;  // == gelu_tanh(x), bit for bit
  gr = __builtin_fmaf(2.f * x * s * (1.f - s), __builtin_fmaf(k3, x2, k0), s);
}
__device__ __forceinline__ float gelu_tanh_grad(float x) {
  float gl, gr;
  gelu_tanh_both(x, gl, gr);
  return gr;
}

__device__ __forceinline__ float silu(float x) { return x * fast_rcp(1.f + fast_exp(-x)); }
__device__ __forceinline__ float silu_grad(float x) {
  const float s = fast_rcp(1.f + fast_exp(-x));
  return s * (1.f + x * (1.f - s));
}

// ---- few-row GEMV path (pz_gemv.hip), chosen by pz_gemm's planner ------------------
bool pz_gemv_supported(const pz_gemm_args* a);
int pz_gemv_launch(const pz_gemm_args* a, hipStream_t st);

// ---- host side error plumbing -------------------------------------------------
void pz_set_error(const char* fmt, ...);
#define PZ_CHECK_ARG(cond, ...)          \
  do {                                   \
    if (!(cond)) {                       \
      pz_set_error(__VA_ARGS__);         \
      return PZ_ERR_INVALID_ARG;         \
    }                                    \
  } while (0)
#define PZ_CHECK_LAUNCH()                                                   \
  do {                                                                      \
    hipError_t e_ = hipGetLastError();                                      \
    if (e_ != hipSuccess) {                                                 \
      pz_set_error("%s: launch failed: %s", __func__, hipGetErrorString(e_)); \
      return PZ_ERR_LAUNCH;                                                 \
    }                                                                       \
  } while (0)
#define PZ_ALIGNED(p, n) ((((uintptr_t)(p)) % (n)) == 0)

// RoPE rotation of one pair (utils.py:4-16: x*cos + rotate_half(x)*sin) with every product rounded
// separately (no FMA contraction): every kernel that applies RoPE (qkv_rope_split, the GEMV and the 8-phase
// GEMM epilogues) produces the same bits from the same bf16 inputs
// (__fmul_rn / __fadd_rn alone do not stop hipcc's default -ffp-contract=fast from fusing a product into
// the add after inlining, differently per call site: contraction is switched off for this scope)
__device__ __forceinline__ void rope_pair(float x1, float x2, float co, float si, float& o1, float& o2) {
#pragma clang fp contract(off)
  o1 = x1 * co - x2 * si;
  o2 = x2 * co + x1 * si;
}


