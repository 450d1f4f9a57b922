// Blockwise 8-bit AdamW over the flat parameter arena (the reference's bnb.optim.AdamW8bit,
// src/agent/train.py:171-175,194-198; algorithm restated in oracle/adamw8bit.py).
//
// HBM-bound: per element it reads p (bf16), g (bf16) and two 1-byte state codes and writes p and
// the two codes (10 B/element vs 22 B for fp32-state AdamW), plus two fp32 absmax per 256 elements.
// One wave owns one 256-element block: 4 consecutive elements per lane (8-byte p/g loads, 4-byte
// code loads), the block's new absmax is a wave max, codes come from a 7-step binary search in the
// LDS-resident 256-entry maps.  Tensors below bnb's min_8bit_size keep fp32 state (segment kind 1),
// in the same launch.  Deterministic (no atomics).
#include "pz_common.h"

namespace {

// 7-step binary search from pivot 127 with midpoint rounding (oracle/adamw8bit.py quantize)
__device__ __forceinline__ unsigned quantize8(const float* __restrict__ q, float x, bool sgn) {
  int pivot = 127, up = 255, lo = 0;
  float lower = sgn ? -1.f : 0.f, upper = 1.f;
  float val = q[pivot];
#pragma unroll
  for (int i = 64; i > 0; i >>= 1) {
    if (x > val) {
      lo = pivot;
      lower = val;
      pivot += i;
    } else {
      up = pivot;
      upper = val;
      pivot -= i;
    }
    val = q[pivot];
  }
  if (x > val) return x > (upper + val) * 0.5f ? (unsigned)up : (unsigned)pivot;
  return x < (lower + val) * 0.5f ? (unsigned)lo : (unsigned)pivot;
}

__global__ void __launch_bounds__(256) adamw8_kernel(pz_adamw8_args a) {
  __shared__ float q1[256], q2[256];
  q1[threadIdx.x] = a.qmap1[threadIdx.x];
  q2[threadIdx.x] = a.qmap2[threadIdx.x];
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int64_t bi = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (bi >= a.nblocks) return;
  // segment of block bi (seg rows: elem offset, numel, first block, fp32-state offset or -1)
  int64_t lo = 0, hi = a.nseg - 1;
  while (lo < hi) {
    const int64_t mid = (lo + hi + 1) >> 1;
    if (a.seg[4 * mid + 2] <= bi) lo = mid;
    else hi = mid - 1;
  }
  const int64_t* sg = a.seg + 4 * lo;
  const int64_t e0 = sg[0] + (bi - sg[2]) * 256 + lane * 4;
  const int64_t end = sg[0] + sg[1];
  const int nv = (int)(end - e0 < 4 ? (end - e0 < 0 ? 0 : end - e0) : 4);
  const float gs = a.gscale ? a.gscale[0] : 1.f;
  bf16_t* P = (bf16_t*)a.p;
  const bf16_t* G = (const bf16_t*)a.g;
  float p[4] = {0.f, 0.f, 0.f, 0.f}, g[4] = {0.f, 0.f, 0.f, 0.f};
  if (nv == 4) {
    const u32x2 pr = *reinterpret_cast<const u32x2*>(P + e0);
    const u32x2 gr = *reinterpret_cast<const u32x2*>(G + e0);
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      p[2 * k] = __uint_as_float(pr[k] << 16);
      p[2 * k + 1] = __uint_as_float(pr[k] & 0xffff0000u);
      g[2 * k] = __uint_as_float(gr[k] << 16);
      g[2 * k + 1] = __uint_as_float(gr[k] & 0xffff0000u);
    }
  } else {
    for (int k = 0; k < nv; ++k) {
      p[k] = bf2f(P[e0 + k]);
      g[k] = bf2f(G[e0 + k]);
    }
  }
  float m[4], v[4];
  const bool fp32_state = sg[3] >= 0;
  if (fp32_state) {
    const int64_t so = sg[3] + (e0 - sg[0]);
    for (int k = 0; k < 4; ++k) {
      m[k] = k < nv ? a.m32[so + k] : 0.f;
      v[k] = k < nv ? a.v32[so + k] : 0.f;
    }
  } else {
    const float am1 = a.absmax1[bi], am2 = a.absmax2[bi];
    unsigned c1 = 0, c2 = 0;
    if (nv == 4) {
      c1 = *reinterpret_cast<const unsigned*>(a.s1 + e0);
      c2 = *reinterpret_cast<const unsigned*>(a.s2 + e0);
    } else {
      for (int k = 0; k < nv; ++k) {
        c1 |= (unsigned)a.s1[e0 + k] << (8 * k);
        c2 |= (unsigned)a.s2[e0 + k] << (8 * k);
      }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      m[k] = __fmul_rn(q1[(c1 >> (8 * k)) & 255], am1);
      v[k] = __fmul_rn(q2[(c2 >> (8 * k)) & 255], am2);
    }
  }
  // every op individually rounded (no FMA contraction): bit-identical to the float32 oracle
  float mx1 = 0.f, mx2 = 0.f;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float gg = __fmul_rn(g[k], gs);
    m[k] = __fadd_rn(__fmul_rn(a.beta1, m[k]), __fmul_rn(a.omb1, gg));
    v[k] = __fadd_rn(__fmul_rn(a.beta2, v[k]), __fmul_rn(a.omb2, __fmul_rn(gg, gg)));
    float pv = __fadd_rn(p[k], __fmul_rn(a.step, __fdiv_rn(m[k], __fadd_rn(__fsqrt_rn(v[k]), a.epsc))));
    if (a.decay != 1.f) pv = __fmul_rn(pv, a.decay);
    p[k] = pv;
    if (k < nv) {
      mx1 = fmaxf(mx1, fabsf(m[k]));
      mx2 = fmaxf(mx2, fabsf(v[k]));
    }
  }
  if (nv == 4) {
    *reinterpret_cast<u32x2*>(P + e0) = u32x2{pack2bf(p[0], p[1]), pack2bf(p[2], p[3])};
  } else {
    for (int k = 0; k < nv; ++k) P[e0 + k] = f2bf(p[k]);
  }
  if (fp32_state) {
    const int64_t so = sg[3] + (e0 - sg[0]);
    for (int k = 0; k < nv; ++k) {
      a.m32[so + k] = m[k];
      a.v32[so + k] = v[k];
    }
    return;
  }
  mx1 = warp_max(mx1);
  mx2 = warp_max(mx2);
  unsigned c1 = 0, c2 = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    // the oracle divides (m / absmax); a reciprocal multiply would differ by an ulp at code midpoints
    const float x1 = mx1 > 0.f ? __fdiv_rn(m[k], mx1) : 0.f, x2 = mx2 > 0.f ? __fdiv_rn(v[k], mx2) : 0.f;
    unsigned k1 = quantize8(q1, x1, true);
    // bnb's sign fix: the m code keeps m's sign bit (a tiny negative m does not collapse to +0)
    if (signbit(q1[k1]) != signbit(m[k])) k1 = m[k] > 0.f ? k1 + 1 : k1 - 1;
    c1 |= (k1 & 255u) << (8 * k);
    c2 |= quantize8(q2, x2, false) << (8 * k);
  }
  if (nv == 4) {
    *reinterpret_cast<unsigned*>(a.s1 + e0) = c1;
    *reinterpret_cast<unsigned*>(a.s2 + e0) = c2;
  } else {
    for (int k = 0; k < nv; ++k) {
      a.s1[e0 + k] = (uint8_t)(c1 >> (8 * k));
      a.s2[e0 + k] = (uint8_t)(c2 >> (8 * k));
    }
  }
  if (lane == 0) {
    a.absmax1[bi] = mx1;
    a.absmax2[bi] = mx2;
  }
}

}  // namespace

extern "C" int pz_adamw8bit(const pz_adamw8_args* a, void* stream) {
  PZ_CHECK_ARG(a && a->p && a->g && a->seg && a->nseg > 0 && a->nblocks > 0 && a->qmap1 && a->qmap2,
               "adamw8bit: bad args");
  PZ_CHECK_ARG(PZ_ALIGNED(a->p, 8) && PZ_ALIGNED(a->g, 8) && (!a->s1 || PZ_ALIGNED(a->s1, 4)) &&
                   (!a->s2 || PZ_ALIGNED(a->s2, 4)),
               "adamw8bit: p/g must be 8-byte and codes 4-byte aligned");
  const int64_t grid = (a->nblocks + 3) / 4;
  PZ_CHECK_ARG(grid < (1LL << 31), "adamw8bit: too many blocks");
  hipLaunchKernelGGL(adamw8_kernel, dim3((unsigned)grid), dim3(256), 0, (hipStream_t)stream, *a);
  PZ_CHECK_LAUNCH();
  return PZ_OK;
}
