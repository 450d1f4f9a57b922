// Blockwise 8-bit AdamW over the flat parameter arena (the reference's bnb.optim.AdamW8bit,
// src/agent/train.py:171-175,194-198; algorithm restated in oracle/adamw8bit.py).
//
// HBM-bound: per element it reads p (bf16), g (bf16) and two 1-byte state codes and writes p and
// the two codes (10 B/element vs 22 B for fp32-state AdamW), plus two fp32 absmax per 256 elements.
// One wave owns one 256-element block: 4 consecutive elements per lane (8-byte p/g loads, 4-byte
// code loads), the block's new absmax is a wave max, codes come from a 7-step binary search in the
// LDS-resident 256-entry maps (searched in breadth-first order: conflict-free banks).  Tensors below bnb's min_8bit_size keep fp32 state (segment kind 1),
// in the same launch.  Deterministic (no atomics).
#include "pz_common.h"

namespace {

// 7-step binary search from pivot 127 with midpoint rounding (oracle/adamw8bit.py quantize), for a lane's 4 codes
// of one map at once, advanced together so each step has 4 independent LDS reads in flight.  The search tree is the complete BST over entries 0..254 (root 127): every
// path ends in a leaf p7 = 2 (j - 127) (even), and the bracketing values it tracks (lower / upper, codes lo / up)
// are always the leaf's in-order neighbours -- entries p7 - 1 and p7 + 1, or the initial sentinels (lower -1 / 0,
// upper 1, lo 0, up 255) at the two ends -- so only the node index is carried per step and the neighbours are
// read once at the end.  The map is read in breadth-first (Eytzinger) order e[j] (node j's children 2j + 1,
// 2j + 2): a depth's candidates are consecutive LDS words.  Same comparisons and float expressions as the oracle,
// so the same codes.
template <bool SGN>
__device__ __forceinline__ void quantize8x4(const float* __restrict__ sq, const float* __restrict__ e,
                                            const float (&x)[4], unsigned (&code)[4]) {
  int j[4];
  float val[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    j[q] = 0;
    val[q] = e[0];
  }
#pragma unroll
  for (int step = 0; step < 7; ++step) {
#pragma unroll
    for (int q = 0; q < 4; ++q) j[q] = 2 * j[q] + (x[q] > val[q] ? 2 : 1);
#pragma unroll
    for (int q = 0; q < 4; ++q) val[q] = e[j[q]];
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int p7 = 2 * (j[q] - 127);
    const float lower = p7 > 0 ? sq[p7 - 1] : (SGN ? -1.f : 0.f);
    const float upper = p7 < 254 ? sq[p7 + 1] : 1.f;
    const unsigned hi_code = x[q] > (upper + val[q]) * 0.5f ? (unsigned)(p7 + 1) : (unsigned)p7;
    const unsigned lo_code = x[q] < (lower + val[q]) * 0.5f ? (unsigned)(p7 > 0 ? p7 - 1 : 0) : (unsigned)p7;
    code[q] = x[q] > val[q] ? hi_code : lo_code;
  }
}

// A block's loads, issued together before its update (the loop below): p / g (8 B per lane), the two 4-code words
// and the two absmax.  Only for whole 8-bit-state lanes (nv == 4); the rest load inside adamw8_block.
struct A8Pre {
  u32x2 pr, gr;
  unsigned c1, c2;
  float am1, am2;
};

// one segment-table row held in registers (reloaded only when a wave's run crosses into the next tensor: the
// update's stores could alias the table as far as the compiler knows, so reading it per block would drain every
// load in flight)
struct A8Seg {
  int64_t off, n, first, s32;
};

__device__ __forceinline__ int64_t rfl64(int64_t x) {  // wave-uniform value -> SGPRs
  const int lo = __builtin_amdgcn_readfirstlane((int)(x & 0xffffffff));
  const int hi = __builtin_amdgcn_readfirstlane((int)(x >> 32));
  return (int64_t)(((uint64_t)(unsigned)hi << 32) | (unsigned)lo);
}

__device__ __forceinline__ A8Seg a8_seg(const pz_adamw8_args& a, int64_t i) {
  return A8Seg{rfl64(a.seg[4 * i]), rfl64(a.seg[4 * i + 1]), rfl64(a.seg[4 * i + 2]), rfl64(a.seg[4 * i + 3])};
}

__device__ __forceinline__ void adamw8_fetch(const pz_adamw8_args& a, int64_t bi, const A8Seg& sg, int lane,
                                             A8Pre& f) {
  const int64_t e0 = sg.off + (bi - sg.first) * 256 + lane * 4;
  if (sg.s32 >= 0 || sg.off + sg.n - e0 < 4) return;
  f.pr = *reinterpret_cast<const u32x2*>((const bf16_t*)a.p + e0);
  f.gr = *reinterpret_cast<const u32x2*>((const bf16_t*)a.g + e0);
  f.c1 = *reinterpret_cast<const unsigned*>(a.s1 + e0);
  f.c2 = *reinterpret_cast<const unsigned*>(a.s2 + e0);
  f.am1 = a.absmax1[bi];
  f.am2 = a.absmax2[bi];
}

__device__ __forceinline__ void adamw8_block(const pz_adamw8_args& a, const float* q1, const float* q2,
                                             const float* e1, const float* e2, int64_t bi, const A8Seg& sg,
                                             int lane, const A8Pre& f, float gs) {
  const int64_t e0 = sg.off + (bi - sg.first) * 256 + lane * 4;
  const int64_t end = sg.off + sg.n;
  const int nv = (int)(end - e0 < 4 ? (end - e0 < 0 ? 0 : end - e0) : 4);
  bf16_t* P = (bf16_t*)a.p;
  const bf16_t* G = (const bf16_t*)a.g;
  float p[4] = {0.f, 0.f, 0.f, 0.f}, g[4] = {0.f, 0.f, 0.f, 0.f};
  const bool fp32_state = sg.s32 >= 0;
  if (nv == 4) {
    const u32x2 pr = fp32_state ? *reinterpret_cast<const u32x2*>(P + e0) : f.pr;
    const u32x2 gr = fp32_state ? *reinterpret_cast<const u32x2*>(G + e0) : f.gr;
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
  if (fp32_state) {
    const int64_t so = sg.s32 + (e0 - sg.off);
    for (int k = 0; k < 4; ++k) {
      m[k] = k < nv ? a.m32[so + k] : 0.f;
      v[k] = k < nv ? a.v32[so + k] : 0.f;
    }
  } else {
    float am1 = f.am1, am2 = f.am2;
    unsigned c1 = 0, c2 = 0;
    if (nv == 4) {
      c1 = f.c1;
      c2 = f.c2;
    } else {
      am1 = a.absmax1[bi];
      am2 = a.absmax2[bi];
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
    const int64_t so = sg.s32 + (e0 - sg.off);
    for (int k = 0; k < nv; ++k) {
      a.m32[so + k] = m[k];
      a.v32[so + k] = v[k];
    }
    return;
  }
  mx1 = warp_max(mx1);
  mx2 = warp_max(mx2);
  unsigned c1 = 0, c2 = 0;
  {
    float xs[4];
    unsigned code[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)  // the oracle divides (m / absmax); a reciprocal multiply would differ by an ulp
      xs[k] = mx1 > 0.f ? __fdiv_rn(m[k], mx1) : 0.f;
    quantize8x4<true>(q1, e1, xs, code);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      unsigned k1 = code[k];
      // bnb's sign fix: the m code keeps m's sign bit (a tiny negative m does not collapse to +0)
      if (signbit(q1[k1]) != signbit(m[k])) k1 = m[k] > 0.f ? k1 + 1 : k1 - 1;
      c1 |= (k1 & 255u) << (8 * k);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) xs[k] = mx2 > 0.f ? __fdiv_rn(v[k], mx2) : 0.f;
    quantize8x4<false>(q2, e2, xs, code);
#pragma unroll
    for (int k = 0; k < 4; ++k) c2 |= code[k] << (8 * k);
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


// Persistent waves: wave w of the grid updates the contiguous blocks [w * per_wave, (w + 1) * per_wave), so the
// qmaps are staged into LDS once per workgroup and the segment of a block is found by one binary search per wave
// and then advanced (round 4's one-block-per-wave grid paid a 256-entry LDS fill, a barrier and a ~9-step chain of
// dependent segment-table loads per 256 elements: 1.6 TB/s).
__global__ void __launch_bounds__(256) adamw8_kernel(pz_adamw8_args a, int64_t per_wave) {
  __shared__ float q1[256], q2[256], e1[256], e2[256];
  q1[threadIdx.x] = a.qmap1[threadIdx.x];
  q2[threadIdx.x] = a.qmap2[threadIdx.x];
  {  // BFS node j (depth d, position k in its level) = sorted entry (2k + 1) * 2^(7 - d) - 1
    const int j = threadIdx.x, d = 31 - __clz(j + 1), k = j + 1 - (1 << d);
    const int src = j < 255 ? ((2 * k + 1) << (7 - d)) - 1 : 255;
    e1[j] = a.qmap1[src];
    e2[j] = a.qmap2[src];
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int64_t w = (int64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t b0 = w * per_wave, b1 = min(a.nblocks, b0 + per_wave);
  if (b0 >= b1) return;
  int64_t lo = 0, hi = a.nseg - 1;  // segment of b0 (rows: elem offset, numel, first block, fp32-state offset or -1)
  while (lo < hi) {
    const int64_t mid = (lo + hi + 1) >> 1;
    if (a.seg[4 * mid + 2] <= b0) lo = mid;
    else hi = mid - 1;
  }
  const float gs = a.gscale ? a.gscale[0] : 1.f;
  // per tensor (segment) of the run, block by block: each block's loads, then its update.  (Issuing block bi + 1's
  // loads before block bi's update measured no faster: 14.9 vs 14.4 ms per step, profiles/r06/optim_bench_r6b.log --
  // the update's dependent search / division chain, not load latency, sets the time; profiles/r05/optim_bench_r5.txt)
  lo = rfl64(lo);
  for (int64_t bi = b0; bi < b1; ++lo) {
    const A8Seg sg = a8_seg(a, lo);
    const int64_t send = min(b1, lo + 1 < a.nseg ? rfl64(a.seg[4 * (lo + 1) + 2]) : a.nblocks);
    for (; bi < send; ++bi) {
      A8Pre cur{};
      adamw8_fetch(a, bi, sg, lane, cur);
      adamw8_block(a, q1, q2, e1, e2, bi, sg, lane, cur, gs);
    }
  }
}

}  // namespace

extern "C" int pz_adamw8bit(const pz_adamw8_args* a, void* stream) {
  PZ_CHECK_ARG(a && a->p && a->g && a->seg && a->nseg > 0 && a->nblocks > 0 && a->qmap1 && a->qmap2,
               "adamw8bit: bad args");
  PZ_CHECK_ARG(PZ_ALIGNED(a->p, 8) && PZ_ALIGNED(a->g, 8) && (!a->s1 || PZ_ALIGNED(a->s1, 4)) &&
                   (!a->s2 || PZ_ALIGNED(a->s2, 4)),
               "adamw8bit: p/g must be 8-byte and codes 4-byte aligned");
  // as many workgroups of 4 waves per CU as are resident at once (the occupancy query), each wave a contiguous run
  // of blocks
  int dev = 0, cus = 256, per_cu = 4;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, adamw8_kernel, 256, 0) != hipSuccess || per_cu < 1)
    per_cu = 4;
  (void)hipGetLastError();
  const int64_t waves = (int64_t)cus * per_cu * 4;
  const int64_t per_wave = (a->nblocks + waves - 1) / waves;
  const int64_t grid = ((a->nblocks + per_wave - 1) / per_wave + 3) / 4;
  hipLaunchKernelGGL(adamw8_kernel, dim3((unsigned)grid), dim3(256), 0, (hipStream_t)stream, *a, per_wave);
  PZ_CHECK_LAUNCH();
  return PZ_OK;
}
