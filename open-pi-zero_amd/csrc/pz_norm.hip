// Row normalisations for the Pi0 path (memory-bound, one wave per row,
// 16-byte vector loads, fp32 statistics):
//   Gemma RMSNorm (paligemma/modules.py:7-21) and SigLIP LayerNorm
//   (siglip.py:211,217,290), forward + backward, plus the column reductions
//   used for norm-weight / bias / position-embedding gradients.
#include <string.h>

#include "pz_common.h"

namespace {

constexpr int ROWS_PER_PART = 16;  // rows folded into one fp32 partial row of dw/db (4 per wave: enough workgroups to hide latency)

__device__ __forceinline__ void load8(const bf16_t* p, float (&v)[8]) {
  u32x4 r = *reinterpret_cast<const u32x4*>(p);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = __uint_as_float(r[i] << 16);
    v[2 * i + 1] = __uint_as_float(r[i] & 0xffff0000u);
  }
}
__device__ __forceinline__ void unpack8(const u32x4& r, float (&v)[8]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = __uint_as_float(r[i] << 16);
    v[2 * i + 1] = __uint_as_float(r[i] & 0xffff0000u);
  }
}
__device__ __forceinline__ void store8(bf16_t* p, const float (&v)[8]) {
  u32x4 r;
#pragma unroll
  for (int i = 0; i < 4; ++i) r[i] = pack2bf(v[2 * i], v[2 * i + 1]);
  *reinterpret_cast<u32x4*>(p) = r;
}

// --------------------------------------------------------------- RMSNorm ---
template <int MAXC>
__global__ void __launch_bounds__(256) rmsnorm_fwd_kernel(const bf16_t* __restrict__ x, int64_t ldx,
                                                          const bf16_t* __restrict__ w, bf16_t* y,
                                                          int64_t ldy, float* rstd, int64_t R, int D,
                                                          float eps) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= R) return;
  const int nc = D / 8;
  // the weight chunks loaded with the row, not after its reduction: one memory round trip
  u32x4 wq[MAXC];
#pragma unroll
  for (int c = 0; c < MAXC; ++c)
    wq[c] = lane + 64 * c < nc ? *reinterpret_cast<const u32x4*>(w + (lane + 64 * c) * 8) : u32x4{0u, 0u, 0u, 0u};
  float v[MAXC][8];
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int ch = lane + 64 * c;
    if (ch < nc) {
      load8(x + row * ldx + ch * 8, v[c]);
#pragma unroll
      for (int i = 0; i < 8; ++i) ss += v[c][i] * v[c][i];
    }
  }
  ss = warp_sum(ss);
  const float r = rsqrtf(ss / (float)D + eps);
  if (rstd && lane == 0) rstd[row] = r;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int ch = lane + 64 * c;
    if (ch < nc) {
      float wv[8], o[8];
      unpack8(wq[c], wv);
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = v[c][i] * r * (1.f + wv[i]);
      store8(y + row * ldy + ch * 8, o);
    }
  }
}

// one block = ROWS_PER_PART rows (4 waves x 4 rows); dw partial per block
template <int MAXC>
__global__ void __launch_bounds__(256) rmsnorm_bwd_kernel(
    const bf16_t* __restrict__ dy, int64_t lddy, const bf16_t* __restrict__ x, int64_t ldx,
    const bf16_t* __restrict__ w, const float* __restrict__ rstd, const bf16_t* dres, bf16_t* dx,
    int64_t lddx, float* dw_part, int64_t R, int D) {
  __shared__ float red[4][MAXC * 64 * 8 > 4096 ? 4096 : MAXC * 64 * 8];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nc = D / 8;
  float dwacc[MAXC][8];
#pragma unroll
  for (int c = 0; c < MAXC; ++c)
#pragma unroll
    for (int i = 0; i < 8; ++i) dwacc[c][i] = 0.f;
  const int64_t r0 = (int64_t)blockIdx.x * ROWS_PER_PART;
  for (int rr = wave; rr < ROWS_PER_PART; rr += 4) {
    const int64_t row = r0 + rr;
    if (row >= R) break;
    const float r = rstd[row];
    float xv[MAXC][8], gv[MAXC][8];
    float dot = 0.f;
    u32x4 dr[MAXC];  // residual gradient: loaded with x / dy, not after the row reduction (one memory round trip)
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      const int ch = lane + 64 * c;
      dr[c] = u32x4{0u, 0u, 0u, 0u};
      if (ch < nc && dres) dr[c] = *reinterpret_cast<const u32x4*>(dres + row * lddx + ch * 8);
    }
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      const int ch = lane + 64 * c;
      if (ch < nc) {
        float dyv[8], wv[8];
        load8(x + row * ldx + ch * 8, xv[c]);
        load8(dy + row * lddy + ch * 8, dyv);
        load8(w + ch * 8, wv);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          gv[c][i] = dyv[i] * (1.f + wv[i]);
          dot += gv[c][i] * xv[c][i];
          dwacc[c][i] += dyv[i] * xv[c][i] * r;
        }
      }
    }
    dot = warp_sum(dot);
    const float k = r * r * r * dot / (float)D;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      const int ch = lane + 64 * c;
      if (ch < nc) {
        float o[8];
        unpack8(dr[c], o);
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] += r * gv[c][i] - k * xv[c][i];
        store8(dx + row * lddx + ch * 8, o);
      }
    }
  }
  if (!dw_part) return;
  // reduce dwacc over the 4 waves -> one partial row
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int ch = lane + 64 * c;
    if (ch < nc)
#pragma unroll
      for (int i = 0; i < 8; ++i) red[wave][ch * 8 + i] = dwacc[c][i];
  }
  __syncthreads();
  for (int n = threadIdx.x; n < D; n += 256)
    dw_part[(int64_t)blockIdx.x * D + n] = red[0][n] + red[1][n] + red[2][n] + red[3][n];
}

// ------------------------------------------------------------- LayerNorm ---
template <int MAXC>
__global__ void __launch_bounds__(256) layernorm_fwd_kernel(const bf16_t* __restrict__ x, int64_t ldx,
                                                            const bf16_t* __restrict__ w,
                                                            const bf16_t* __restrict__ b, bf16_t* y,
                                                            int64_t ldy, float* mean, float* rstd,
                                                            int64_t R, int D, float eps) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= R) return;
  const int nc = D / 8;
  // the weight and bias chunks loaded with the row, not after its reductions: one memory round trip
  u32x4 wq[MAXC], bq[MAXC];
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const bool ok = lane + 64 * c < nc;
    wq[c] = ok ? *reinterpret_cast<const u32x4*>(w + (lane + 64 * c) * 8) : u32x4{0u, 0u, 0u, 0u};
    bq[c] = ok ? *reinterpret_cast<const u32x4*>(b + (lane + 64 * c) * 8) : u32x4{0u, 0u, 0u, 0u};
  }
  float v[MAXC][8];
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int ch = lane + 64 * c;
    if (ch < nc) {
      load8(x + row * ldx + ch * 8, v[c]);
#pragma unroll
      for (int i = 0; i < 8; ++i) s += v[c][i];
    }
  }
  const float mu = warp_sum(s) / (float)D;
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int ch = lane + 64 * c;
    if (ch < nc)
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float d = v[c][i] - mu;
        ss += d * d;
      }
  }
  const float r = rsqrtf(warp_sum(ss) / (float)D + eps);
  if (lane == 0) {
    if (mean) mean[row] = mu;
    if (rstd) rstd[row] = r;
  }
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int ch = lane + 64 * c;
    if (ch < nc) {
      float wv[8], bv[8], o[8];
      unpack8(wq[c], wv);
      unpack8(bq[c], bv);
#pragma unroll
      for (int i = 0; i < 8; ++i) o[i] = (v[c][i] - mu) * r * wv[i] + bv[i];
      store8(y + row * ldy + ch * 8, o);
    }
  }
}

template <int MAXC>
__global__ void __launch_bounds__(256) layernorm_bwd_kernel(
    const bf16_t* __restrict__ dy, int64_t lddy, const bf16_t* __restrict__ x, int64_t ldx,
    const bf16_t* __restrict__ w, const float* __restrict__ mean, const float* __restrict__ rstd,
    const bf16_t* dres, bf16_t* dx, int64_t lddx, float* dw_part, float* db_part, int64_t R, int D) {
  __shared__ float red[4][2048];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int nc = D / 8;
  float dwacc[MAXC][8], dbacc[MAXC][8];
#pragma unroll
  for (int c = 0; c < MAXC; ++c)
#pragma unroll
    for (int i = 0; i < 8; ++i) dwacc[c][i] = dbacc[c][i] = 0.f;
  const int64_t r0 = (int64_t)blockIdx.x * ROWS_PER_PART;
  for (int rr = wave; rr < ROWS_PER_PART; rr += 4) {
    const int64_t row = r0 + rr;
    if (row >= R) break;
    const float mu = mean[row], r = rstd[row];
    float xh[MAXC][8], gv[MAXC][8];
    float sg = 0.f, sgx = 0.f;
    u32x4 dr[MAXC];  // residual gradient: loaded with x / dy, not after the row reductions
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      const int ch = lane + 64 * c;
      dr[c] = u32x4{0u, 0u, 0u, 0u};
      if (ch < nc && dres) dr[c] = *reinterpret_cast<const u32x4*>(dres + row * lddx + ch * 8);
    }
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      const int ch = lane + 64 * c;
      if (ch < nc) {
        float dyv[8], wv[8];
        load8(x + row * ldx + ch * 8, xh[c]);
        load8(dy + row * lddy + ch * 8, dyv);
        load8(w + ch * 8, wv);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          xh[c][i] = (xh[c][i] - mu) * r;
          gv[c][i] = dyv[i] * wv[i];
          sg += gv[c][i];
          sgx += gv[c][i] * xh[c][i];
          dwacc[c][i] += dyv[i] * xh[c][i];
          dbacc[c][i] += dyv[i];
        }
      }
    }
    sg = warp_sum(sg) / (float)D;
    sgx = warp_sum(sgx) / (float)D;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      const int ch = lane + 64 * c;
      if (ch < nc) {
        float o[8];
        unpack8(dr[c], o);
#pragma unroll
        for (int i = 0; i < 8; ++i) o[i] += r * (gv[c][i] - sg - xh[c][i] * sgx);
        store8(dx + row * lddx + ch * 8, o);
      }
    }
  }
  for (int pass = 0; pass < 2; ++pass) {
    float* dst = pass == 0 ? dw_part : db_part;
    if (!dst) continue;
#pragma unroll
    for (int c = 0; c < MAXC; ++c) {
      const int ch = lane + 64 * c;
      if (ch < nc)
#pragma unroll
        for (int i = 0; i < 8; ++i) red[wave][ch * 8 + i] = pass == 0 ? dwacc[c][i] : dbacc[c][i];
    }
    __syncthreads();
    for (int n = threadIdx.x; n < D; n += 256)
      dst[(int64_t)blockIdx.x * D + n] = red[0][n] + red[1][n] + red[2][n] + red[3][n];
    __syncthreads();
  }
}

__global__ void reduce_parts_kernel(const float* __restrict__ part, int64_t P, int64_t D, bf16_t* out,
                                    int beta) {
  const int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= D) return;
  float s = 0.f;
  for (int64_t p = 0; p < P; ++p) s += part[p * D + n];
  if (beta) s += bf2f(out[n]);
  out[n] = f2bf(s);
}

// Vectorised fixed-order reduction of P fp32 partial rows (D % 4 == 0): a 256-thread block owns
// 4*CT columns; CT column-threads read float4s, 256/CT part-lanes stride over P (4 loads in flight),
// then the part-lanes are folded through LDS in a fixed order (deterministic, run to run).
template <int CT>
__device__ __forceinline__ void reduce_parts4_body(const float* __restrict__ part, int64_t P, int64_t D, bf16_t* out,
                                                   int beta, int64_t bid) {
  constexpr int PL = 256 / CT;
  __shared__ f32x4 red[PL][CT];
  const int ct = threadIdx.x % CT, pl = threadIdx.x / CT;
  const int64_t c = (bid * CT + ct) * 4;
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
  if (c < D) {
    const float* src = part + c;
    int64_t p = pl;
    // 16 loads in flight per thread (the norm-backward partials: P = rows / 16, e.g. 1104 x 2048 -> 17 per
    // part-lane, one round instead of five), summed in a fixed tree
    for (; p + 15 * PL < P; p += 16 * PL) {
      f32x4 v[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) v[u] = *reinterpret_cast<const f32x4*>(src + (p + u * PL) * D);
#pragma unroll
      for (int w = 8; w > 0; w >>= 1)
#pragma unroll
        for (int u = 0; u < w; ++u) v[u] += v[u + w];
      s += v[0];
    }
    for (; p + 3 * PL < P; p += 4 * PL) {
      const f32x4 a = *reinterpret_cast<const f32x4*>(src + p * D);
      const f32x4 b = *reinterpret_cast<const f32x4*>(src + (p + PL) * D);
      const f32x4 e = *reinterpret_cast<const f32x4*>(src + (p + 2 * PL) * D);
      const f32x4 f = *reinterpret_cast<const f32x4*>(src + (p + 3 * PL) * D);
      s += (a + b) + (e + f);
    }
    for (; p < P; p += PL) s += *reinterpret_cast<const f32x4*>(src + p * D);
  }
  red[pl][ct] = s;
  __syncthreads();
  // fold the part-lanes as a fixed tree (log2(PL) barrier steps instead of PL - 1 dependent LDS reads)
#pragma unroll
  for (int w = PL / 2; w > 0; w >>= 1) {
    if (pl < w) red[pl][ct] += red[pl + w][ct];
    __syncthreads();
  }
  if (pl == 0 && c < D) {
    s = red[0][ct];
    u32x2 o;
    if (beta) {
      const u32x2 prev = *reinterpret_cast<const u32x2*>(out + c);
      s[0] += __uint_as_float(prev[0] << 16);
      s[1] += __uint_as_float(prev[0] & 0xffff0000u);
      s[2] += __uint_as_float(prev[1] << 16);
      s[3] += __uint_as_float(prev[1] & 0xffff0000u);
    }
    o[0] = pack2bf(s[0], s[1]);
    o[1] = pack2bf(s[2], s[3]);
    *reinterpret_cast<u32x2*>(out + c) = o;
  }
}

template <int CT>
__global__ void __launch_bounds__(256) reduce_parts4_kernel(const float* __restrict__ part, int64_t P,
                                                            int64_t D, bf16_t* out, int beta) {
  reduce_parts4_body<CT>(part, P, D, out, beta, blockIdx.x);
}

// several independent reductions in one launch (a layer's norm weight / bias and Linear bias gradients):
// workgroup ranges [blk0[i], blk0[i + 1]) belong to segment i
constexpr int RED_MAXSEG = 8;
struct RedSegs {
  const float* part[RED_MAXSEG];
  bf16_t* out[RED_MAXSEG];
  int64_t P[RED_MAXSEG], D[RED_MAXSEG];
  int beta[RED_MAXSEG], blk0[RED_MAXSEG + 1];
  int n;
};

__global__ void __launch_bounds__(256) reduce_parts4_multi_kernel(RedSegs a) {
  int i = 0;
  while (i + 1 < a.n && (int)blockIdx.x >= a.blk0[i + 1]) ++i;  // workgroup-uniform
  reduce_parts4_body<4>(a.part[i], a.P[i], a.D[i], a.out[i], a.beta[i], (int64_t)blockIdx.x - a.blk0[i]);
}

// column sums of a bf16 matrix: pass 1 -> ws[chunk][n], pass 2 -> out
__global__ void colsum_pass1(const bf16_t* __restrict__ X, int64_t ld, int64_t M, int64_t N,
                             int64_t rows_per_chunk, float* ws) {
  const int64_t n2 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 2;
  if (n2 >= N) return;
  const int64_t r0 = (int64_t)blockIdx.y * rows_per_chunk;
  const int64_t r1 = min(M, r0 + rows_per_chunk);
  float s0 = 0.f, s1 = 0.f;
  const bool two = n2 + 1 < N;
  for (int64_t r = r0; r < r1; ++r) {
    s0 += bf2f(X[r * ld + n2]);
    if (two) s1 += bf2f(X[r * ld + n2 + 1]);
  }
  ws[blockIdx.y * N + n2] = s0;
  if (two) ws[blockIdx.y * N + n2 + 1] = s1;
}

// colsum pass 1 for N % 8 == 0, ld % 8 == 0: 32 column-threads x 8 row-lanes per block, 16-B
// loads (8 columns), one block row per `rpc` rows -> ws[chunk][N] (fp32, fixed order).
__global__ void __launch_bounds__(256) colsum8_pass1(const bf16_t* __restrict__ X, int64_t ld, int64_t M,
                                                     int64_t N, int64_t rpc, float* ws) {
  __shared__ float red[8][32 * 8 + 4];
  const int ct = threadIdx.x & 31, rl = threadIdx.x >> 5;
  const int64_t c = ((int64_t)blockIdx.x * 32 + ct) * 8;
  const int64_t r0 = (int64_t)blockIdx.y * rpc;
  const int64_t r1 = min(M, r0 + rpc);
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (c < N) {
    int64_t r = r0 + rl;
    for (; r + 56 < r1; r += 64) {  // 8 rows' 16-B loads in flight per thread
      u32x4 w[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) w[u] = *reinterpret_cast<const u32x4*>(X + (r + 8 * u) * ld + c);
#pragma unroll
      for (int u = 0; u < 8; ++u)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          s[2 * e] += __uint_as_float(w[u][e] << 16);
          s[2 * e + 1] += __uint_as_float(w[u][e] & 0xffff0000u);
        }
    }
    for (; r < r1; r += 8) {
      float v[8];
      load8(X + r * ld + c, v);
#pragma unroll
      for (int i = 0; i < 8; ++i) s[i] += v[i];
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) red[rl][ct * 8 + i] = s[i];
  __syncthreads();
  const int64_t c0 = (int64_t)blockIdx.x * 256;
  const int j = threadIdx.x;  // one output column per thread
  if (c0 + j < N) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) t += red[i][j];
    ws[blockIdx.y * N + c0 + j] = t;
  }
}

// GELU / SiLU backward fused with the bias gradient (SigLIP fc1: siglip.py:183-192 autograd): dpre = dh * act'(pre)
// (act_bwd8's arithmetic; dpre may alias dh), and the column sums of the bf16 dpre over this workgroup's rpc rows
// -> ws[chunk][N] (fp32, fixed order), folded by reduce_parts.  Thread = 8 columns, 8 rows' loads in flight.
__global__ void __launch_bounds__(256) act_bwd_colsum8_kernel(const bf16_t* dh, int64_t lddh, const bf16_t* pre,
                                                              int64_t ldpre, bf16_t* dpre, int64_t M, int64_t N,
                                                              int64_t rpc, int act, float* ws) {
  const int64_t c = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 8;
  if (c >= N) return;
  const int64_t r0 = (int64_t)blockIdx.y * rpc, r1 = min(M, r0 + rpc);
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  auto row = [&](const u32x4& xp, const u32x4& xd, int64_t r) {
    float x[8], d[8];
    unpack8(xp, x);
    unpack8(xd, d);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      x[e] = bf2f(f2bf(d[e] * (act == PZ_EPI_GELU ? gelu_tanh_grad(x[e]) : silu_grad(x[e]))));
      s[e] += x[e];
    }
    store8(dpre + r * ldpre + c, x);
  };
  int64_t r = r0;
  for (; r + 7 < r1; r += 8) {  // 8 rows' loads in flight
    u32x4 xp[8], xd[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      xp[u] = *reinterpret_cast<const u32x4*>(pre + (r + u) * ldpre + c);
      xd[u] = *reinterpret_cast<const u32x4*>(dh + (r + u) * lddh + c);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) row(xp[u], xd[u], r + u);
  }
  for (; r < r1; ++r)
    row(*reinterpret_cast<const u32x4*>(pre + r * ldpre + c), *reinterpret_cast<const u32x4*>(dh + r * lddh + c), r);
  float* w = ws + (int64_t)blockIdx.y * N + c;
  *reinterpret_cast<f32x4*>(w) = f32x4{s[0], s[1], s[2], s[3]};
  *reinterpret_cast<f32x4*>(w + 4) = f32x4{s[4], s[5], s[6], s[7]};
}

__global__ void batch_sum_kernel(const bf16_t* __restrict__ X, int64_t B, int64_t stride, int64_t n,
                                 bf16_t* out, int beta) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float s = 0.f;
  for (int64_t b = 0; b < B; ++b) s += bf2f(X[b * stride + i]);
  if (beta) s += bf2f(out[i]);
  out[i] = f2bf(s);
}

}  // namespace

extern "C" int64_t pz_norm_rows_per_part(void) { return ROWS_PER_PART; }

// Backward, one ROW per workgroup step (default): thread t owns the 8 columns 8t .. 8t + 7 of every
// row (D <= 2048), so the dw / db accumulators are 8 + 8 registers per thread, the partial row is
// written without an LDS reduction, and occupancy is high; the next row's x / dy / residual-gradient
// loads are issued before the current row's reductions (two rows in flight per workgroup); the two
// row sums go through a double-buffered LDS slot (one barrier per row).  The wave-per-row kernels
// above hold MAXC x 8 accumulators per thread (2 waves / SIMD at D >= 1152): PZ_NORM_BWD=wave (A/B).
// PF = rows loaded ahead (2: three rows of x / dy / residual gradient in flight per workgroup, so a partly filled
// last round of workgroups is not latency-bound; PF = 1 measured 138 vs 131.5 us at 65536 x 1152,
// profiles/r05/norm_bench.log).
template <bool LN, int PF>
__global__ void __launch_bounds__(256) norm_bwd_row_kernel(
    const bf16_t* __restrict__ dy, int64_t lddy, const bf16_t* __restrict__ x, int64_t ldx,
    const bf16_t* __restrict__ w, const float* __restrict__ mean, const float* __restrict__ rstd,
    const bf16_t* dres, bf16_t* dx, int64_t lddx, float* dw_part, float* db_part, int64_t R, int D,
    float* dx_part) {
  __shared__ float red[2][2][4];  // [row parity][sum][wave]
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const bool act = t < D / 8;
  float wv[8];
  if (act) load8(w + t * 8, wv);
  else {
#pragma unroll
    for (int i = 0; i < 8; ++i) wv[i] = 0.f;
  }
  float dwa[8], dba[8], dxa[8];  // dxa: column sums of the bf16 dx (dx_part: the bias gradient of the Linear
                                 // whose output gradient dx is -- SigLIP fc2 / out_proj, colsum fused)
#pragma unroll
  for (int i = 0; i < 8; ++i) dwa[i] = dba[i] = dxa[i] = 0.f;
  const int64_t r0 = (int64_t)blockIdx.x * ROWS_PER_PART;
  const int nrows = (int)(R - r0 < ROWS_PER_PART ? R - r0 : ROWS_PER_PART);
  const u32x4 z4 = {0u, 0u, 0u, 0u};
  u32x4 xr = z4, dyr = z4, drr = z4, x1 = z4, dy1 = z4, dr1 = z4;
  if (act) {
    xr = *reinterpret_cast<const u32x4*>(x + r0 * ldx + t * 8);
    dyr = *reinterpret_cast<const u32x4*>(dy + r0 * lddy + t * 8);
    if (dres) drr = *reinterpret_cast<const u32x4*>(dres + r0 * lddx + t * 8);
    if (PF == 2 && nrows > 1) {
      x1 = *reinterpret_cast<const u32x4*>(x + (r0 + 1) * ldx + t * 8);
      dy1 = *reinterpret_cast<const u32x4*>(dy + (r0 + 1) * lddy + t * 8);
      if (dres) dr1 = *reinterpret_cast<const u32x4*>(dres + (r0 + 1) * lddx + t * 8);
    }
  }
  for (int i = 0; i < nrows; ++i) {
    const int64_t row = r0 + i;
    u32x4 xn = z4, dyn = z4, drn = z4;
    if (act && i + PF < nrows) {  // the row PF ahead in flight during this row's reductions
      xn = *reinterpret_cast<const u32x4*>(x + (row + PF) * ldx + t * 8);
      dyn = *reinterpret_cast<const u32x4*>(dy + (row + PF) * lddy + t * 8);
      if (dres) drn = *reinterpret_cast<const u32x4*>(dres + (row + PF) * lddx + t * 8);
    }
    const float r = rstd[row], mu = LN ? mean[row] : 0.f;
    float xv[8], dv[8], g[8];
    unpack8(xr, xv);
    unpack8(dyr, dv);
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      if (LN) {
        xv[e] = (xv[e] - mu) * r;  // x-hat
        g[e] = dv[e] * wv[e];
        s1 += g[e];
        s2 += g[e] * xv[e];
        dwa[e] += dv[e] * xv[e];
        dba[e] += dv[e];
      } else {
        g[e] = dv[e] * (1.f + wv[e]);  // Gemma RMSNorm scales by (1 + w)
        s1 += g[e] * xv[e];
        dwa[e] += dv[e] * xv[e] * r;
      }
    }
    s1 = warp_sum(s1);
    if (LN) s2 = warp_sum(s2);
    if (lane == 0) {
      red[i & 1][0][wave] = s1;
      red[i & 1][1][wave] = s2;
    }
    __syncthreads();
    s1 = red[i & 1][0][0] + red[i & 1][0][1] + red[i & 1][0][2] + red[i & 1][0][3];
    s2 = red[i & 1][1][0] + red[i & 1][1][1] + red[i & 1][1][2] + red[i & 1][1][3];
    if (act) {
      float o[8];
      unpack8(drr, o);
      if (LN) {
        const float a = s1 / (float)D, c = s2 / (float)D;
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] += r * (g[e] - a - xv[e] * c);
      } else {
        const float k = r * r * r * s1 / (float)D;
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] += r * g[e] - k * xv[e];
      }
      store8(dx + row * lddx + t * 8, o);
      if (dx_part) {
#pragma unroll
        for (int e = 0; e < 8; ++e) dxa[e] += bf2f(f2bf(o[e]));
      }
    }
    if (PF == 2) {
      xr = x1, dyr = dy1, drr = dr1;
      x1 = xn, dy1 = dyn, dr1 = drn;
    } else {
      xr = xn, dyr = dyn, drr = drn;
    }
  }
  if (!act) return;
  if (dx_part) {
    float* d = dx_part + (int64_t)blockIdx.x * D + t * 8;
    *reinterpret_cast<f32x4*>(d) = f32x4{dxa[0], dxa[1], dxa[2], dxa[3]};
    *reinterpret_cast<f32x4*>(d + 4) = f32x4{dxa[4], dxa[5], dxa[6], dxa[7]};
  }
  if (dw_part) {
    float* d = dw_part + (int64_t)blockIdx.x * D + t * 8;
    *reinterpret_cast<f32x4*>(d) = f32x4{dwa[0], dwa[1], dwa[2], dwa[3]};
    *reinterpret_cast<f32x4*>(d + 4) = f32x4{dwa[4], dwa[5], dwa[6], dwa[7]};
  }
  if (LN && db_part) {
    float* d = db_part + (int64_t)blockIdx.x * D + t * 8;
    *reinterpret_cast<f32x4*>(d) = f32x4{dba[0], dba[1], dba[2], dba[3]};
    *reinterpret_cast<f32x4*>(d + 4) = f32x4{dba[4], dba[5], dba[6], dba[7]};
  }
}

// ---- fp8 inference (C5): the norm with the per-row e4m3 quantisation of its output in the same pass ----------------
// (the A operand of the following W8A8 GEMM: the output is rounded to bf16 first, so the codes and the scale equal
// pz_rmsnorm_fwd / pz_layernorm_fwd followed by pz_fp8_quant_rows -- one launch and no bf16 row written)
__device__ __forceinline__ unsigned q8enc4(float a, float b, float c, float d) {
  int v = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  v = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, v, true);
  return (unsigned)v;
}

template <int MAXC>
__device__ __forceinline__ void q8_store_row(float (&o)[MAXC][8], int nc, int lane, uint8_t* q, float* qscale) {
  float m = 0.f;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    if (lane + 64 * c < nc)
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        o[c][i] = bf2f(f2bf(o[c][i]));
        m = fmaxf(m, fabsf(o[c][i]));
      }
  }
  m = warp_max(m);
  const float sc = m > 0.f ? __fdiv_rn(m, 448.f) : 1.f;
  const float inv = __fdiv_rn(1.f, sc);
  if (lane == 0) *qscale = sc;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int ch = lane + 64 * c;
    if (ch < nc) {
      float f[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) f[i] = fminf(fmaxf(o[c][i] * inv, -448.f), 448.f);
      *reinterpret_cast<u32x2*>(q + ch * 8) = u32x2{q8enc4(f[0], f[1], f[2], f[3]), q8enc4(f[4], f[5], f[6], f[7])};
    }
  }
}

template <int MAXC>
__global__ void __launch_bounds__(256) rmsnorm_q8_kernel(const bf16_t* __restrict__ x, int64_t ldx,
                                                         const bf16_t* __restrict__ w, uint8_t* q, int64_t ldq,
                                                         float* qscale, int64_t R, int D, float eps) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= R) return;
  const int nc = D / 8;
  // the weight chunks loaded with the row, not after its reduction: one memory round trip
  u32x4 wq[MAXC];
#pragma unroll
  for (int c = 0; c < MAXC; ++c)
    wq[c] = lane + 64 * c < nc ? *reinterpret_cast<const u32x4*>(w + (lane + 64 * c) * 8) : u32x4{0u, 0u, 0u, 0u};
  float v[MAXC][8];
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int ch = lane + 64 * c;
    if (ch < nc) {
      load8(x + row * ldx + ch * 8, v[c]);
#pragma unroll
      for (int i = 0; i < 8; ++i) ss += v[c][i] * v[c][i];
    }
  }
  ss = warp_sum(ss);
  const float r = rsqrtf(ss / (float)D + eps);
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int ch = lane + 64 * c;
    if (ch < nc) {
      float wv[8];
      unpack8(wq[c], wv);
#pragma unroll
      for (int i = 0; i < 8; ++i) v[c][i] = v[c][i] * r * (1.f + wv[i]);
    }
  }
  q8_store_row<MAXC>(v, nc, lane, q + row * ldq, qscale + row);
}

template <int MAXC>
__global__ void __launch_bounds__(256) layernorm_q8_kernel(const bf16_t* __restrict__ x, int64_t ldx,
                                                           const bf16_t* __restrict__ w, const bf16_t* __restrict__ b,
                                                           uint8_t* q, int64_t ldq, float* qscale, int64_t R, int D,
                                                           float eps) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= R) return;
  const int nc = D / 8;
  // the weight and bias chunks loaded with the row, not after its reductions: one memory round trip
  u32x4 wq[MAXC], bq[MAXC];
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const bool ok = lane + 64 * c < nc;
    wq[c] = ok ? *reinterpret_cast<const u32x4*>(w + (lane + 64 * c) * 8) : u32x4{0u, 0u, 0u, 0u};
    bq[c] = ok ? *reinterpret_cast<const u32x4*>(b + (lane + 64 * c) * 8) : u32x4{0u, 0u, 0u, 0u};
  }
  float v[MAXC][8];
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int ch = lane + 64 * c;
    if (ch < nc) {
      load8(x + row * ldx + ch * 8, v[c]);
#pragma unroll
      for (int i = 0; i < 8; ++i) s += v[c][i];
    }
  }
  const float mu = warp_sum(s) / (float)D;
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int ch = lane + 64 * c;
    if (ch < nc)
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float d = v[c][i] - mu;
        ss += d * d;
      }
  }
  const float r = rsqrtf(warp_sum(ss) / (float)D + eps);
#pragma unroll
  for (int c = 0; c < MAXC; ++c) {
    const int ch = lane + 64 * c;
    if (ch < nc) {
      float wv[8], bv[8];
      unpack8(wq[c], wv);
      unpack8(bq[c], bv);
#pragma unroll
      for (int i = 0; i < 8; ++i) v[c][i] = (v[c][i] - mu) * r * wv[i] + bv[i];
    }
  }
  q8_store_row<MAXC>(v, nc, lane, q + row * ldq, qscale + row);
}

static bool norm_bwd_rows() {
  const char* e = getenv("PZ_NORM_BWD");
  return !(e && e[0] == 'w');
}



#define NORM_DISPATCH(KERNEL, GRID, ...)                                                   \
  do {                                                                                    \
    const int nc = (int)(D / 8);                                                          \
    if (nc <= 64) hipLaunchKernelGGL(KERNEL<1>, GRID, dim3(256), 0, st, __VA_ARGS__);     \
    else if (nc <= 128) hipLaunchKernelGGL(KERNEL<2>, GRID, dim3(256), 0, st, __VA_ARGS__); \
    else if (nc <= 192) hipLaunchKernelGGL(KERNEL<3>, GRID, dim3(256), 0, st, __VA_ARGS__); \
    else hipLaunchKernelGGL(KERNEL<4>, GRID, dim3(256), 0, st, __VA_ARGS__);              \
  } while (0)

static int check_norm(const void* x, int64_t ldx, const void* y, int64_t ldy, int64_t D) {
  PZ_CHECK_ARG(D % 8 == 0 && D <= 2048, "norm: D=%lld must be a multiple of 8 and <= 2048", (long long)D);
  PZ_CHECK_ARG(ldx % 8 == 0 && ldy % 8 == 0 && PZ_ALIGNED(x, 16) && PZ_ALIGNED(y, 16),
               "norm: rows must be 16-byte aligned");
  return PZ_OK;
}

extern "C" int pz_rmsnorm_fwd(const void* x, int64_t ldx, const void* w, void* y, int64_t ldy, float* rstd,
                              int64_t R, int64_t D, float eps, void* stream) {
  int e = check_norm(x, ldx, y, ldy, D);
  if (e) return e;
  if (R == 0) return PZ_OK;
  hipStream_t st = (hipStream_t)stream;
  dim3 grid((unsigned)((R + 3) / 4));
  NORM_DISPATCH(rmsnorm_fwd_kernel, grid, (const bf16_t*)x, ldx, (const bf16_t*)w, (bf16_t*)y, ldy, rstd, R,
                (int)D, eps);
  PZ_CHECK_LAUNCH();
  return PZ_OK;
}

extern "C" int pz_rmsnorm_bwd(const void* dy, int64_t lddy, const void* x, int64_t ldx, const void* w,
                              const float* rstd, const void* dres, void* dx, int64_t lddx, float* dw_part,
                              int64_t R, int64_t D, void* stream) {
  int e = check_norm(x, ldx, dx, lddx, D);
  if (e) return e;
  PZ_CHECK_ARG(lddy % 8 == 0, "rmsnorm_bwd: lddy");
  if (R == 0) return PZ_OK;
  hipStream_t st = (hipStream_t)stream;
  dim3 grid((unsigned)((R + ROWS_PER_PART - 1) / ROWS_PER_PART));
  if (norm_bwd_rows() && PZ_ALIGNED(dy, 16) && (!dres || PZ_ALIGNED(dres, 16)) && PZ_ALIGNED(dw_part, 16))
    hipLaunchKernelGGL((norm_bwd_row_kernel<false, 2>), grid,
                       dim3(256), 0, st, (const bf16_t*)dy, lddy, (const bf16_t*)x, ldx, (const bf16_t*)w, nullptr,
                       rstd, (const bf16_t*)dres, (bf16_t*)dx, lddx, dw_part, nullptr, R, (int)D, nullptr);
  else
    NORM_DISPATCH(rmsnorm_bwd_kernel, grid, (const bf16_t*)dy, lddy, (const bf16_t*)x, ldx, (const bf16_t*)w,
                  rstd, (const bf16_t*)dres, (bf16_t*)dx, lddx, dw_part, R, (int)D);
  PZ_CHECK_LAUNCH();
  return PZ_OK;
}

extern "C" int pz_layernorm_fwd(const void* x, int64_t ldx, const void* w, const void* b, void* y, int64_t ldy,
                                float* mean, float* rstd, int64_t R, int64_t D, float eps, void* stream) {
  int e = check_norm(x, ldx, y, ldy, D);
  if (e) return e;
  if (R == 0) return PZ_OK;
  hipStream_t st = (hipStream_t)stream;
  dim3 grid((unsigned)((R + 3) / 4));
  NORM_DISPATCH(layernorm_fwd_kernel, grid, (const bf16_t*)x, ldx, (const bf16_t*)w, (const bf16_t*)b,
                (bf16_t*)y, ldy, mean, rstd, R, (int)D, eps);
  PZ_CHECK_LAUNCH();
  return PZ_OK;
}

extern "C" int pz_layernorm_bwd(const void* dy, int64_t lddy, const void* x, int64_t ldx, const void* w,
                                const float* mean, const float* rstd, const void* dres, void* dx, int64_t lddx,
                                float* dw_part, float* db_part, int64_t R, int64_t D, float* dx_part, void* stream) {
  int e = check_norm(x, ldx, dx, lddx, D);
  if (e) return e;
  PZ_CHECK_ARG(lddy % 8 == 0, "layernorm_bwd: lddy");
  if (R == 0) return PZ_OK;
  hipStream_t st = (hipStream_t)stream;
  dim3 grid((unsigned)((R + ROWS_PER_PART - 1) / ROWS_PER_PART));
  if (norm_bwd_rows() && PZ_ALIGNED(dy, 16) && (!dres || PZ_ALIGNED(dres, 16)) && PZ_ALIGNED(dw_part, 16) &&
      PZ_ALIGNED(db_part, 16) && (!dx_part || PZ_ALIGNED(dx_part, 16)))
    hipLaunchKernelGGL((norm_bwd_row_kernel<true, 2>), grid,
                       dim3(256), 0, st, (const bf16_t*)dy, lddy, (const bf16_t*)x, ldx, (const bf16_t*)w, mean, rstd,
                       (const bf16_t*)dres, (bf16_t*)dx, lddx, dw_part, db_part, R, (int)D, dx_part);
  else if (dx_part)
    PZ_CHECK_ARG(false, "layernorm_bwd: dx_part (fused column sums of dx) needs the row kernel (16-byte aligned "
                        "dy / dres / partials / dx_part, PZ_NORM_BWD != wave)");
  else
    NORM_DISPATCH(layernorm_bwd_kernel, grid, (const bf16_t*)dy, lddy, (const bf16_t*)x, ldx, (const bf16_t*)w,
                  mean, rstd, (const bf16_t*)dres, (bf16_t*)dx, lddx, dw_part, db_part, R, (int)D);
  PZ_CHECK_LAUNCH();
  return PZ_OK;
}

static void launch_reduce_parts(const float* part, int64_t P, int64_t D, bf16_t* out, int beta, hipStream_t st) {
  if (D % 4 == 0 && PZ_ALIGNED(part, 16) && PZ_ALIGNED(out, 8)) {
    // column-threads per block: enough blocks to cover the chip when D is small, wide rows when D is large
    if (D >= 256 * 256)
      hipLaunchKernelGGL(reduce_parts4_kernel<64>, dim3((unsigned)((D + 255) / 256)), dim3(256), 0, st, part, P, D,
                         out, beta);
    else if (D >= 256 * 64)
      hipLaunchKernelGGL(reduce_parts4_kernel<16>, dim3((unsigned)((D + 63) / 64)), dim3(256), 0, st, part, P, D,
                         out, beta);
    else
      hipLaunchKernelGGL(reduce_parts4_kernel<4>, dim3((unsigned)((D + 15) / 16)), dim3(256), 0, st, part, P, D,
                         out, beta);
  } else {
    hipLaunchKernelGGL(reduce_parts_kernel, dim3((unsigned)((D + 255) / 256)), dim3(256), 0, st, part, P, D, out,
                       beta);
  }
}

extern "C" int pz_reduce_parts(const float* part, int64_t P, int64_t D, void* out, int32_t beta, void* stream) {
  PZ_CHECK_ARG(part && out && P > 0 && D > 0, "reduce_parts: bad args");
  launch_reduce_parts(part, P, D, (bf16_t*)out, (int)beta, (hipStream_t)stream);
  PZ_CHECK_LAUNCH();
  return PZ_OK;
}

extern "C" int pz_reduce_parts_multi(const pz_reduce_seg* segs, int32_t nseg, void* stream) {
  PZ_CHECK_ARG(segs && nseg > 0, "reduce_parts_multi: bad args");
  RedSegs a;
  memset(&a, 0, sizeof(a));
  hipStream_t st = (hipStream_t)stream;
  int blocks = 0;
  for (int32_t i = 0; i < nseg; ++i) {
    const pz_reduce_seg& g = segs[i];
    PZ_CHECK_ARG(g.part && g.out && g.P > 0 && g.D > 0 && g.D % 4 == 0 && PZ_ALIGNED(g.part, 16) && PZ_ALIGNED(g.out, 8),
                 "reduce_parts_multi: segment %d needs D %% 4 == 0, 16-byte aligned partials, 8-byte aligned out", i);
    if (a.n == RED_MAXSEG) {  // flush a full table
      a.blk0[a.n] = blocks;
      hipLaunchKernelGGL(reduce_parts4_multi_kernel, dim3((unsigned)blocks), dim3(256), 0, st, a);
      PZ_CHECK_LAUNCH();
      memset(&a, 0, sizeof(a));
      blocks = 0;
    }
    const int k = a.n++;
    a.part[k] = g.part;
    a.out[k] = (bf16_t*)g.out;
    a.P[k] = g.P;
    a.D[k] = g.D;
    a.beta[k] = g.beta;
    a.blk0[k] = blocks;
    blocks += (int)((g.D + 15) / 16);
  }
  a.blk0[a.n] = blocks;
  hipLaunchKernelGGL(reduce_parts4_multi_kernel, dim3((unsigned)blocks), dim3(256), 0, st, a);
  PZ_CHECK_LAUNCH();
  return PZ_OK;
}

extern "C" int pz_colsum(const void* X, int64_t ld, int64_t M, int64_t N, void* out, int32_t beta, float* ws,
                         void* stream) {
  PZ_CHECK_ARG(X && out && ws && M > 0 && N > 0, "colsum: bad args");
  hipStream_t st = (hipStream_t)stream;
  int64_t chunks = M < 64 ? M : 64;  // ws holds 64 partial rows (pz_abi.h)
  if (N % 8 == 0 && ld % 8 == 0 && PZ_ALIGNED(X, 16)) {
    const int64_t rpc = (M + chunks - 1) / chunks;
    chunks = (M + rpc - 1) / rpc;
    dim3 grid((unsigned)((N + 255) / 256), (unsigned)chunks);
    hipLaunchKernelGGL(colsum8_pass1, grid, dim3(256), 0, st, (const bf16_t*)X, ld, M, N, rpc, ws);
  } else {
    const int64_t rpc = (M + chunks - 1) / chunks;
    dim3 grid((unsigned)((N / 2 + 1 + 255) / 256), (unsigned)chunks);
    hipLaunchKernelGGL(colsum_pass1, grid, dim3(256), 0, st, (const bf16_t*)X, ld, M, N, rpc, ws);
  }
  PZ_CHECK_LAUNCH();
  launch_reduce_parts(ws, chunks, N, (bf16_t*)out, (int)beta, st);
  PZ_CHECK_LAUNCH();
  return PZ_OK;
}

extern "C" int pz_act_bwd_colsum(const void* dh, int64_t lddh, const void* pre, int64_t ldpre, void* dpre, int64_t M,
                                 int64_t N, int32_t act, float* ws, int64_t ws_rows, void* dbias, int32_t beta,
                                 void* stream) {
  PZ_CHECK_ARG(dh && pre && dpre && ws && dbias && M > 0 && N > 0 && ws_rows > 0 &&
                   (act == PZ_EPI_GELU || act == PZ_EPI_SILU),
               "act_bwd_colsum: bad args");
  PZ_CHECK_ARG(N % 8 == 0 && lddh % 8 == 0 && ldpre % 8 == 0 && PZ_ALIGNED(dh, 16) && PZ_ALIGNED(pre, 16) &&
                   PZ_ALIGNED(dpre, 16) && PZ_ALIGNED(ws, 16),
               "act_bwd_colsum: N, strides %% 8 and 16-byte alignment");
  hipStream_t st = (hipStream_t)stream;
  // row chunks: up to ws_rows partial rows, >= 16 rows each (3072 workgroups for the SigLIP fc1 gradient at 1024)
  int64_t chunks = ws_rows < (M + 15) / 16 ? ws_rows : (M + 15) / 16;
  const int64_t rpc = (M + chunks - 1) / chunks;
  chunks = (M + rpc - 1) / rpc;
  hipLaunchKernelGGL(act_bwd_colsum8_kernel, dim3((unsigned)((N / 8 + 255) / 256), (unsigned)chunks), dim3(256), 0, st,
                     (const bf16_t*)dh, lddh, (const bf16_t*)pre, ldpre, (bf16_t*)dpre, M, N, rpc, (int)act, ws);
  PZ_CHECK_LAUNCH();
  launch_reduce_parts(ws, chunks, N, (bf16_t*)dbias, (int)beta, st);
  PZ_CHECK_LAUNCH();
  return PZ_OK;
}

extern "C" int pz_batch_sum(const void* X, int64_t B, int64_t stride, int64_t n, void* out, int32_t beta,
                            void* stream) {
  PZ_CHECK_ARG(X && out && B > 0 && n > 0, "batch_sum: bad args");
  hipLaunchKernelGGL(batch_sum_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     (const bf16_t*)X, B, stride, n, (bf16_t*)out, (int)beta);
  PZ_CHECK_LAUNCH();
  return PZ_OK;
}

extern "C" int pz_rmsnorm_fwd_f8(const void* x, int64_t ldx, const void* w, void* q, int64_t ldq, float* qscale,
                                 int64_t R, int64_t D, float eps, void* stream) {
  PZ_CHECK_ARG(x && w && q && qscale && D % 8 == 0 && D <= 2048 && ldx % 8 == 0 && ldq % 8 == 0 &&
                   PZ_ALIGNED(x, 16) && PZ_ALIGNED(q, 8),
               "rmsnorm_fwd_f8: bad args (D %% 8 == 0, D <= 2048, aligned rows)");
  if (R == 0) return PZ_OK;
  hipStream_t st = (hipStream_t)stream;
  dim3 grid((unsigned)((R + 3) / 4));
  NORM_DISPATCH(rmsnorm_q8_kernel, grid, (const bf16_t*)x, ldx, (const bf16_t*)w, (uint8_t*)q, ldq, qscale, R, (int)D,
                eps);
  PZ_CHECK_LAUNCH();
  return PZ_OK;
}

extern "C" int pz_layernorm_fwd_f8(const void* x, int64_t ldx, const void* w, const void* b, void* q, int64_t ldq,
                                   float* qscale, int64_t R, int64_t D, float eps, void* stream) {
  PZ_CHECK_ARG(x && w && b && q && qscale && D % 8 == 0 && D <= 2048 && ldx % 8 == 0 && ldq % 8 == 0 &&
                   PZ_ALIGNED(x, 16) && PZ_ALIGNED(q, 8),
               "layernorm_fwd_f8: bad args (D %% 8 == 0, D <= 2048, aligned rows)");
  if (R == 0) return PZ_OK;
  hipStream_t st = (hipStream_t)stream;
  dim3 grid((unsigned)((R + 3) / 4));
  NORM_DISPATCH(layernorm_q8_kernel, grid, (const bf16_t*)x, ldx, (const bf16_t*)w, (const bf16_t*)b, (uint8_t*)q, ldq,
                qscale, R, (int)D, eps);
  PZ_CHECK_LAUNCH();
  return PZ_OK;
}
