// Attention pieces around the MFMA GEMMs (pz_gemm.hip computes S = QK^T and
// O = PV batched per sample, MQA heads stacked as rows -> no repeat_kv copy):
//   * RoPE table + fused QKV split/rotate into the joint (vlm|proprio|action)
//     token buffers (joint_model.py:170-257, utils.py:4-16, modules.py:24-67)
//   * softmax with Gemma tanh soft-cap and the Pi0 block mask generated
//     arithmetically from per-sample prefix counts (joint_model.py:261-275,
//     pizero.py:271-306), fully-masked rows -> uniform (finfo.min semantics)
//   * the matching backward.
#include "pz_common.h"

namespace {

__global__ void rope_table_kernel(float* cs, int64_t max_pos, int hd, float theta) {
  const int half = hd / 2;
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (max_pos + 1) * half) return;
  const int64_t pos = idx / half;
  const int i = (int)(idx % half);
  const float expo = (float)(2 * i) / (float)hd;
  const float inv = 1.0f / powf(theta, expo);
  const float f = (float)pos * inv;
  cs[2 * idx] = cosf(f);
  cs[2 * idx + 1] = sinf(f);
}

// grid: (T, B); block 256. qkv row = [q (nh*hd) | k (nkv*hd) | v (nkv*hd)]
__global__ void qkv_rope_split_kernel(const bf16_t* __restrict__ qkv, const int64_t* __restrict__ pos,
                                      const float* __restrict__ cs, bf16_t* q_out, bf16_t* k_out,
                                      bf16_t* v_out, int64_t T, int nh, int nkv, int hd, int64_t Lq,
                                      int64_t qoff, int64_t Lk, int64_t koff) {
  const int64_t t = blockIdx.x, b = blockIdx.y;
  const int64_t tok = b * T + t;
  const int half = hd / 2;
  const int width = (nh + 2 * nkv) * hd;
  const bf16_t* src = qkv + tok * width;
  const float* c = cs + pos[tok] * hd;  // [half][2]
  if (q_out) {
    bf16_t* dq = q_out + (b * Lq + qoff + t) * (int64_t)(nh * hd);
    for (int e = threadIdx.x; e < nh * half; e += blockDim.x) {
      const int h = e / half, i = e % half;
      const float x1 = bf2f(src[h * hd + i]), x2 = bf2f(src[h * hd + i + half]);
      const float co = c[2 * i], si = c[2 * i + 1];
      float o1, o2;
      rope_pair(x1, x2, co, si, o1, o2);
      dq[h * hd + i] = f2bf(o1);
      dq[h * hd + i + half] = f2bf(o2);
    }
  }
  bf16_t* dk = k_out + (b * Lk + koff + t) * (int64_t)(nkv * hd);
  bf16_t* dv = v_out + (b * Lk + koff + t) * (int64_t)(nkv * hd);
  const bf16_t* sk = src + nh * hd;
  const bf16_t* sv = src + (nh + nkv) * hd;
  for (int e = threadIdx.x; e < nkv * half; e += blockDim.x) {
    const int h = e / half, i = e % half;
    const float x1 = bf2f(sk[h * hd + i]), x2 = bf2f(sk[h * hd + i + half]);
    const float co = c[2 * i], si = c[2 * i + 1];
    float o1, o2;
    rope_pair(x1, x2, co, si, o1, o2);
    dk[h * hd + i] = f2bf(o1);
    dk[h * hd + i + half] = f2bf(o2);
  }
  for (int e = threadIdx.x; e < nkv * hd; e += blockDim.x) dv[e] = sv[e];
}

__global__ void qkv_rope_split_bwd_kernel(const bf16_t* __restrict__ dq, const bf16_t* __restrict__ dk,
                                          const bf16_t* __restrict__ dv, const int64_t* __restrict__ pos,
                                          const float* __restrict__ cs, bf16_t* dqkv, int64_t T, int nh,
                                          int nkv, int hd, int64_t Lq, int64_t qoff, int64_t Lk,
                                          int64_t koff) {
  const int64_t t = blockIdx.x, b = blockIdx.y;
  const int64_t tok = b * T + t;
  const int half = hd / 2;
  const int width = (nh + 2 * nkv) * hd;
  bf16_t* dst = dqkv + tok * width;
  const float* c = cs + pos[tok] * hd;
  const bf16_t* sq = dq ? dq + (b * Lq + qoff + t) * (int64_t)(nh * hd) : nullptr;
  for (int e = threadIdx.x; e < nh * half; e += blockDim.x) {
    const int h = e / half, i = e % half;
    float o1 = 0.f, o2 = 0.f;
    if (sq) {
      const float y1 = bf2f(sq[h * hd + i]), y2 = bf2f(sq[h * hd + i + half]);
      const float co = c[2 * i], si = c[2 * i + 1];
      o1 = y1 * co + y2 * si;
      o2 = y2 * co - y1 * si;
    }
    dst[h * hd + i] = f2bf(o1);
    dst[h * hd + i + half] = f2bf(o2);
  }
  const bf16_t* sk = dk + (b * Lk + koff + t) * (int64_t)(nkv * hd);
  const bf16_t* sv = dv + (b * Lk + koff + t) * (int64_t)(nkv * hd);
  bf16_t* ok = dst + nh * hd;
  bf16_t* ov = dst + (nh + nkv) * hd;
  for (int e = threadIdx.x; e < nkv * half; e += blockDim.x) {
    const int h = e / half, i = e % half;
    const float y1 = bf2f(sk[h * hd + i]), y2 = bf2f(sk[h * hd + i + half]);
    const float co = c[2 * i], si = c[2 * i + 1];
    ok[h * hd + i] = f2bf(y1 * co + y2 * si);
    ok[h * hd + i + half] = f2bf(y2 * co - y1 * si);
  }
  for (int e = threadIdx.x; e < nkv * hd; e += blockDim.x) ov[e] = sv[e];
}

__device__ __forceinline__ bool block_allowed(int64_t i, int64_t j, int64_t cnt, int64_t P, int64_t C) {
  if (i < P) return i < cnt && j < cnt;
  if (i < P + C) return j < cnt || (j >= P && j < P + C);
  return j < cnt || j >= P;
}

// one wave per row, MAXE elements per lane
template <int MAXE>
__global__ void __launch_bounds__(256) softmax_kernel(pz_softmax_args a) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= a.R) return;
  const float* s = a.S + row * a.lds;
  int64_t b = 0, qi = 0;
  if (a.mask_mode != 0) {
    b = row / a.rows_per_batch;
    qi = a.qoff + (row % a.rows_per_batch) / a.heads;
  }
  const int64_t cnt = a.mask_mode == 1 ? (int64_t)a.cnt[b] : 0;
  const float* mrow = a.mask_mode == 2 ? a.mask + b * a.mask_bstride + (qi - a.qoff) * a.ldm : nullptr;
  float x[MAXE];
  bool ok[MAXE];
  float mx = -INFINITY;
#pragma unroll
  for (int e = 0; e < MAXE; ++e) {
    const int64_t j = lane + 64 * e;
    ok[e] = false;
    x[e] = 0.f;
    if (j < a.N) {
      float v = s[j] * a.scale;
      if (a.cap > 0.f) v = a.cap * tanhf(v / a.cap);
      bool al = true;
      if (a.mask_mode == 1) al = block_allowed(qi, j, cnt, a.prefix, a.cond);
      else if (a.mask_mode == 2) {  // additive (joint_model.py:271): finfo.min absorbs v, like the reference
        v += mrow[j];
        al = v > -INFINITY;
      }
      x[e] = v;
      ok[e] = al;
      if (al) mx = fmaxf(mx, v);
    }
  }
  mx = warp_max(mx);
  bf16_t* prow = (bf16_t*)a.P + row * a.ldp;
  bf16_t* trow = a.tcap ? (bf16_t*)a.tcap + row * a.ldp : nullptr;
  if (mx == -INFINITY) {  // fully masked row: finfo.min + s absorbs s -> uniform (pizero.py:291)
    const float u = 1.f / (float)a.N;
    for (int64_t j = lane; j < a.ldp; j += 64) {
      prow[j] = f2bf(j < a.N ? u : 0.f);
      if (trow) trow[j] = 0;
    }
    return;
  }
  float sum = 0.f;
#pragma unroll
  for (int e = 0; e < MAXE; ++e) {
    const float p = ok[e] ? __expf(x[e] - mx) : 0.f;
    x[e] = p;
    sum += p;
  }
  const float inv = 1.f / warp_sum(sum);
#pragma unroll
  for (int e = 0; e < MAXE; ++e) {
    const int64_t j = lane + 64 * e;
    if (j < a.N) {
      prow[j] = f2bf(x[e] * inv);
      if (trow) {
        float v = s[j] * a.scale;
        trow[j] = f2bf(a.cap > 0.f ? tanhf(v / a.cap) : 0.f);
      }
    }
  }
  for (int64_t j = a.N + lane; j < a.ldp; j += 64) {
    prow[j] = 0;
    if (trow) trow[j] = 0;
  }
}

// Vectorised variants (rows 16-B aligned, ld % 4 == 0): one wave per row, each lane owns groups of 4
// consecutive columns (float4 logits, 8-B bf16 stores), 32-bit index math, fast tanh for the cap.
__device__ __forceinline__ u32x2 pack4bf(const float (&v)[4]) { return u32x2{pack2bf(v[0], v[1]), pack2bf(v[2], v[3])}; }

template <int MAXV>
__global__ void __launch_bounds__(256) softmax4_kernel(pz_softmax_args a) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= a.R) return;
  const float* s = a.S + row * a.lds;
  int b = 0, qi = 0;
  if (a.mask_mode != 0) {
    const int rr = (int)row, rpb = (int)a.rows_per_batch;
    b = rr / rpb;
    qi = (int)a.qoff + (rr - b * rpb) / (int)a.heads;
  }
  const int cnt = a.mask_mode == 1 ? a.cnt[b] : 0;
  const int P = (int)a.prefix, Cc = (int)a.cond, N = (int)a.N;
  const float* mrow = a.mask_mode == 2 ? a.mask + b * a.mask_bstride + (qi - a.qoff) * a.ldm : nullptr;
  const float inv_cap = a.cap > 0.f ? 1.f / a.cap : 0.f;
  float x[MAXV][4], th[MAXV][4];
  bool ok[MAXV][4];
  float mx = -INFINITY;
#pragma unroll
  for (int e = 0; e < MAXV; ++e) {
    const int j0 = 4 * (lane + 64 * e);
    f32x4 sv = {0.f, 0.f, 0.f, 0.f};
    if (j0 < N) sv = *reinterpret_cast<const f32x4*>(s + j0);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int j = j0 + i;
      float v = j < N ? sv[i] * a.scale : 0.f;  // padded columns may hold anything
      th[e][i] = 0.f;
      if (a.cap > 0.f && j < N) {
        th[e][i] = tanh_fast(v * inv_cap);
        v = a.cap * th[e][i];
      }
      bool al = j < N;
      if (al && a.mask_mode == 1) al = block_allowed(qi, j, cnt, P, Cc);
      else if (al && a.mask_mode == 2) {  // additive mask
        v += mrow[j];
        al = v > -INFINITY;
      }
      x[e][i] = v;
      ok[e][i] = al;
      if (al) mx = fmaxf(mx, v);
    }
  }
  mx = warp_max(mx);
  bf16_t* prow = (bf16_t*)a.P + row * a.ldp;
  bf16_t* trow = a.tcap ? (bf16_t*)a.tcap + row * a.ldp : nullptr;
  const int ldp = (int)a.ldp;
  if (mx == -INFINITY) {  // fully masked row: finfo.min + s absorbs s -> uniform (pizero.py:291)
    const float u = 1.f / (float)N;
    for (int j0 = 4 * lane; j0 < ldp; j0 += 256) {
      float v[4] = {j0 < N ? u : 0.f, j0 + 1 < N ? u : 0.f, j0 + 2 < N ? u : 0.f, j0 + 3 < N ? u : 0.f};
      *reinterpret_cast<u32x2*>(prow + j0) = pack4bf(v);
      if (trow) *reinterpret_cast<u32x2*>(trow + j0) = u32x2{0u, 0u};
    }
    return;
  }
  float sum = 0.f;
#pragma unroll
  for (int e = 0; e < MAXV; ++e)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float pv = ok[e][i] ? __expf(x[e][i] - mx) : 0.f;
      x[e][i] = pv;
      sum += pv;
    }
  const float inv = 1.f / warp_sum(sum);
#pragma unroll
  for (int e = 0; e < MAXV; ++e) {
    const int j0 = 4 * (lane + 64 * e);
    if (j0 < ldp) {  // columns N..ldp-1 come out 0 (x = 0, th = 0 there)
      float v[4] = {x[e][0] * inv, x[e][1] * inv, x[e][2] * inv, x[e][3] * inv};
      *reinterpret_cast<u32x2*>(prow + j0) = pack4bf(v);
      if (trow) *reinterpret_cast<u32x2*>(trow + j0) = pack4bf(th[e]);
    }
  }
}

template <int MAXV>
__global__ void __launch_bounds__(256) softmax_bwd4_kernel(const bf16_t* __restrict__ Pm, const float* __restrict__ dP,
                                                           int64_t lddp, const bf16_t* __restrict__ tcap, bf16_t* dS,
                                                           int64_t ldp, int64_t R, int N, float scale, float cap) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= R) return;
  const bf16_t* prow = Pm + row * ldp;
  const float* drow = dP + row * lddp;
  float p[MAXV][4], d[MAXV][4];
  float dot = 0.f;
#pragma unroll
  for (int e = 0; e < MAXV; ++e) {
    const int j0 = 4 * (lane + 64 * e);
    u32x2 pw = {0u, 0u};
    f32x4 dv = {0.f, 0.f, 0.f, 0.f};
    if (j0 < N) {
      pw = *reinterpret_cast<const u32x2*>(prow + j0);
      dv = *reinterpret_cast<const f32x4*>(drow + j0);
    }
    p[e][0] = __uint_as_float(pw[0] << 16);
    p[e][1] = __uint_as_float(pw[0] & 0xffff0000u);
    p[e][2] = __uint_as_float(pw[1] << 16);
    p[e][3] = __uint_as_float(pw[1] & 0xffff0000u);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      d[e][i] = j0 + i < N ? dv[i] : 0.f;
      dot += p[e][i] * d[e][i];
    }
  }
  dot = warp_sum(dot);
  bf16_t* orow = dS + row * ldp;
#pragma unroll
  for (int e = 0; e < MAXV; ++e) {
    const int j0 = 4 * (lane + 64 * e);
    if (j0 < (int)ldp) {
      float g[4];
      u32x2 tw = {0u, 0u};
      if (cap > 0.f && j0 < N) tw = *reinterpret_cast<const u32x2*>(tcap + row * ldp + j0);
      const float t[4] = {__uint_as_float(tw[0] << 16), __uint_as_float(tw[0] & 0xffff0000u),
                          __uint_as_float(tw[1] << 16), __uint_as_float(tw[1] & 0xffff0000u)};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        g[i] = j0 + i < N ? p[e][i] * (d[e][i] - dot) * scale : 0.f;
        if (cap > 0.f) g[i] *= (1.f - t[i] * t[i]);
      }
      *reinterpret_cast<u32x2*>(orow + j0) = pack4bf(g);
    }
  }
}

template <int MAXE>
__global__ void __launch_bounds__(256) softmax_bwd_kernel(const bf16_t* __restrict__ P,
                                                          const float* __restrict__ dP, int64_t lddp,
                                                          const bf16_t* __restrict__ tcap, bf16_t* dS,
                                                          int64_t ldp, int64_t R, int64_t N, float scale,
                                                          float cap) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= R) return;
  const bf16_t* prow = P + row * ldp;
  const float* drow = dP + row * lddp;
  float p[MAXE], d[MAXE];
  float dot = 0.f;
#pragma unroll
  for (int e = 0; e < MAXE; ++e) {
    const int64_t j = lane + 64 * e;
    p[e] = 0.f;
    d[e] = 0.f;
    if (j < N) {
      p[e] = bf2f(prow[j]);
      d[e] = drow[j];
      dot += p[e] * d[e];
    }
  }
  dot = warp_sum(dot);
  bf16_t* orow = dS + row * ldp;
#pragma unroll
  for (int e = 0; e < MAXE; ++e) {
    const int64_t j = lane + 64 * e;
    if (j < N) {
      float g = p[e] * (d[e] - dot) * scale;
      if (cap > 0.f) {
        const float t = bf2f(tcap[row * ldp + j]);
        g *= (1.f - t * t);
      }
      orow[j] = f2bf(g);
    }
  }
  for (int64_t j = N + lane; j < ldp; j += 64) orow[j] = 0;
}

}  // namespace

extern "C" int pz_rope_table(float* cs, int64_t max_pos, int64_t head_dim, float theta, void* stream) {
  PZ_CHECK_ARG(cs && max_pos >= 0 && head_dim % 2 == 0, "rope_table: bad args");
  const int64_t n = (max_pos + 1) * (head_dim / 2);
  hipLaunchKernelGGL(rope_table_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, cs,
                     max_pos, (int)head_dim, theta);
  PZ_CHECK_LAUNCH();
  return PZ_OK;
}

extern "C" int pz_qkv_rope_split(const void* qkv, const int64_t* pos, const float* cs, void* q_out, void* k_out,
                                 void* v_out, int64_t B, int64_t T, int64_t nh, int64_t nkv, int64_t hd,
                                 int64_t Lq, int64_t qoff, int64_t Lk, int64_t koff, void* stream) {
  PZ_CHECK_ARG(qkv && pos && cs && k_out && v_out && B > 0 && T > 0 && hd % 2 == 0, "qkv_rope_split: bad args");
  PZ_CHECK_ARG(koff + T <= Lk && (!q_out || qoff + T <= Lq), "qkv_rope_split: token range");
  hipLaunchKernelGGL(qkv_rope_split_kernel, dim3((unsigned)T, (unsigned)B), dim3(256), 0, (hipStream_t)stream,
                     (const bf16_t*)qkv, pos, cs, (bf16_t*)q_out, (bf16_t*)k_out, (bf16_t*)v_out, T, (int)nh,
                     (int)nkv, (int)hd, Lq, qoff, Lk, koff);
  PZ_CHECK_LAUNCH();
  return PZ_OK;
}

extern "C" int pz_qkv_rope_split_bwd(const void* dq, const void* dk, const void* dv, const int64_t* pos,
                                     const float* cs, void* dqkv, int64_t B, int64_t T, int64_t nh, int64_t nkv,
                                     int64_t hd, int64_t Lq, int64_t qoff, int64_t Lk, int64_t koff, void* stream) {
  PZ_CHECK_ARG(dk && dv && pos && cs && dqkv && B > 0 && T > 0, "qkv_rope_split_bwd: bad args");
  hipLaunchKernelGGL(qkv_rope_split_bwd_kernel, dim3((unsigned)T, (unsigned)B), dim3(256), 0,
                     (hipStream_t)stream, (const bf16_t*)dq, (const bf16_t*)dk, (const bf16_t*)dv, pos, cs,
                     (bf16_t*)dqkv, T, (int)nh, (int)nkv, (int)hd, Lq, qoff, Lk, koff);
  PZ_CHECK_LAUNCH();
  return PZ_OK;
}

extern "C" int pz_attn_softmax(const pz_softmax_args* a, void* stream) {
  PZ_CHECK_ARG(a && a->S && a->P && a->R > 0 && a->N > 0 && a->ldp >= a->N && a->lds >= a->N,
               "attn_softmax: bad args");
  PZ_CHECK_ARG(a->N <= 1024, "attn_softmax: N=%lld > 1024 unsupported", (long long)a->N);
  if (a->mask_mode == 1) PZ_CHECK_ARG(a->cnt && a->rows_per_batch > 0 && a->heads > 0, "attn_softmax: block mask");
  if (a->mask_mode == 2) PZ_CHECK_ARG(a->mask && a->rows_per_batch > 0 && a->heads > 0, "attn_softmax: mask");
  dim3 grid((unsigned)((a->R + 3) / 4));
  hipStream_t st = (hipStream_t)stream;
  const bool vec = a->lds % 4 == 0 && a->ldp % 4 == 0 && PZ_ALIGNED(a->S, 16) && PZ_ALIGNED(a->P, 8) &&
                   (!a->tcap || PZ_ALIGNED(a->tcap, 8)) && a->R < (1LL << 31) && a->ldp <= 1024;
  if (vec) {
    if (a->ldp <= 512) hipLaunchKernelGGL(softmax4_kernel<2>, grid, dim3(256), 0, st, *a);
    else hipLaunchKernelGGL(softmax4_kernel<4>, grid, dim3(256), 0, st, *a);
    PZ_CHECK_LAUNCH();
    return PZ_OK;
  }
  if (a->N <= 256) hipLaunchKernelGGL(softmax_kernel<4>, grid, dim3(256), 0, st, *a);
  else if (a->N <= 512) hipLaunchKernelGGL(softmax_kernel<8>, grid, dim3(256), 0, st, *a);
  else hipLaunchKernelGGL(softmax_kernel<16>, grid, dim3(256), 0, st, *a);
  PZ_CHECK_LAUNCH();
  return PZ_OK;
}

extern "C" int pz_attn_softmax_bwd(const void* P, const float* dP, int64_t lddp, const void* tcap, void* dS,
                                   int64_t ldp, int64_t R, int64_t N, float scale, float cap, void* stream) {
  PZ_CHECK_ARG(P && dP && dS && R > 0 && N > 0 && N <= 1024 && (cap <= 0.f || tcap), "attn_softmax_bwd: bad args");
  dim3 grid((unsigned)((R + 3) / 4));
  hipStream_t st = (hipStream_t)stream;
  if (lddp % 4 == 0 && ldp % 4 == 0 && ldp <= 1024 && PZ_ALIGNED(dP, 16) && PZ_ALIGNED(P, 8) && PZ_ALIGNED(dS, 8) &&
      (cap <= 0.f || PZ_ALIGNED(tcap, 8))) {
    if (ldp <= 512)
      hipLaunchKernelGGL(softmax_bwd4_kernel<2>, grid, dim3(256), 0, st, (const bf16_t*)P, dP, lddp,
                         (const bf16_t*)tcap, (bf16_t*)dS, ldp, R, (int)N, scale, cap);
    else
      hipLaunchKernelGGL(softmax_bwd4_kernel<4>, grid, dim3(256), 0, st, (const bf16_t*)P, dP, lddp,
                         (const bf16_t*)tcap, (bf16_t*)dS, ldp, R, (int)N, scale, cap);
    PZ_CHECK_LAUNCH();
    return PZ_OK;
  }
  if (N <= 256)
    hipLaunchKernelGGL(softmax_bwd_kernel<4>, grid, dim3(256), 0, st, (const bf16_t*)P, dP, lddp,
                       (const bf16_t*)tcap, (bf16_t*)dS, ldp, R, N, scale, cap);
  else if (N <= 512)
    hipLaunchKernelGGL(softmax_bwd_kernel<8>, grid, dim3(256), 0, st, (const bf16_t*)P, dP, lddp,
                       (const bf16_t*)tcap, (bf16_t*)dS, ldp, R, N, scale, cap);
  else
    hipLaunchKernelGGL(softmax_bwd_kernel<16>, grid, dim3(256), 0, st, (const bf16_t*)P, dP, lddp,
                       (const bf16_t*)tcap, (bf16_t*)dS, ldp, R, N, scale, cap);
  PZ_CHECK_LAUNCH();
  return PZ_OK;
}
