// Small fused kernels around the Pi0 transformer stacks:
//   patch im2col (siglip.py:42-76), token embed + image merge (pizero.py:376-414),
//   sinusoidal time embedding + action-encoder concat (vla/modules.py:9-53),
//   flow-matching psi / loss / Euler update (pizero.py:479-489,597-661),
//   activation backward for fused GEMM epilogues, fused flat AdamW +
//   grad-norm clip (train.py:171-198,371-379), deterministic synthetic fill.
#include <math.h>

#include "pz_common.h"

namespace {

__global__ void patchify_kernel(const bf16_t* __restrict__ pix, bf16_t* cols, int64_t B, int64_t H, int64_t W,
                                int ps, int64_t ldc) {
  const int64_t gw = W / ps, gh = H / ps;
  const int64_t patch = blockIdx.x;  // over B*gh*gw
  const int64_t b = patch / (gh * gw), py = (patch / gw) % gh, px = patch % gw;
  bf16_t* out = cols + patch * ldc;
  const int kk = 3 * ps * ps;
  for (int k = threadIdx.x; k < ldc; k += blockDim.x) {
    bf16_t v = 0;
    if (k < kk) {
      const int c = k / (ps * ps), ky = (k / ps) % ps, kx = k % ps;
      v = pix[((b * 3 + c) * H + py * ps + ky) * W + px * ps + kx];
    }
    out[k] = v;
  }
}

__global__ void embed_merge_kernel(const int64_t* __restrict__ ids, const bf16_t* __restrict__ table, int64_t vocab,
                                   const bf16_t* __restrict__ img, bf16_t* out, int64_t P, int64_t D,
                                   int64_t n_img, int64_t image_token, int64_t pad_token, float emb_scale,
                                   float img_scale) {
  __shared__ int rank_s;
  const int64_t i = blockIdx.x, b = blockIdx.y;
  const int64_t id = ids[b * P + i];
  bf16_t* o = out + (b * P + i) * D;
  if (id == image_token) {
    if (threadIdx.x == 0) {
      int r = 0;
      for (int64_t j = 0; j < i; ++j) r += ids[b * P + j] == image_token;
      rank_s = r;
    }
    __syncthreads();
    const int64_t k = rank_s;
    if (k >= n_img) {
      for (int64_t d = threadIdx.x; d < D; d += blockDim.x) o[d] = 0;
      return;
    }
    const bf16_t* src = img + (b * n_img + k) * D;
    for (int64_t d = threadIdx.x; d < D; d += blockDim.x) o[d] = f2bf(bf2f(src[d]) * img_scale);
  } else if (id == pad_token || id < 0 || id >= vocab) {  // out-of-vocabulary ids never read the table
    for (int64_t d = threadIdx.x; d < D; d += blockDim.x) o[d] = 0;
  } else {
    const bf16_t* src = table + id * D;
    for (int64_t d = threadIdx.x; d < D; d += blockDim.x) o[d] = f2bf(bf2f(src[d]) * emb_scale);
  }
}

__global__ void embed_merge_bwd_kernel(const int64_t* __restrict__ ids, const bf16_t* __restrict__ dout,
                                       bf16_t* dimg, int64_t P, int64_t D, int64_t n_img, int64_t image_token,
                                       float img_scale) {
  __shared__ int rank_s;
  const int64_t i = blockIdx.x, b = blockIdx.y;
  if (ids[b * P + i] != image_token) return;
  if (threadIdx.x == 0) {
    int r = 0;
    for (int64_t j = 0; j < i; ++j) r += ids[b * P + j] == image_token;
    rank_s = r;
  }
  __syncthreads();
  const int64_t k = rank_s;
  if (k >= n_img) return;
  const bf16_t* src = dout + (b * P + i) * D;
  bf16_t* dst = dimg + (b * n_img + k) * D;
  for (int64_t d = threadIdx.x; d < D; d += blockDim.x) dst[d] = f2bf(bf2f(src[d]) * img_scale);
}

// mode 0: fp32 frequencies and product (the fp32 oracle's semantics);
// mode 1: the reference's bf16 arithmetic when the model runs in bf16 (vla/modules.py:15-22 with t in bf16,
// train.py:311): arange(half) in bf16 (integers above 256 round to even), every op's result rounded to bf16
__global__ void time_embed_kernel(const float* __restrict__ t, bf16_t* out, int64_t B, int D, float max_period,
                                  int mode) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= B * D) return;
  const int64_t b = idx / D;
  const int j = (int)(idx % D), half = D / 2;
  const int i = j < half ? j : j - half;
  const float e = (float)(log((double)max_period) / (double)(half - 1));
  float a;
  if (mode == 0) {
    a = t[b] * expf((float)i * -e);
  } else {
    const float ib = bf2f(f2bf((float)i));
    const float f = bf2f(f2bf(expf(bf2f(f2bf(ib * -e)))));
    a = bf2f(f2bf(bf2f(f2bf(t[b])) * f));
  }
  out[idx] = f2bf(j < half ? sinf(a) : cosf(a));
}

// time embedding written straight into the first D columns of the action encoder's concat input (inference:
// every one of a sample's H rows gets its sample's embedding; time_embed_kernel's arithmetic)
// column j of the time embedding of time tb (time_embed_kernel's arithmetic, both modes)
__device__ __forceinline__ bf16_t time_embed_col(float tb, int j, int D, float max_period, int mode) {
  const int half = D / 2;
  const int i = j < half ? j : j - half;
  const float e = (float)(log((double)max_period) / (double)(half - 1));
  float a;
  if (mode == 0) {
    a = tb * expf((float)i * -e);
  } else {
    const float ib = bf2f(f2bf((float)i));
    const float f = bf2f(f2bf(expf(bf2f(f2bf(ib * -e)))));
    a = bf2f(f2bf(bf2f(f2bf(tb)) * f));
  }
  return f2bf(j < half ? sinf(a) : cosf(a));
}

__global__ void time_embed_rows_kernel(const float* __restrict__ t, bf16_t* out, int64_t ldo, int64_t rows,
                                       int64_t H, int D, float max_period, int mode) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= rows * D) return;
  const int64_t r = idx / D;
  const int j = (int)(idx % D);
  out[r * ldo + j] = time_embed_col(t[r / H], j, D, max_period, mode);
}

// Denoise-step input in one launch (inference): cat[r] = [time embedding of sample r / H | linear_1(bf16(action[r]))]
// -- the bf16 cast, the 7 -> D action Linear (gemm_small_kernel's arithmetic: fp32 sum over k in order, bias, one
// bf16 rounding) and time_embed_rows_kernel, bit for bit, in one launch instead of three
__global__ void action_in_kernel(const float* __restrict__ action, int64_t A, const bf16_t* __restrict__ W1,
                                 const bf16_t* __restrict__ b1, const float* __restrict__ t, bf16_t* cat, int64_t ldc,
                                 int64_t rows, int64_t H, int D, float max_period, int mode) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= rows * 2 * D) return;
  const int64_t r = idx / (2 * D);
  const int j = (int)(idx % (2 * D));
  if (j < D) {
    cat[r * ldc + j] = time_embed_col(t[r / H], j, D, max_period, mode);
    return;
  }
  const int n = j - D;
  float s = 0.f;
  if (A <= 8) {  // (the action dims of every Pi0 config) all loads in flight before the first product, same sum order
    float xa[8], wa[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      xa[k] = k < A ? action[r * A + k] : 0.f;
      wa[k] = k < A ? bf2f(W1[n * A + k]) : 0.f;
    }
    const float bias = b1 ? bf2f(b1[n]) : 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (k < A) s += bf2f(f2bf(xa[k])) * wa[k];
    s *= 1.f;
    if (b1) s += bias;
  } else {
    for (int64_t k = 0; k < A; ++k) s += bf2f(f2bf(action[r * A + k])) * bf2f(W1[n * A + k]);
    s *= 1.f;
    if (b1) s += bf2f(b1[n]);
  }
  cat[r * ldc + j] = f2bf(s);
}

// Denoise-step output in one launch (inference), one wave per row: the action expert's final RMSNorm
// (rmsnorm_fwd_kernel's arithmetic: 8-element chunks lane + 64 c, fp32 sum of squares, y = x r (1 + w) rounded to
// bf16), the D -> A action decoder (gemm_small_rowwave_kernel's arithmetic on the same chunks, butterfly sum, bias,
// bf16 v) and the Euler update action += dt v (euler_kernel), bit for bit -- one launch instead of three.  D <= 1024,
// D % 8 == 0, A <= 8.
__global__ void __launch_bounds__(256) action_out_kernel(const bf16_t* __restrict__ x, int64_t ldx,
                                                         const bf16_t* __restrict__ nw, float eps,
                                                         const bf16_t* __restrict__ Wd, const bf16_t* __restrict__ bd,
                                                         int D, int A, float* action, float* t, int64_t rows,
                                                         int64_t H, float dt) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int nc = D / 8;
  constexpr int NMAX = 8;
  // every global load up front (the row, the norm weights, the decoder rows, bias and action): one memory round trip
  // instead of three dependent ones; the arithmetic below is unchanged
  u32x4 xq[2], wq[2], wd[2][NMAX];
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int ch = lane + 64 * c;
    const bool ok = ch < nc;
    xq[c] = ok ? *reinterpret_cast<const u32x4*>(x + row * ldx + ch * 8) : u32x4{0u, 0u, 0u, 0u};
    wq[c] = ok ? *reinterpret_cast<const u32x4*>(nw + ch * 8) : u32x4{0u, 0u, 0u, 0u};
#pragma unroll
    for (int n = 0; n < NMAX; ++n)
      wd[c][n] = ok && n < A ? *reinterpret_cast<const u32x4*>(Wd + n * (int64_t)D + ch * 8) : u32x4{0u, 0u, 0u, 0u};
  }
  const float bias = lane < A && bd ? bf2f(bd[lane]) : 0.f;
  const float act = lane < A ? action[row * A + lane] : 0.f;
  float v[2][8];
  float ss = 0.f;
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int ch = lane + 64 * c;
    if (ch < nc) {
      const u32x4 q = xq[c];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        v[c][2 * i] = __uint_as_float(q[i] << 16);
        v[c][2 * i + 1] = __uint_as_float(q[i] & 0xffff0000u);
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) ss += v[c][i] * v[c][i];
    }
  }
  ss = warp_sum(ss);
  const float r = rsqrtf(ss / (float)D + eps);
  u32x4 y[2] = {u32x4{0u, 0u, 0u, 0u}, u32x4{0u, 0u, 0u, 0u}};
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int ch = lane + 64 * c;
    if (ch < nc) {
      const u32x4 q = wq[c];
      float o[8];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        o[2 * i] = v[c][2 * i] * r * (1.f + __uint_as_float(q[i] << 16));
        o[2 * i + 1] = v[c][2 * i + 1] * r * (1.f + __uint_as_float(q[i] & 0xffff0000u));
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) y[c][i] = pack2bf(o[2 * i], o[2 * i + 1]);
    }
  }
  float s[NMAX];
#pragma unroll
  for (int n = 0; n < NMAX; ++n) s[n] = 0.f;
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int64_t k = 8 * lane + 512 * c;
    if (k >= D) break;
    const u32x4 xa = y[c];
    float xf[8];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      xf[2 * e] = bf2f(xa[e] & 0xffff);
      xf[2 * e + 1] = bf2f(xa[e] >> 16);
    }
#pragma unroll
    for (int n = 0; n < NMAX; ++n) {
      if (n >= A) break;
      const u32x4 wb = wd[c][n];
#pragma unroll
      for (int e = 0; e < 4; ++e) s[n] += xf[2 * e] * bf2f(wb[e] & 0xffff) + xf[2 * e + 1] * bf2f(wb[e] >> 16);
    }
  }
#pragma unroll
  for (int n = 0; n < NMAX; ++n) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) s[n] += __shfl_xor(s[n], off);
  }
  if (lane < A) {
    float o = 0.f;
#pragma unroll
    for (int n = 0; n < NMAX; ++n)
      if (n == lane) o = s[n];
    o *= 1.f;
    if (bd) o += bias;
    action[row * A + lane] = act + dt * bf2f(f2bf(o));
  }
  if (t && lane == 0 && row % H == 0) t[row / H] += dt;
}

__global__ void concat_time_kernel(const bf16_t* __restrict__ temb, const bf16_t* __restrict__ e1, bf16_t* out,
                                   int64_t rows, int64_t H, int64_t D) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= rows * 2 * D) return;
  const int64_t r = idx / (2 * D), c = idx % (2 * D);
  out[idx] = c < D ? temb[(r / H) * D + c] : e1[r * D + c - D];
}

__global__ void split_time_grad_kernel(const bf16_t* __restrict__ dcat, bf16_t* de1, int64_t rows, int64_t D) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= rows * D) return;
  const int64_t r = idx / D, c = idx % D;
  de1[idx] = dcat[r * 2 * D + D + c];
}

__global__ void flow_psi_kernel(const float* x0, const float* x1, const float* t, bf16_t* psi, int64_t B,
                                int64_t HA, float sig) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= B * HA) return;
  const float tt = t[idx / HA];
  psi[idx] = f2bf((1.f - (1.f - sig) * tt) * x0[idx] + tt * x1[idx]);
}

__global__ void flow_loss_kernel(const bf16_t* __restrict__ v, int64_t ldv, int64_t vbs,
                                 const float* __restrict__ x0, const float* __restrict__ x1, float* loss,
                                 bf16_t* dv, const float* __restrict__ gscale, int64_t H, int64_t rows, int64_t A,
                                 float sig) {
  __shared__ float red[4];
  const int64_t n = rows * A;
  float s = 0.f;
  const float g = gscale ? gscale[0] : 1.f;
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
    const int64_t r = i / A, c = i % A;
    const int64_t vo = (r / H) * vbs + (r % H) * ldv + c;
    const float d = x1[i] - (1.f - sig) * x0[i];
    const float e = bf2f(v[vo]) - d;
    s += e * e;
    if (dv) dv[vo] = f2bf(g * 2.f * e / (float)n);
  }
  s = block_sum<4>(s, red);
  if (threadIdx.x == 0) loss[0] = s / (float)n;
}

__global__ void euler_kernel(float* action, const bf16_t* __restrict__ v, int64_t ldv, int64_t vbs, float* t,
                             int64_t B, int64_t H, int64_t A, float dt) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx < B * H * A) {
    const int64_t r = idx / A, c = idx % A;
    action[idx] += dt * bf2f(v[(r / H) * vbs + (r % H) * ldv + c]);
  }
  if (t && idx < B) t[idx] += dt;
}


__global__ void copy_rows_kernel(const bf16_t* __restrict__ src, int64_t sld, int64_t sbs, bf16_t* dst, int64_t dld,
                                 int64_t dbs, int64_t rows, int64_t D, float scale, int beta) {
  const int64_t b = blockIdx.y;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < rows * D; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / D, d = i % D;
    float v = scale * bf2f(src[b * sbs + r * sld + d]);
    bf16_t* o = dst + b * dbs + r * dld + d;
    if (beta) v += bf2f(*o);
    *o = f2bf(v);
  }
}

__global__ void clamp_kernel(float* x, int64_t n, float lo, float hi) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx < n) x[idx] = fminf(fmaxf(x[idx], lo), hi);
}

__global__ void geglu_bwd_kernel(const bf16_t* __restrict__ dh, int64_t lddh, const bf16_t* gu, int64_t ldgu,
                                 bf16_t* dgu, bf16_t* h_out, int64_t ldh, int64_t M, int64_t I) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= M * I) return;
  const int64_t m = idx / I, n = idx % I;
  const float g = bf2f(gu[m * ldgu + n]), u = bf2f(gu[m * ldgu + I + n]);
  const float d = bf2f(dh[m * lddh + n]);
  float ge, gr;
  gelu_tanh_both(g, ge, gr);
  if (h_out) h_out[m * ldh + n] = f2bf(ge * u);
  dgu[m * ldgu + n] = f2bf(d * u * gr);
  dgu[m * ldgu + I + n] = f2bf(d * ge);
}

// vectorised forms (8 columns per thread, 16-byte accesses): the split dgrad + activation-backward
// of the training MLPs (HBM-bound: dh + saved activations read, d(pre) written once)
__device__ __forceinline__ void ld8(const bf16_t* p, float (&f)[8]) {
  const u32x4 r = *reinterpret_cast<const u32x4*>(p);
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    f[2 * e] = __uint_as_float(r[e] << 16);
    f[2 * e + 1] = __uint_as_float(r[e] & 0xffff0000u);
  }
}
__device__ __forceinline__ void st8(bf16_t* p, const float (&f)[8]) {
  *reinterpret_cast<u32x4*>(p) = u32x4{pack2bf(f[0], f[1]), pack2bf(f[2], f[3]), pack2bf(f[4], f[5]), pack2bf(f[6], f[7])};
}

__global__ void __launch_bounds__(256) geglu_bwd8_kernel(const bf16_t* __restrict__ dh, int64_t lddh, const bf16_t* gu,
                                                         int64_t ldgu, bf16_t* dgu, int64_t M, int64_t I8) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= M * I8) return;
  const int64_t m = idx / I8, n = (idx % I8) * 8, I = I8 * 8;
  float g[8], u[8], d[8], dg[8], du[8];
  ld8(gu + m * ldgu + n, g);
  ld8(gu + m * ldgu + I + n, u);
  ld8(dh + m * lddh + n, d);
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    float gl_, gr_;
    gelu_tanh_both(g[e], gl_, gr_);
    dg[e] = d[e] * u[e] * gr_;
    du[e] = d[e] * gl_;
  }
  st8(dgu + m * ldgu + n, dg);
  st8(dgu + m * ldgu + I + n, du);
}

__global__ void __launch_bounds__(256) act_bwd8_kernel(const bf16_t* __restrict__ dh, int64_t lddh, const bf16_t* pre,
                                                       int64_t ldpre, bf16_t* dpre, int64_t M, int64_t N8, int act) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= M * N8) return;
  const int64_t m = idx / N8, n = (idx % N8) * 8;
  float x[8], d[8];
  ld8(pre + m * ldpre + n, x);
  ld8(dh + m * lddh + n, d);
#pragma unroll
  for (int e = 0; e < 8; ++e) x[e] = d[e] * (act == PZ_EPI_GELU ? gelu_tanh_grad(x[e]) : silu_grad(x[e]));
  st8(dpre + m * ldpre + n, x);
}

__global__ void act_bwd_kernel(const bf16_t* __restrict__ dh, int64_t lddh, const bf16_t* pre, int64_t ldpre,
                               bf16_t* dpre, bf16_t* h_out, int64_t ldh, int64_t M, int64_t N, int act) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= M * N) return;
  const int64_t m = idx / N, n = idx % N;
  const float x = bf2f(pre[m * ldpre + n]);
  const float d = bf2f(dh[m * lddh + n]);
  float h, gr;
  if (act == PZ_EPI_GELU) {
    gelu_tanh_both(x, h, gr);
  } else {
    h = silu(x);
    gr = silu_grad(x);
  }
  if (h_out) h_out[m * ldh + n] = f2bf(h);
  dpre[m * ldpre + n] = f2bf(d * gr);
}

// AdamW (torch.optim.AdamW, decoupled weight decay), fp32 math, bf16 params
__global__ void adamw_kernel(bf16_t* __restrict__ p, const bf16_t* __restrict__ g, float* __restrict__ m,
                             float* __restrict__ v, int64_t n, float lr, float b1, float b2, float eps, float wd,
                             float bc1, float bc2, const float* __restrict__ gscale) {
  const float gs = gscale ? gscale[0] : 1.f;
  const float step = lr / bc1;
  const float bc2s = sqrtf(bc2);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float gr = bf2f(g[i]) * gs;
    float pv = bf2f(p[i]);
    pv *= (1.f - lr * wd);
    const float mi = b1 * m[i] + (1.f - b1) * gr;
    const float vi = b2 * v[i] + (1.f - b2) * gr * gr;
    m[i] = mi;
    v[i] = vi;
    pv -= step * mi / (sqrtf(vi) / bc2s + eps);
    p[i] = f2bf(pv);
  }
}

// one fp32 partial per block (no atomics): the global norm is summed in a fixed order by
// clip_coef_kernel, so the clip coefficient -- and training -- is bitwise reproducible
__global__ void sumsq_kernel(const bf16_t* __restrict__ g, int64_t n, float* parts) {
  __shared__ float red[4];
  float s = 0.f;
  const int64_t n8 = n / 8;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (int64_t)gridDim.x * blockDim.x) {
    u32x4 r = reinterpret_cast<const u32x4*>(g)[i];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float a = __uint_as_float(r[k] << 16), b = __uint_as_float(r[k] & 0xffff0000u);
      s += a * a + b * b;
    }
  }
  if (blockIdx.x == 0)
    for (int64_t i = n8 * 8 + threadIdx.x; i < n; i += blockDim.x) {
      const float a = bf2f(g[i]);
      s += a * a;
    }
  s = block_sum<4>(s, red);
  if (threadIdx.x == 0) parts[blockIdx.x] = s;
}

__global__ void clip_coef_kernel(const float* __restrict__ parts, int64_t nparts, float* coef, float* norm_out,
                                 float max_norm) {
  __shared__ float red[4];
  float s = 0.f;
  for (int64_t i = threadIdx.x; i < nparts; i += blockDim.x) s += parts[i];
  s = block_sum<4>(s, red);
  if (threadIdx.x == 0) {
    const float nrm = sqrtf(s);
    if (norm_out) norm_out[0] = nrm;
    coef[0] = fminf(1.f, max_norm / (nrm + 1e-6f));
  }
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ void fill_uniform_kernel(void* x, int out_fp32, int64_t n, uint64_t seed, float off, float scale) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t z = splitmix64(seed + (uint64_t)i);
    const float u = (float)(uint32_t)(z >> 40) * 0x1p-23f - 1.0f;
    // oracle/synth.py computes off + scale*u with two fp32 roundings: reproduce exactly
    const float w = __fadd_rn(off, __fmul_rn(scale, u));
    if (out_fp32) ((float*)x)[i] = w;
    else ((bf16_t*)x)[i] = f2bf(w);
  }
}

__global__ void cast_f32_bf16_kernel(const float* x, bf16_t* y, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = f2bf(x[i]);
}
__global__ void cast_bf16_f32_kernel(const bf16_t* x, float* y, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) y[i] = bf2f(x[i]);
}

inline unsigned nblk(int64_t n, int bs = 256) { return (unsigned)((n + bs - 1) / bs); }

}  // namespace

#define ST ((hipStream_t)stream)

extern "C" int pz_patchify(const void* pix, void* cols, int64_t B, int64_t H, int64_t W, int64_t ps, int64_t ldc,
                           void* stream) {
  PZ_CHECK_ARG(pix && cols && B > 0 && H % ps == 0 && W % ps == 0 && ldc >= 3 * ps * ps, "patchify: bad args");
  hipLaunchKernelGGL(patchify_kernel, dim3((unsigned)(B * (H / ps) * (W / ps))), dim3(256), 0, ST,
                     (const bf16_t*)pix, (bf16_t*)cols, B, H, W, (int)ps, ldc);
  PZ_CHECK_LAUNCH();
  return PZ_OK;
}

extern "C" int pz_embed_merge(const int64_t* ids, const void* table, int64_t vocab, const void* img, void* out,
                              int64_t B, int64_t P, int64_t D, int64_t n_img, int64_t image_token, int64_t pad_token,
                              float emb_scale, float img_scale, void* stream) {
  PZ_CHECK_ARG(ids && table && img && out && B > 0 && P > 0 && D > 0 && vocab > 0, "embed_merge: bad args");
  hipLaunchKernelGGL(embed_merge_kernel, dim3((unsigned)P, (unsigned)B), dim3(256), 0, ST, ids,
                     (const bf16_t*)table, vocab, (const bf16_t*)img, (bf16_t*)out, P, D, n_img, image_token,
                     pad_token, emb_scale, img_scale);
  PZ_CHECK_LAUNCH();
  return PZ_OK;
}

extern "C" int pz_embed_merge_bwd(const int64_t* ids, const void* dout, void* dimg, int64_t B, int64_t P,
                                  int64_t D, int64_t n_img, int64_t image_token, float img_scale, void* stream) {
  PZ_CHECK_ARG(ids && dout && dimg && B > 0 && P > 0 && D > 0, "embed_merge_bwd: bad args");
  hipLaunchKernelGGL(embed_merge_bwd_kernel, dim3((unsigned)P, (unsigned)B), dim3(256), 0, ST, ids,
                     (const bf16_t*)dout, (bf16_t*)dimg, P, D, n_img, image_token, img_scale);
  PZ_CHECK_LAUNCH();
  return PZ_OK;
}

extern "C" int pz_time_embed(const float* t, void* out, int64_t B, int64_t D, float max_period, int32_t mode,
                             void* stream) {
  PZ_CHECK_ARG(t && out && B > 0 && D % 2 == 0 && D >= 4 && (mode == 0 || mode == 1), "time_embed: bad args");
  hipLaunchKernelGGL(time_embed_kernel, dim3(nblk(B * D)), dim3(256), 0, ST, t, (bf16_t*)out, B, (int)D,
                     max_period, (int)mode);
  PZ_CHECK_LAUNCH();
  return PZ_OK;
}

extern "C" int pz_time_embed_rows(const float* t, void* out, int64_t ldo, int64_t B, int64_t H, int64_t D,
                                  float max_period, int32_t mode, void* stream) {
  PZ_CHECK_ARG(t && out && B > 0 && H > 0 && D >= 4 && D % 2 == 0 && ldo >= D && (mode == 0 || mode == 1),
               "time_embed_rows: bad args");
  hipLaunchKernelGGL(time_embed_rows_kernel, dim3(nblk(B * H * D)), dim3(256), 0, ST, t, (bf16_t*)out, ldo, B * H, H,
                     (int)D, max_period, (int)mode);
  PZ_CHECK_LAUNCH();
  return PZ_OK;
}

extern "C" int pz_action_in(const float* action, int64_t A, const void* w1, const void* b1, const float* t, void* cat,
                            int64_t ldc, int64_t B, int64_t H, int64_t D, float max_period, int32_t mode, void* stream) {
  PZ_CHECK_ARG(action && w1 && t && cat && A > 0 && B > 0 && H > 0 && D >= 4 && D % 2 == 0 && ldc >= 2 * D &&
                   (mode == 0 || mode == 1),
               "action_in: bad args");
  hipLaunchKernelGGL(action_in_kernel, dim3(nblk(B * H * 2 * D)), dim3(256), 0, ST, action, A, (const bf16_t*)w1,
                     (const bf16_t*)b1, t, (bf16_t*)cat, ldc, B * H, H, (int)D, max_period, (int)mode);
  PZ_CHECK_LAUNCH();
  return PZ_OK;
}

extern "C" int pz_action_out(const void* x, int64_t ldx, const void* norm_w, float eps, const void* wd, const void* bd,
                             int64_t D, int64_t A, float* action, float* t, int64_t B, int64_t H, float dt,
                             void* stream) {
  PZ_CHECK_ARG(x && norm_w && wd && action && B > 0 && H > 0 && A >= 1 && A <= 8 && D >= 8 && D <= 1024 &&
                   D % 8 == 0 && ldx % 8 == 0 && PZ_ALIGNED(x, 16) && PZ_ALIGNED(norm_w, 16) && PZ_ALIGNED(wd, 16),
               "action_out: D <= 1024, D %% 8 == 0, A <= 8, 16-byte aligned rows");
  const int64_t rows = B * H;
  hipLaunchKernelGGL(action_out_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, ST, (const bf16_t*)x, ldx,
                     (const bf16_t*)norm_w, eps, (const bf16_t*)wd, (const bf16_t*)bd, (int)D, (int)A, action, t, rows,
                     H, dt);
  PZ_CHECK_LAUNCH();
  return PZ_OK;
}

extern "C" int pz_concat_time(const void* temb, const void* e1, void* out, int64_t B, int64_t H, int64_t D,
                              void* stream) {
  PZ_CHECK_ARG(temb && e1 && out && B > 0 && H > 0 && D > 0, "concat_time: bad args");
  hipLaunchKernelGGL(concat_time_kernel, dim3(nblk(B * H * 2 * D)), dim3(256), 0, ST, (const bf16_t*)temb,
                     (const bf16_t*)e1, (bf16_t*)out, B * H, H, D);
  PZ_CHECK_LAUNCH();
  return PZ_OK;
}

extern "C" int pz_split_time_grad(const void* dcat, void* de1, int64_t rows, int64_t D, void* stream) {
  PZ_CHECK_ARG(dcat && de1 && rows > 0 && D > 0, "split_time_grad: bad args");
  hipLaunchKernelGGL(split_time_grad_kernel, dim3(nblk(rows * D)), dim3(256), 0, ST, (const bf16_t*)dcat,
                     (bf16_t*)de1, rows, D);
  PZ_CHECK_LAUNCH();
  return PZ_OK;
}

extern "C" int pz_flow_psi(const float* x0, const float* x1, const float* t, void* psi, int64_t B, int64_t HA,
                           float sig_min, void* stream) {
  PZ_CHECK_ARG(x0 && x1 && t && psi && B > 0 && HA > 0, "flow_psi: bad args");
  hipLaunchKernelGGL(flow_psi_kernel, dim3(nblk(B * HA)), dim3(256), 0, ST, x0, x1, t, (bf16_t*)psi, B, HA,
                     sig_min);
  PZ_CHECK_LAUNCH();
  return PZ_OK;
}

extern "C" int pz_flow_loss(const void* v, int64_t ldv, int64_t v_bstride, const float* x0, const float* x1,
                            float* loss, void* dv, const float* grad_scale, int64_t B, int64_t H, int64_t A,
                            float sig_min, void* stream) {
  PZ_CHECK_ARG(v && x0 && x1 && loss && B > 0 && H > 0 && A > 0, "flow_loss: bad args");
  hipLaunchKernelGGL(flow_loss_kernel, dim3(1), dim3(256), 0, ST, (const bf16_t*)v, ldv, v_bstride, x0, x1, loss,
                     (bf16_t*)dv, grad_scale, H, B * H, A, sig_min);
  PZ_CHECK_LAUNCH();
  return PZ_OK;
}

extern "C" int pz_euler_step(float* action, const void* v, int64_t ldv, int64_t v_bstride, float* t, int64_t B,
                             int64_t H, int64_t A, float dt, void* stream) {
  PZ_CHECK_ARG(action && v && B > 0, "euler_step: bad args");
  const int64_t n = B * H * A > B ? B * H * A : B;
  hipLaunchKernelGGL(euler_kernel, dim3(nblk(n)), dim3(256), 0, ST, action, (const bf16_t*)v, ldv, v_bstride, t, B,
                     H, A, dt);
  PZ_CHECK_LAUNCH();
  return PZ_OK;
}

extern "C" int pz_copy_rows(const void* src, int64_t sld, int64_t sbs, void* dst, int64_t dld, int64_t dbs, int64_t B,
                            int64_t rows, int64_t D, float scale, int32_t beta, void* stream) {
  PZ_CHECK_ARG(src && dst && B > 0 && rows > 0 && D > 0, "copy_rows: bad args");
  const int64_t n = rows * D;
  const unsigned gx = (unsigned)(n / 256 + 1 < 1024 ? n / 256 + 1 : 1024);
  hipLaunchKernelGGL(copy_rows_kernel, dim3(gx, (unsigned)B), dim3(256), 0, ST, (const bf16_t*)src, sld, sbs,
                     (bf16_t*)dst, dld, dbs, rows, D, scale, (int)beta);
  PZ_CHECK_LAUNCH();
  return PZ_OK;
}

extern "C" int pz_clamp(float* x, int64_t n, float lo, float hi, void* stream) {
  PZ_CHECK_ARG(x && n > 0, "clamp: bad args");
  hipLaunchKernelGGL(clamp_kernel, dim3(nblk(n)), dim3(256), 0, ST, x, n, lo, hi);
  PZ_CHECK_LAUNCH();
  return PZ_OK;
}

extern "C" int pz_geglu_bwd(const void* dh, int64_t lddh, const void* gu, int64_t ldgu, void* dgu, void* h_out,
                            int64_t ldh, int64_t M, int64_t I, void* stream) {
  PZ_CHECK_ARG(dh && gu && dgu && M > 0 && I > 0, "geglu_bwd: bad args");
  if (!h_out && I % 8 == 0 && lddh % 8 == 0 && ldgu % 8 == 0 && PZ_ALIGNED(dh, 16) && PZ_ALIGNED(gu, 16) &&
      PZ_ALIGNED(dgu, 16)) {
    const int64_t n = M * (I / 8);
    hipLaunchKernelGGL(geglu_bwd8_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, ST, (const bf16_t*)dh,
                       lddh, (const bf16_t*)gu, ldgu, (bf16_t*)dgu, M, I / 8);
    PZ_CHECK_LAUNCH();
    return PZ_OK;
  }
  hipLaunchKernelGGL(geglu_bwd_kernel, dim3(nblk(M * I)), dim3(256), 0, ST, (const bf16_t*)dh, lddh,
                     (const bf16_t*)gu, ldgu, (bf16_t*)dgu, (bf16_t*)h_out, ldh, M, I);
  PZ_CHECK_LAUNCH();
  return PZ_OK;
}

extern "C" int pz_act_bwd(const void* dh, int64_t lddh, const void* pre, int64_t ldpre, void* dpre, void* h_out,
                          int64_t ldh, int64_t M, int64_t N, int32_t act, void* stream) {
  PZ_CHECK_ARG(dh && pre && dpre && M > 0 && N > 0 && (act == PZ_EPI_GELU || act == PZ_EPI_SILU),
               "act_bwd: bad args");
  if (!h_out && N % 8 == 0 && lddh % 8 == 0 && ldpre % 8 == 0 && PZ_ALIGNED(dh, 16) && PZ_ALIGNED(pre, 16) &&
      PZ_ALIGNED(dpre, 16)) {
    const int64_t n = M * (N / 8);
    hipLaunchKernelGGL(act_bwd8_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, ST, (const bf16_t*)dh, lddh,
                       (const bf16_t*)pre, ldpre, (bf16_t*)dpre, M, N / 8, (int)act);
    PZ_CHECK_LAUNCH();
    return PZ_OK;
  }
  hipLaunchKernelGGL(act_bwd_kernel, dim3(nblk(M * N)), dim3(256), 0, ST, (const bf16_t*)dh, lddh,
                     (const bf16_t*)pre, ldpre, (bf16_t*)dpre, (bf16_t*)h_out, ldh, M, N, (int)act);
  PZ_CHECK_LAUNCH();
  return PZ_OK;
}

extern "C" int pz_adamw(void* p, const void* g, float* m, float* v, int64_t n, float lr, float beta1, float beta2,
                        float eps, float wd, float bc1, float bc2, const float* gscale, void* stream) {
  PZ_CHECK_ARG(p && g && m && v && n >= 0, "adamw: bad args");
  if (n == 0) return PZ_OK;
  const int64_t blocks = n / 256 + 1 < 8192 ? n / 256 + 1 : 8192;
  hipLaunchKernelGGL(adamw_kernel, dim3((unsigned)blocks), dim3(256), 0, ST, (bf16_t*)p, (const bf16_t*)g, m, v, n,
                     lr, beta1, beta2, eps, wd, bc1, bc2, gscale);
  PZ_CHECK_LAUNCH();
  return PZ_OK;
}

extern "C" int pz_sumsq(const void* g, int64_t n, float* parts, void* stream) {
  PZ_CHECK_ARG(g && parts && n >= 0 && PZ_ALIGNED(g, 16), "sumsq: bad args (16-byte alignment)");
  hipLaunchKernelGGL(sumsq_kernel, dim3(PZ_SUMSQ_PARTS), dim3(256), 0, ST, (const bf16_t*)g, n, parts);
  PZ_CHECK_LAUNCH();
  return PZ_OK;
}

extern "C" int pz_clip_coef(const float* parts, int64_t nparts, float* coef, float* norm_out, float max_norm,
                            void* stream) {
  PZ_CHECK_ARG(parts && coef && nparts > 0, "clip_coef: bad args");
  hipLaunchKernelGGL(clip_coef_kernel, dim3(1), dim3(256), 0, ST, parts, nparts, coef, norm_out, max_norm);
  PZ_CHECK_LAUNCH();
  return PZ_OK;
}

extern "C" int pz_fill_uniform(void* x, int32_t out_fp32, int64_t n, uint64_t seed, float off, float scale,
                               void* stream) {
  PZ_CHECK_ARG(x && n >= 0, "fill_uniform: bad args");
  if (n == 0) return PZ_OK;
  const int64_t blocks = n / 256 + 1 < 16384 ? n / 256 + 1 : 16384;
  hipLaunchKernelGGL(fill_uniform_kernel, dim3((unsigned)blocks), dim3(256), 0, ST, x, (int)out_fp32, n, seed, off,
                     scale);
  PZ_CHECK_LAUNCH();
  return PZ_OK;
}

extern "C" int pz_cast_f32_bf16(const float* x, void* y, int64_t n, void* stream) {
  PZ_CHECK_ARG(x && y && n >= 0, "cast: bad args");
  if (n == 0) return PZ_OK;
  hipLaunchKernelGGL(cast_f32_bf16_kernel, dim3(nblk(n)), dim3(256), 0, ST, x, (bf16_t*)y, n);
  PZ_CHECK_LAUNCH();
  return PZ_OK;
}

extern "C" int pz_cast_bf16_f32(const void* x, float* y, int64_t n, void* stream) {
  PZ_CHECK_ARG(x && y && n >= 0, "cast: bad args");
  if (n == 0) return PZ_OK;
  hipLaunchKernelGGL(cast_bf16_f32_kernel, dim3(nblk(n)), dim3(256), 0, ST, (const bf16_t*)x, y, n);
  PZ_CHECK_LAUNCH();
  return PZ_OK;
}

// ---- test instrument (tests/test_train_loop_gpu.py, PZ_POISON_LDS) ------------------------------------------------
// Fill the LDS of every CU with one 32-bit word (0xffffffff is NaN as fp32 and as both bf16 halves), so a kernel that
// reads LDS it never wrote meets NaN instead of an earlier kernel's mostly-finite leftovers.  One 160 KiB workgroup
// per CU at a time, 8 x the CU count of them: every CU runs several.
constexpr int PZ_LDS_BYTES = 160 * 1024;

__global__ void __launch_bounds__(256) poison_lds_kernel(uint32_t word) {
  extern __shared__ __attribute__((aligned(16))) char pz_poison_smem[];
  volatile u32x4* p = reinterpret_cast<volatile u32x4*>(pz_poison_smem);
  for (int i = threadIdx.x; i < PZ_LDS_BYTES / 16; i += 256) {
    p[i].x = word;
    p[i].y = word;
    p[i].z = word;
    p[i].w = word;
  }
}

extern "C" int pz_debug_poison_lds(uint32_t word, void* stream) {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
      cus = 256;
    if (hipFuncSetAttribute((const void*)poison_lds_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                            PZ_LDS_BYTES) != hipSuccess)
      (void)hipGetLastError();
  }
  hipLaunchKernelGGL(poison_lds_kernel, dim3((unsigned)(8 * cus)), dim3(256), PZ_LDS_BYTES, ST, word);
  PZ_CHECK_LAUNCH();
  return PZ_OK;
}

// test instrument (tools/contention_probe.py): `wgs` workgroups that each hold a CU (96 KiB of LDS: one per CU, and no
// 160 KiB persistent / 8-phase workgroup fits beside it) for `ticks` of the constant-rate wall clock -- a stand-in
// for the RCCL kernels that share the CUs with the backward under data parallelism
__global__ void __launch_bounds__(64) spin_kernel(int64_t ticks) {
  extern __shared__ __attribute__((aligned(16))) char pz_spin_smem[];
  const uint64_t t0 = wall_clock64();
  while ((int64_t)(wall_clock64() - t0) < ticks) __builtin_amdgcn_s_sleep(8);
  if (threadIdx.x == 0 && ticks < 0) pz_spin_smem[0] = 0;  // (never: keeps the LDS allocation)
}

extern "C" int pz_debug_spin(int64_t wgs, int64_t ticks, void* stream) {
  PZ_CHECK_ARG(wgs > 0 && wgs <= 65536 && ticks >= 0, "debug_spin: bad args");
  static bool attr = false;
  if (!attr) {
    if (hipFuncSetAttribute((const void*)spin_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024) !=
        hipSuccess)
      (void)hipGetLastError();
    attr = true;
  }
  hipLaunchKernelGGL(spin_kernel, dim3((unsigned)wgs), dim3(64), 96 * 1024, ST, ticks);
  PZ_CHECK_LAUNCH();
  return PZ_OK;
}
