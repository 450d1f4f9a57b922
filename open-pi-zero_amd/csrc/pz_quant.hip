// fp8 (OCP e4m3fn) quantisation for the C5 fp8 path (BASELINE.json configs[4]: "fp8 MFMA attention/MLP").
//
// Activations: per-row scales (one workgroup per row holds the row in registers: max|x| by a block
// reduction, then every element divided by s = max/448 and converted with v_cvt_pk_fp8_f32 -- RNE,
// in range by construction, so no saturation path is ever taken).  Weights: one per-tensor scale,
// computed once at load from pz_fp8_absmax partials.  HBM-bound byte work: 2 B read + 1 B written
// per element.
#include "pz_common.h"

namespace {

constexpr float E4M3_MAX = 448.f;

__device__ __forceinline__ unsigned enc4(float a, float b, float c, float d) {
  int v = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  v = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, v, true);
  return (unsigned)v;
}

__device__ __forceinline__ void unpack8f(const u32x4& r, float (&f)[8]) {
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    f[2 * e] = __uint_as_float(r[e] << 16);
    f[2 * e + 1] = __uint_as_float(r[e] & 0xffff0000u);
  }
}

// one row per workgroup; thread t owns 8-element chunks t, t + 256, ... (CH of them, in registers)
template <int CH>
__global__ void __launch_bounds__(256) quant_rows_kernel(const bf16_t* __restrict__ x, int64_t ldx, uint8_t* q,
                                                         int64_t ldq, float* row_scale, int64_t D) {
  __shared__ float red[4];
  const int64_t r = blockIdx.x;
  const int t = threadIdx.x;
  const int64_t nch = D / 8;
  const bf16_t* xr = x + r * ldx;
  u32x4 v[CH];
  float m = 0.f;
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int64_t ch = t + (int64_t)c * 256;
    v[c] = ch < nch ? *reinterpret_cast<const u32x4*>(xr + ch * 8) : u32x4{0u, 0u, 0u, 0u};
    float f[8];
    unpack8f(v[c], f);
#pragma unroll
    for (int e = 0; e < 8; ++e) m = fmaxf(m, fabsf(f[e]));
  }
  m = warp_max(m);
  if ((t & 63) == 0) red[t >> 6] = m;
  __syncthreads();
  m = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  const float s = m > 0.f ? __fdiv_rn(m, E4M3_MAX) : 1.f;  // IEEE quotients (reproducible scales)
  const float inv = __fdiv_rn(1.f, s);
  if (t == 0) row_scale[r] = s;
  uint8_t* qr = q + r * ldq;
#pragma unroll
  for (int c = 0; c < CH; ++c) {
    const int64_t ch = t + (int64_t)c * 256;
    if (ch >= nch) break;
    float f[8];
    unpack8f(v[c], f);
    // clamp guards the one rounding case x/s = 448 * (1 + ulp) (never above the max code)
#pragma unroll
    for (int e = 0; e < 8; ++e) f[e] = fminf(fmaxf(f[e] * inv, -E4M3_MAX), E4M3_MAX);
    *reinterpret_cast<u32x2*>(qr + ch * 8) = u32x2{enc4(f[0], f[1], f[2], f[3]), enc4(f[4], f[5], f[6], f[7])};
  }
}

__global__ void __launch_bounds__(256) quant_tensor_kernel(const bf16_t* __restrict__ x, int64_t n8, uint8_t* q,
                                                           float inv_scale) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n8) return;
  float f[8];
  unpack8f(*reinterpret_cast<const u32x4*>(x + i * 8), f);
#pragma unroll
  for (int e = 0; e < 8; ++e) f[e] = fminf(fmaxf(f[e] * inv_scale, -E4M3_MAX), E4M3_MAX);
  *reinterpret_cast<u32x2*>(q + i * 8) = u32x2{enc4(f[0], f[1], f[2], f[3]), enc4(f[4], f[5], f[6], f[7])};
}

// max |x| partials: grid-stride over 8-element chunks, one partial per workgroup (fixed order)
__global__ void __launch_bounds__(256) absmax_kernel(const bf16_t* __restrict__ x, int64_t n8, float* parts) {
  __shared__ float red[4];
  float m = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    float f[8];
    unpack8f(*reinterpret_cast<const u32x4*>(x + i * 8), f);
#pragma unroll
    for (int e = 0; e < 8; ++e) m = fmaxf(m, fabsf(f[e]));
  }
  m = warp_max(m);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) parts[blockIdx.x] = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}

// V^T codes for the fp8 attention (pz_flash_fwd_f8): one scale per head dim d (the column max over the nk keys:
// O[q][d] = s_d sum_k P[q][k] v_kd, so a per-column scale factors out of the P V sum exactly), codes written transposed
// [256 d][ldt keys], zeros for nk <= k < ldt.  Workgroup (sample, 8 d-columns): pass 1 -- thread (key phase kp of 32,
// column dl of 8) takes the max over keys kp, kp + 32, ... (8 loads in flight), reduced through LDS; pass 2 -- thread
// (dl, 16-key group) reads its 16 keys' values and writes their 16 codes as one 16-B store.
__global__ void __launch_bounds__(256) quant_vt_kernel(const bf16_t* __restrict__ v, int64_t ldv, int64_t vb, int64_t nk,
                                                       uint8_t* vt, float* vs, int64_t ldt) {
  __shared__ float red[32][8];
  __shared__ float sc[8];
  const int64_t b = blockIdx.x;
  const int dl = threadIdx.x & 7, kp = threadIdx.x >> 3;
  const int64_t d0 = (int64_t)blockIdx.y * 8;
  const bf16_t* V = v + b * vb + d0 + dl;
  float m = 0.f;
  int64_t k = kp;
  for (; k + 7 * 32 < nk; k += 8 * 32) {
    float x[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) x[u] = fabsf(bf2f(V[(k + 32 * u) * ldv]));
#pragma unroll
    for (int u = 0; u < 8; ++u) m = fmaxf(m, x[u]);
  }
  for (; k < nk; k += 32) m = fmaxf(m, fabsf(bf2f(V[k * ldv])));
  red[kp][dl] = m;
  __syncthreads();
  if (threadIdx.x < 8) {
    float mm = 0.f;
    for (int i = 0; i < 32; ++i) mm = fmaxf(mm, red[i][threadIdx.x]);
    const float s = mm > 0.f ? __fdiv_rn(mm, E4M3_MAX) : 1.f;
    sc[threadIdx.x] = s;
    vs[b * 256 + d0 + threadIdx.x] = s;
  }
  __syncthreads();
  const float inv = __fdiv_rn(1.f, sc[dl]);
  uint8_t* T = vt + (b * 256 + d0 + dl) * ldt;
  for (int64_t k0 = (int64_t)kp * 16; k0 < ldt; k0 += 32 * 16) {
    float f[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const int64_t kk = k0 + e;
      f[e] = kk < nk ? fminf(fmaxf(bf2f(V[kk * ldv]) * inv, -E4M3_MAX), E4M3_MAX) : 0.f;
    }
    *reinterpret_cast<u32x4*>(T + k0) = u32x4{enc4(f[0], f[1], f[2], f[3]), enc4(f[4], f[5], f[6], f[7]),
                                              enc4(f[8], f[9], f[10], f[11]), enc4(f[12], f[13], f[14], f[15])};
  }
}

// all operands of one fp8 attention launch in ONE launch (pz_fp8_quant_attn): rows of Q then rows of K (256 wide,
// per-row scales as quant_rows_kernel: one wave per row, 4 values per lane), then V^T (quant_vt_kernel's workgroups)
__global__ void __launch_bounds__(256) quant_attn_kernel(const bf16_t* __restrict__ q, int64_t nqr,
                                                         const bf16_t* __restrict__ k, int64_t nkr,
                                                         const bf16_t* __restrict__ v, int64_t ldv, int64_t vb,
                                                         int64_t Z, int64_t nk, uint8_t* qc, float* qs, uint8_t* kc,
                                                         float* ks, uint8_t* vt, float* vs, int64_t ldt) {
  const int64_t row_wgs = (nqr + nkr + 3) / 4;
  if ((int64_t)blockIdx.x >= row_wgs) {  // V^T: workgroup (sample, 8 columns) of the quant_vt_kernel scheme
    const int64_t u = blockIdx.x - row_wgs;
    __shared__ float red[32][8];
    __shared__ float sc[8];
    const int64_t b = u / 32;
    const int dl = threadIdx.x & 7, kp = threadIdx.x >> 3;
    const int64_t d0 = (u % 32) * 8;
    const bf16_t* V = v + b * vb + d0 + dl;
    float m = 0.f;
    int64_t kk = kp;
    for (; kk + 7 * 32 < nk; kk += 8 * 32) {
      float x[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) x[e] = fabsf(bf2f(V[(kk + 32 * e) * ldv]));
#pragma unroll
      for (int e = 0; e < 8; ++e) m = fmaxf(m, x[e]);
    }
    for (; kk < nk; kk += 32) m = fmaxf(m, fabsf(bf2f(V[kk * ldv])));
    red[kp][dl] = m;
    __syncthreads();
    if (threadIdx.x < 8) {
      float mm = 0.f;
      for (int i = 0; i < 32; ++i) mm = fmaxf(mm, red[i][threadIdx.x]);
      const float s = mm > 0.f ? __fdiv_rn(mm, E4M3_MAX) : 1.f;
      sc[threadIdx.x] = s;
      vs[b * 256 + d0 + threadIdx.x] = s;
    }
    __syncthreads();
    const float inv = __fdiv_rn(1.f, sc[dl]);
    uint8_t* T = vt + (b * 256 + d0 + dl) * ldt;
    for (int64_t k0 = (int64_t)kp * 16; k0 < ldt; k0 += 32 * 16) {
      float f[16];
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int64_t key = k0 + e;
        f[e] = key < nk ? fminf(fmaxf(bf2f(V[key * ldv]) * inv, -E4M3_MAX), E4M3_MAX) : 0.f;
      }
      *reinterpret_cast<u32x4*>(T + k0) = u32x4{enc4(f[0], f[1], f[2], f[3]), enc4(f[4], f[5], f[6], f[7]),
                                                enc4(f[8], f[9], f[10], f[11]), enc4(f[12], f[13], f[14], f[15])};
    }
    return;
  }
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= nqr + nkr) return;
  const int lane = threadIdx.x & 63;
  const bool isq = r < nqr;
  const int64_t rr = isq ? r : r - nqr;
  const u32x2 w = *reinterpret_cast<const u32x2*>((isq ? q : k) + rr * 256 + 4 * lane);
  float f[4] = {__uint_as_float(w[0] << 16), __uint_as_float(w[0] & 0xffff0000u), __uint_as_float(w[1] << 16),
                __uint_as_float(w[1] & 0xffff0000u)};
  float m = fmaxf(fmaxf(fabsf(f[0]), fabsf(f[1])), fmaxf(fabsf(f[2]), fabsf(f[3])));
  m = warp_max(m);
  const float s = m > 0.f ? __fdiv_rn(m, E4M3_MAX) : 1.f;
  const float inv = __fdiv_rn(1.f, s);
#pragma unroll
  for (int e = 0; e < 4; ++e) f[e] = fminf(fmaxf(f[e] * inv, -E4M3_MAX), E4M3_MAX);
  *reinterpret_cast<unsigned*>((isq ? qc : kc) + rr * 256 + 4 * lane) = enc4(f[0], f[1], f[2], f[3]);
  if (lane == 0) (isq ? qs : ks)[rr] = s;
}

}  // namespace

extern "C" int pz_fp8_quant_attn(const void* q, int64_t nqr, const void* k, int64_t nkr, const void* v, int64_t ldv,
                                 int64_t v_bstride, int64_t Z, int64_t nk, void* qc, float* qs, void* kc, float* ks,
                                 void* vt, float* vs, int64_t ldt, void* stream) {
  PZ_CHECK_ARG(q && k && v && qc && qs && kc && ks && vt && vs && nqr > 0 && nkr > 0 && Z > 0 && nk > 0 &&
                   ldt >= nk && ldt % 16 == 0 && PZ_ALIGNED(q, 8) && PZ_ALIGNED(k, 8) && PZ_ALIGNED(qc, 4) &&
                   PZ_ALIGNED(kc, 4) && PZ_ALIGNED(vt, 16),
               "fp8_quant_attn: bad args (rows of 256, ldt >= nk, ldt %% 16 == 0, aligned)");
  const int64_t wgs = (nqr + nkr + 3) / 4 + Z * 32;
  PZ_CHECK_ARG(wgs < (1LL << 31), "fp8_quant_attn: too many rows");
  hipLaunchKernelGGL(quant_attn_kernel, dim3((unsigned)wgs), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)q, nqr,
                     (const bf16_t*)k, nkr, (const bf16_t*)v, ldv, v_bstride, Z, nk, (uint8_t*)qc, qs, (uint8_t*)kc,
                     ks, (uint8_t*)vt, vs, ldt);
  PZ_CHECK_LAUNCH();
  return PZ_OK;
}

extern "C" int pz_fp8_quant_vt(const void* v, int64_t ldv, int64_t v_bstride, int64_t Z, int64_t nk, void* vt,
                               float* vs, int64_t ldt, void* stream) {
  PZ_CHECK_ARG(v && vt && vs && Z > 0 && nk > 0 && ldt >= nk && ldt % 16 == 0 && PZ_ALIGNED(vt, 16) && Z < 65536,
               "fp8_quant_vt: bad args (ldt >= nk, ldt %% 16 == 0, 16-byte aligned codes)");
  hipLaunchKernelGGL(quant_vt_kernel, dim3((unsigned)Z, 32), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)v, ldv,
                     v_bstride, nk, (uint8_t*)vt, vs, ldt);
  PZ_CHECK_LAUNCH();
  return PZ_OK;
}

extern "C" int pz_fp8_quant_rows(const void* x, int64_t ldx, void* q, int64_t ldq, float* row_scale, int64_t R,
                                 int64_t D, void* stream) {
  PZ_CHECK_ARG(x && q && row_scale && R > 0 && D > 0 && D % 8 == 0 && D <= 8 * 256 * 8,
               "fp8_quant_rows: bad args (D %% 8 == 0, D <= 16384)");
  PZ_CHECK_ARG(PZ_ALIGNED(x, 16) && PZ_ALIGNED(q, 8) && ldx % 8 == 0 && ldq % 8 == 0 && R < (1LL << 31),
               "fp8_quant_rows: alignment");
  const int ch = (int)((D / 8 + 255) / 256);
  hipStream_t st = (hipStream_t)stream;
  const bf16_t* xb = (const bf16_t*)x;
  uint8_t* qb = (uint8_t*)q;
  switch (ch) {
    case 1: hipLaunchKernelGGL(quant_rows_kernel<1>, dim3((unsigned)R), dim3(256), 0, st, xb, ldx, qb, ldq, row_scale, D); break;
    case 2: hipLaunchKernelGGL(quant_rows_kernel<2>, dim3((unsigned)R), dim3(256), 0, st, xb, ldx, qb, ldq, row_scale, D); break;
    case 3:
    case 4: hipLaunchKernelGGL(quant_rows_kernel<4>, dim3((unsigned)R), dim3(256), 0, st, xb, ldx, qb, ldq, row_scale, D); break;
    default: hipLaunchKernelGGL(quant_rows_kernel<8>, dim3((unsigned)R), dim3(256), 0, st, xb, ldx, qb, ldq, row_scale, D); break;
  }
  PZ_CHECK_LAUNCH();
  return PZ_OK;
}

extern "C" int pz_fp8_quant_tensor(const void* x, int64_t n, void* q, float inv_scale, void* stream) {
  PZ_CHECK_ARG(x && q && n > 0 && n % 8 == 0 && PZ_ALIGNED(x, 16) && PZ_ALIGNED(q, 8) && inv_scale > 0.f,
               "fp8_quant_tensor: bad args (n %% 8 == 0, aligned, inv_scale > 0)");
  const int64_t n8 = n / 8;
  hipLaunchKernelGGL(quant_tensor_kernel, dim3((unsigned)((n8 + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     (const bf16_t*)x, n8, (uint8_t*)q, inv_scale);
  PZ_CHECK_LAUNCH();
  return PZ_OK;
}

extern "C" int pz_fp8_absmax(const void* x, int64_t n, float* parts, void* stream) {
  PZ_CHECK_ARG(x && parts && n > 0 && n % 8 == 0 && PZ_ALIGNED(x, 16), "fp8_absmax: bad args (n %% 8 == 0)");
  hipLaunchKernelGGL(absmax_kernel, dim3(PZ_ABSMAX_PARTS), dim3(256), 0, (hipStream_t)stream, (const bf16_t*)x,
                     n / 8, parts);
  PZ_CHECK_LAUNCH();
  return PZ_OK;
}
