// Few-row GEMV kernels for the B=1..2 inference path (denoise steps: 4-8 action rows; the proprio row
// of the prefill): y[M, N] = epi(x[M, K] . W[N, K]^T) with M <= 8.
//
// Weight streaming is the whole cost (every weight byte read once per call), so the design is the
// decode rule of the CDNA4 guide: every CU in the launch (>= 256 workgroups for the Pi0 widths),
// weights loaded straight into VGPRs with all of a thread's 16-byte loads in flight before the first
// FMA, fp32 FMAs on the VALU (M x 8 per weight chunk -- no MFMA tile to fill), one wave-shuffle +
// LDS reduction at the end.  A block of 256 threads = GPB groups of TPG = min(256, K/8) threads; a
// group owns CPG output columns (GeGLU: CPG gate columns and the matching up columns) and its threads
// split K in 8-element chunks.  Optional fused Gemma RMSNorm of the x rows (the group sees every k,
// so it has the full sum of squares), bias, residual, GELU / SiLU (+ saved pre-activation), GeGLU
// (+ saved g|u).  pz_gemv_qkv_rope adds the RoPE + Q / K-cache / V-cache scatter of the joint
// attention (joint_model.py:170-257, utils.py:4-16) as the epilogue of the q|k|v projection.
#include "pz_common.h"

namespace {

struct GemvP {
  const bf16_t* x;
  int64_t ldx;
  const bf16_t* W;
  int64_t ldw;
  int64_t M, N, K;  // N = output columns (GeGLU: I, W has 2I rows)
  void* y;
  int64_t ldy;
  int c_fp32, beta, epi;
  float alpha;
  const bf16_t* bias;
  const bf16_t* resid;
  int64_t ldr;
  bf16_t* aux;
  int64_t ldaux;
  const bf16_t* nw;
  float neps;
  // RoPE scatter (qkv): pos [M], table cs [(pos)*hd + 2i (+1)], outputs
  const int64_t* pos;
  const float* cs;
  bf16_t *q, *k, *v;
  int64_t T, nh, hd, Lq, qoff, Lk, koff;
};

__device__ __forceinline__ void unpack8(const u32x4& r, float (&f)[8]) {
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    f[2 * e] = __uint_as_float(r[e] << 16);
    f[2 * e + 1] = __uint_as_float(r[e] & 0xffff0000u);
  }
}

// Main body: accumulate acc[r][c] over this thread's k chunks (rows r < M of x, CW weight rows)
template <int MR, int CW, int TPG>
__device__ __forceinline__ void gemv_body(const GemvP& p, const int64_t* wrow, const bool* wok, int j,
                                          float (&acc)[MR][CW], float (&ss)[MR]) {
  const int64_t KC = p.K / 8;
#pragma unroll
  for (int r = 0; r < MR; ++r) {
    ss[r] = 0.f;
#pragma unroll
    for (int c = 0; c < CW; ++c) acc[r][c] = 0.f;
  }
  const bool nrm = p.nw != nullptr;
  for (int64_t kc = j; kc < KC; kc += TPG) {
    u32x4 wr[CW];
#pragma unroll
    for (int c = 0; c < CW; ++c)
      wr[c] = wok[c] ? *reinterpret_cast<const u32x4*>(p.W + wrow[c] * p.ldw + kc * 8) : u32x4{0u, 0u, 0u, 0u};
    u32x4 xr[MR];
#pragma unroll
    for (int r = 0; r < MR; ++r)
      xr[r] = r < p.M ? *reinterpret_cast<const u32x4*>(p.x + r * p.ldx + kc * 8) : u32x4{0u, 0u, 0u, 0u};
    float wn[8];
    if (nrm) unpack8(*reinterpret_cast<const u32x4*>(p.nw + kc * 8), wn);
#pragma unroll
    for (int r = 0; r < MR; ++r) {
      float xf[8];
      unpack8(xr[r], xf);
      if (nrm) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          ss[r] += xf[e] * xf[e];
          xf[e] *= 1.f + wn[e];
        }
      }
#pragma unroll
      for (int c = 0; c < CW; ++c) {
        float wf[8];
        unpack8(wr[c], wf);
#pragma unroll
        for (int e = 0; e < 8; ++e) acc[r][c] += xf[e] * wf[e];
      }
    }
  }
}

// Reduce acc / ss over the TPG threads of each group through LDS (a shuffle tree per accumulator
// costs ~6 dependent cross-lane ops x MR*CW values): every thread writes its NV = MR*CW (+MR) partials
// value-major, then TPO threads per (group, value) sum contiguous slices and finish with
// log2(TPO) shuffles.  Result: fin[g * NV + v] (v < MR*CW: acc[r][c] at r*CW + c; then ss[r]).
template <int MR, int CW, int TPG>
__device__ __forceinline__ void gemv_reduce(float (&acc)[MR][CW], float (&ss)[MR], float* red, float* fin,
                                            bool nrm) {
  constexpr int GPB = 256 / TPG;
  constexpr int NV = MR * CW + MR;
  constexpr int O = GPB * NV;
  constexpr int TPO0 = O >= 256 ? 1 : 256 / O;
  constexpr int TPO = TPO0 >= 16 ? 16 : TPO0 >= 8 ? 8 : TPO0 >= 4 ? 4 : TPO0 >= 2 ? 2 : 1;
  constexpr int SL = TPG / TPO;
  const int t = threadIdx.x;
#pragma unroll
  for (int r = 0; r < MR; ++r) {
#pragma unroll
    for (int c = 0; c < CW; ++c) red[(r * CW + c) * 256 + t] = acc[r][c];
    red[(MR * CW + r) * 256 + t] = nrm ? ss[r] : 0.f;
  }
  __syncthreads();
  for (int ob = 0; ob < O; ob += 256 / TPO) {
    const int o = ob + t / TPO, part = t % TPO;
    float s = 0.f;
    if (o < O) {
      const int g = o / NV, v = o % NV;
      const float4* src = reinterpret_cast<const float4*>(red + v * 256 + g * TPG + part * SL);
#pragma unroll
      for (int i = 0; i < SL / 4; ++i) {
        const float4 q = src[i];
        s += (q.x + q.y) + (q.z + q.w);
      }
    }
#pragma unroll
    for (int w = TPO / 2; w > 0; w >>= 1) s += __shfl_xor(s, w, 64);
    if (o < O && part == 0) fin[o] = s;
  }
  __syncthreads();
}

template <int MR, int CPG, int TPG, bool GEGLU>
__global__ void __launch_bounds__(256) gemv_kernel(GemvP p) {
  constexpr int GPB = 256 / TPG;
  constexpr int CW = GEGLU ? 2 * CPG : CPG;
  constexpr int NV = MR * CW + MR;
  __shared__ __attribute__((aligned(16))) float red[NV * 256];
  __shared__ float fin[GPB * NV];
  const int g = threadIdx.x / TPG, j = threadIdx.x % TPG;
  const int64_t col0 = ((int64_t)blockIdx.x * GPB + g) * CPG;
  int64_t wrow[CW];
  bool wok[CW];
#pragma unroll
  for (int c = 0; c < CPG; ++c) {
    wrow[c] = col0 + c;
    wok[c] = col0 + c < p.N;
    if (GEGLU) {
      wrow[CPG + c] = p.N + col0 + c;
      wok[CPG + c] = wok[c];
    }
  }
  // epilogue: thread j < M*CPG of the group owns (row r, column c); its bias / residual are loaded before the weight
  // stream, not after the reduction (one dependent memory round trip less)
  const int r = j / CPG, c = j % CPG;
  const int64_t n = col0 + c;
  const bool own = j < p.M * CPG && n < p.N;
  float e_bias = 0.f, e_res = 0.f;
  if (!GEGLU && own) {
    if (p.bias) e_bias = bf2f(p.bias[n]);
    if (p.resid) e_res = bf2f(p.resid[r * p.ldr + n]);
  }
  float acc[MR][CW], ss[MR];
  gemv_body<MR, CW, TPG>(p, wrow, wok, j, acc, ss);
  const bool nrm = p.nw != nullptr;
  gemv_reduce<MR, CW, TPG>(acc, ss, red, fin, nrm);
  if (!own) return;
  const float* gr = fin + g * NV;
  float scale = p.alpha;
  if (nrm) scale *= rsqrtf(gr[MR * CW + r] / (float)p.K + p.neps);
  float x = gr[r * CW + c] * scale;
  if (GEGLU) {
    const float u = gr[r * CW + CPG + c] * scale;
    if (p.aux) {
      p.aux[r * p.ldaux + n] = f2bf(x);
      p.aux[r * p.ldaux + p.N + n] = f2bf(u);
    }
    x = gelu_tanh(x) * u;
  } else {
    if (p.bias) x += e_bias;
    if (p.epi == PZ_EPI_GELU || p.epi == PZ_EPI_SILU) {
      if (p.aux) p.aux[r * p.ldaux + n] = f2bf(x);
      x = p.epi == PZ_EPI_GELU ? gelu_tanh(x) : silu(x);
    }
    if (p.resid) x += e_res;
  }
  if (p.c_fp32) {
    float* C = reinterpret_cast<float*>(p.y) + r * p.ldy + n;
    *C = p.beta ? *C + x : x;
  } else {
    bf16_t* C = reinterpret_cast<bf16_t*>(p.y) + r * p.ldy + n;
    *C = f2bf(p.beta ? bf2f(*C) + x : x);
  }
}

// q|k|v projection + RoPE + scatter: a group owns PPG rotation pairs (column i and i + hd/2 of one head
// of the (nh + 2) heads: nh query heads, one key head, one value head -- MQA, bridge.yaml:176)
template <int MR, int PPG, int TPG>
__global__ void __launch_bounds__(256) gemv_qkv_rope_kernel(GemvP p) {
  constexpr int GPB = 256 / TPG;
  constexpr int CW = 2 * PPG;
  constexpr int NV = MR * CW + MR;
  __shared__ __attribute__((aligned(16))) float red[NV * 256];
  __shared__ float fin[GPB * NV];
  const int g = threadIdx.x / TPG, j = threadIdx.x % TPG;
  const int half = (int)(p.hd / 2);
  const int64_t pair0 = ((int64_t)blockIdx.x * GPB + g) * PPG;
  const int64_t npairs = p.N / 2;
  int64_t wrow[CW];
  bool wok[CW];
#pragma unroll
  for (int c = 0; c < PPG; ++c) {
    const int64_t pr = pair0 + c;
    const int64_t h = pr / half, i = pr % half;
    wrow[c] = h * p.hd + i;
    wrow[PPG + c] = h * p.hd + i + half;
    wok[c] = wok[PPG + c] = pr < npairs;
  }
  // the owner of (row r, pair c) reads its position before the weight stream and its (cos, sin) right after it, both
  // off the epilogue's critical path (they were two dependent round trips after the reduction)
  const int r = j / PPG, c = j % PPG;
  const int64_t pr = pair0 + c;
  const bool own = j < p.M * PPG && pr < npairs;
  const int64_t h = own ? pr / half : 0, i = own ? pr % half : 0;
  const bool rot = own && h != p.nh + 1;
  const int64_t ps = rot ? p.pos[r] : 0;
  float acc[MR][CW], ss[MR];
  gemv_body<MR, CW, TPG>(p, wrow, wok, j, acc, ss);
  float co = 0.f, si = 0.f;
  if (rot) {
    const float* cs = p.cs + ps * p.hd;
    co = cs[2 * i];
    si = cs[2 * i + 1];
  }
  const bool nrm = p.nw != nullptr;
  gemv_reduce<MR, CW, TPG>(acc, ss, red, fin, nrm);
  if (!own) return;
  const float* gr = fin + g * NV;
  float scale = 1.f;
  if (nrm) scale = rsqrtf(gr[MR * CW + r] / (float)p.K + p.neps);
  // the unfused path rounds the projection to bf16 before rotating: do the same
  const float y1 = bf2f(f2bf(gr[r * CW + c] * scale)), y2 = bf2f(f2bf(gr[r * CW + PPG + c] * scale));
  const int64_t b = r / p.T, t = r % p.T;
  if (h == p.nh + 1) {  // value head: no rotation
    bf16_t* dv = p.v + (b * p.Lk + p.koff + t) * p.hd;
    dv[i] = f2bf(y1);
    dv[i + half] = f2bf(y2);
    return;
  }
  float o1, o2;
  rope_pair(y1, y2, co, si, o1, o2);
  bf16_t* d = h < p.nh ? p.q + (b * p.Lq + p.qoff + t) * (p.nh * p.hd) + h * p.hd
                       : p.k + (b * p.Lk + p.koff + t) * p.hd;
  d[i] = f2bf(o1);
  d[i + half] = f2bf(o2);
}

template <int MR, int CPG, bool GEGLU>
int launch_gemv(const GemvP& p, hipStream_t st) {
  const int64_t KC = p.K / 8;
  if (KC >= 256) {
    hipLaunchKernelGGL((gemv_kernel<MR, CPG, 256, GEGLU>), dim3((unsigned)((p.N + CPG - 1) / CPG)), dim3(256), 0, st, p);
  } else if (KC >= 128) {
    hipLaunchKernelGGL((gemv_kernel<MR, CPG, 128, GEGLU>), dim3((unsigned)((p.N + 2 * CPG - 1) / (2 * CPG))), dim3(256), 0,
                       st, p);
  } else {
    hipLaunchKernelGGL((gemv_kernel<MR, CPG, 64, GEGLU>), dim3((unsigned)((p.N + 4 * CPG - 1) / (4 * CPG))), dim3(256), 0,
                       st, p);
  }
  PZ_CHECK_LAUNCH();
  return PZ_OK;
}

}  // namespace

// shape/epilogue support of the GEMV path (the planner in pz_gemm.hip asks before choosing it)
bool pz_gemv_supported(const pz_gemm_args* a) {
  if (a->M < 1 || a->M > 8 || a->batch != 1 || !a->a_kcontig || !a->b_kcontig || a->fp8_mode) return false;
  if (a->K % 512 != 0 || a->epilogue > PZ_EPI_SILU) return false;
  if (a->epilogue == PZ_EPI_GEGLU && a->bias) return false;
  if (!PZ_ALIGNED(a->A, 16) || !PZ_ALIGNED(a->B, 16) || a->lda % 8 || a->ldb % 8) return false;
  if (a->norm_w && !PZ_ALIGNED(a->norm_w, 16)) return false;
  return getenv("PZ_GEMV") == nullptr || getenv("PZ_GEMV")[0] != '0';
}

int pz_gemv_launch(const pz_gemm_args* a, hipStream_t st) {
  GemvP p{};
  p.x = (const bf16_t*)a->A;
  p.ldx = a->lda;
  p.W = (const bf16_t*)a->B;
  p.ldw = a->ldb;
  p.M = a->M;
  p.K = a->K;
  const bool geglu = a->epilogue == PZ_EPI_GEGLU;
  p.N = geglu ? a->geglu_inter : a->N;
  p.y = a->C;
  p.ldy = a->ldc;
  p.c_fp32 = a->c_fp32;
  p.beta = a->beta_accum;
  p.epi = a->epilogue;
  p.alpha = a->alpha;
  p.bias = (const bf16_t*)a->bias;
  p.resid = (const bf16_t*)a->resid;
  p.ldr = a->ld_resid;
  p.aux = (bf16_t*)a->aux;
  p.ldaux = a->ld_aux;
  p.nw = (const bf16_t*)a->norm_w;
  p.neps = a->norm_eps;
  // columns per group: >= 256 workgroups for the Pi0 widths (N = 1024: 4 -> 256; GeGLU I = 4096: 4 -> 512)
  if (a->M <= 4) {
    if (geglu) return launch_gemv<4, 4, true>(p, st);
    if (p.N <= 1024) return launch_gemv<4, 4, false>(p, st);
    return launch_gemv<4, 8, false>(p, st);
  }
  if (geglu) return launch_gemv<8, 4, true>(p, st);
  if (p.N <= 1024) return launch_gemv<8, 4, false>(p, st);
  return launch_gemv<8, 8, false>(p, st);
}

extern "C" int pz_gemv_qkv_rope(const pz_qkv_rope_args* a, void* stream) {
  PZ_CHECK_ARG(a && a->x && a->W && a->pos && a->cs && a->k_out && a->v_out && a->M >= 1 && a->M <= 8,
               "gemv_qkv_rope: bad args (M <= 8)");
  PZ_CHECK_ARG(!a->w_fp8, "gemv_qkv_rope: bf16 weights only");
  PZ_CHECK_ARG(a->K % 512 == 0 && a->hd % 2 == 0 && a->N == (a->nh + 2) * a->hd && a->T > 0 && a->M % a->T == 0,
               "gemv_qkv_rope: bad shape");
  PZ_CHECK_ARG(PZ_ALIGNED(a->x, 16) && PZ_ALIGNED(a->W, 16) && a->ldx % 8 == 0 && a->ldw % 8 == 0 &&
                   (!a->norm_w || PZ_ALIGNED(a->norm_w, 16)),
               "gemv_qkv_rope: 16-byte alignment");
  PZ_CHECK_ARG(a->q_out || a->nh == 0, "gemv_qkv_rope: q_out");
  GemvP p{};
  p.x = (const bf16_t*)a->x;
  p.ldx = a->ldx;
  p.W = (const bf16_t*)a->W;
  p.ldw = a->ldw;
  p.M = a->M;
  p.N = a->N;
  p.K = a->K;
  p.nw = (const bf16_t*)a->norm_w;
  p.neps = a->norm_eps;
  p.pos = a->pos;
  p.cs = a->cs;
  p.q = (bf16_t*)a->q_out;
  p.k = (bf16_t*)a->k_out;
  p.v = (bf16_t*)a->v_out;
  p.T = a->T;
  p.nh = a->nh;
  p.hd = a->hd;
  p.Lq = a->Lq;
  p.qoff = a->qoff;
  p.Lk = a->Lk;
  p.koff = a->koff;
  hipStream_t st = (hipStream_t)stream;
  const int64_t pairs = a->N / 2, KC = a->K / 8;
  // 2 pairs per group: N = 2560 -> 1280 pairs -> 320 workgroups at K = 1024 (2 groups of 128 threads)
  constexpr int PPG = 2;
  if (a->M <= 4) {
    if (KC >= 256)
      hipLaunchKernelGGL((gemv_qkv_rope_kernel<4, PPG, 256>), dim3((unsigned)((pairs + PPG - 1) / PPG)), dim3(256), 0,
                         st, p);
    else
      hipLaunchKernelGGL((gemv_qkv_rope_kernel<4, PPG, 128>), dim3((unsigned)((pairs + 2 * PPG - 1) / (2 * PPG))),
                         dim3(256), 0, st, p);
  } else {
    if (KC >= 256)
      hipLaunchKernelGGL((gemv_qkv_rope_kernel<8, PPG, 256>), dim3((unsigned)((pairs + PPG - 1) / PPG)), dim3(256), 0,
                         st, p);
    else
      hipLaunchKernelGGL((gemv_qkv_rope_kernel<8, PPG, 128>), dim3((unsigned)((pairs + 2 * PPG - 1) / (2 * PPG))),
                         dim3(256), 0, st, p);
  }
  PZ_CHECK_LAUNCH();
  return PZ_OK;
}
