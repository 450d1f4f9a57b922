// Decode-shaped joint attention for the denoise steps (pizero.py:461-481 with joint_model.py:130-304):
// the H action tokens of one sample x nh query heads (MQA: one K/V head of 256 shared by all heads,
// so every (token, head) is a query row of the same keys) against every cached key (vlm + proprio +
// the action tokens themselves).
//
// Two launches, each short and wide:
//   decode_attn_mfma: one workgroup per (group of 32-key chunks, 32-row tile) of one sample (C4: one row
//     tile holds all 4 tokens x 8 heads; C5's chunk of 50 tokens = 13 row tiles), S^T and P.V on the MFMA
//     with an online softmax over the group's chunks, fp32 (O, m, l) partials to the caller's workspace
//     (one group: O written directly, no second launch);
//   decode_attn_combine: one workgroup per query row merges the groups' (m, l, O) in fixed order.
// The K/V cache of a sample is read once (spread over nk/32 workgroups) instead of once per head.
// Deterministic (no atomics).
#include <stdlib.h>
#include <string.h>

#include "pz_common.h"

namespace {

constexpr int DA_KC = 32;    // keys per chunk (workgroup)
constexpr int DA_R = 32;     // query rows per row tile (tokens x heads)
constexpr int DA_RMAX = 1024;  // query rows per sample
constexpr int DA_HD = 256;   // head dim (Gemma)
constexpr int DA_RS = DA_HD + 4;  // workspace row: O[256], m, l (16-byte aligned rows)

__device__ __forceinline__ bool da_allowed(int t, int j, int nk, int cnt, int P, int C) {
  if (j >= nk) return false;
  if (t < P) return t < cnt && j < cnt;
  if (t < P + C) return j < cnt || (j >= P && j < P + C);
  return j < cnt || j >= P;
}

// grid (R, B), 256 threads: thread = head dim; merges the chunks in order 0..nchunks-1
__global__ void __launch_bounds__(256) decode_attn_combine(pz_decode_attn_args a, int nchunks) {
  const int r = blockIdx.x, b = blockIdx.y, d = threadIdx.x;
  const int nh = (int)a.nh, t = r / nh, h = r % nh;
  const int Rpad = ((int)(a.T * a.nh) + DA_R - 1) / DA_R * DA_R;
  const int64_t cs = (int64_t)Rpad * DA_RS;  // chunk stride
  const float* ws = a.ws + (int64_t)b * nchunks * cs + r * DA_RS;
  // batches of 16 chunks: every (m, l, O[d]) load of a batch issued before any is consumed (the merge
  // is a chain of tiny dependent loads otherwise); running max / rescale across batches, fixed order
  constexpr int CB = 16;
  float M = -INFINITY, o = 0.f, l = 0.f;
  for (int c0 = 0; c0 < nchunks; c0 += CB) {
    float mv[CB], lv[CB], ov[CB];
#pragma unroll
    for (int u = 0; u < CB; ++u) {
      const bool ok = c0 + u < nchunks;
      const float* w = ws + (int64_t)(ok ? c0 + u : 0) * cs;
      mv[u] = ok ? w[DA_HD] : -INFINITY;
      lv[u] = ok ? w[DA_HD + 1] : 0.f;
      ov[u] = ok ? w[d] : 0.f;
    }
    float Mn = M;
#pragma unroll
    for (int u = 0; u < CB; ++u) Mn = fmaxf(Mn, mv[u]);
    const float sc = M == -INFINITY ? 0.f : __expf(M - Mn);
    o *= sc;
    l *= sc;
#pragma unroll
    for (int u = 0; u < CB; ++u) {
      const float s = mv[u] == -INFINITY ? 0.f : __expf(mv[u] - Mn);
      o += s * ov[u];
      l += s * lv[u];
    }
    M = Mn;
  }
  bf16_t* out = (bf16_t*)a.o + ((int64_t)b * a.T + t) * a.ldo + (int64_t)h * DA_HD + d;
  *out = f2bf(l > 0.f ? o / l : 0.f);
}

// ---- MFMA decode attention (default): P.V on the matrix cores --------------------------------------------
// grid (ngroups, B * rtiles), 256 threads: workgroup = (group of nch consecutive 32-key chunks, sample b, 32-row
// tile) with an online softmax over its chunks; ngroups == 1 writes O itself (no merge launch), otherwise fp32
// (O, m, l) partials (workspace rows [b][group][Rpad][DA_RS], Rpad = 32 * rtiles) for decode_attn_combine.  Per chunk: V(c) staged
// into an LDS image read transposed (ds_read_b64_tr_b16), S^T = K Q^T on the MFMA (K fragments straight from
// global), soft-cap + block mask into LDS, the softmax of each row by 8 lanes (4 keys each, shuffle max / sum,
// online (m, l) kept in all 8 lanes), bf16 P, and O^T += V^T P^T on the MFMA (16 per chunk instead of the VALU
// kernel's 1024 FMAs per thread); chunk c + 1's K fragments and V rows are loaded during chunk c.
__device__ __forceinline__ int da_sw(int k) { return ((k & 3) | (((k >> 3) & 1) << 2)) << 2; }

// A fragment of the MFMA from the k-strided [32 key][256 dim] V image: rows (dims) 16 * dt .. + 15, k = keys
// 8 (lane >> 4) .. + 7 (the transposed-read layout of pz_gemm.hip's k-strided operands)
__device__ __forceinline__ bf16x8 da_vfrag(const char* img, int dt, int lane) {
  const int q = (lane & 15) >> 2, p = lane & 3;
  s16x8 out;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int k = 8 * (lane >> 4) + 4 * t + q;
    const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) s16x4*)(img + k * 512 + (((4 * dt + p) ^ da_sw(k)) << 3)));
    out[4 * t + 0] = v[0];
    out[4 * t + 1] = v[1];
    out[4 * t + 2] = v[2];
    out[4 * t + 3] = v[3];
  }
  return __builtin_bit_cast(bf16x8, out);
}

__global__ void __launch_bounds__(256) decode_attn_mfma(pz_decode_attn_args a, int nch) {
  __shared__ float S[DA_R][DA_KC + 1];
  __shared__ __attribute__((aligned(16))) bf16_t Pm[DA_R][DA_KC + 8];  // bf16 probabilities [row][key]
  __shared__ __attribute__((aligned(16))) char Vimg[DA_KC * 512];       // one chunk of V, transposed reads
  __shared__ float alpha_s[DA_R];
  __shared__ float ml_s[DA_R][2];  // final (m, l) per row
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int T = (int)a.T, nh = (int)a.nh, nk = (int)a.nk, R = T * nh;
  const int rtiles = (R + DA_R - 1) / DA_R, Rpad = rtiles * DA_R;
  const int grp = blockIdx.x, b = blockIdx.y / rtiles, rt = blockIdx.y % rtiles, r0 = rt * DA_R;
  const bool masked = a.cnt != nullptr;
  const int cnt = masked ? a.cnt[b] : nk;
  const bf16_t* K = (const bf16_t*)a.k + (int64_t)b * a.k_bstride;
  const bf16_t* V = (const bf16_t*)a.v + (int64_t)b * a.v_bstride;
  const int nchunks = (nk + DA_KC - 1) / DA_KC;
  const int c0 = grp * nch, c1 = min(nchunks, c0 + nch);
  const int g = lane >> 4;
  // S^T tile of this wave: key tile kt (16 keys) x row block rb (16 rows)
  const int kt = wave & 1, rb = wave >> 1;
  const int row = r0 + rb * 16 + (lane & 15);
  const bool rok = row < R;
  const int t = rok ? row / nh : 0, h = rok ? row % nh : 0;
  const int qt = (int)a.qtok0 + t;
  bf16x8 qf[8];
  {
    const bf16_t* qp = (const bf16_t*)a.q + ((int64_t)b * a.Lq + a.qoff + t) * a.ldq + (int64_t)h * DA_HD + 8 * g;
#pragma unroll
    for (int dc = 0; dc < 8; ++dc) qf[dc] = rok ? *reinterpret_cast<const bf16x8*>(qp + dc * 32) : bf16x8{};
  }
  auto load_k = [&](int c, bf16x8 (&kf)[8]) {
    const int key = min(c * DA_KC + kt * 16 + (lane & 15), nk - 1);
    const bf16_t* kp = K + (int64_t)key * DA_HD + 8 * g;
#pragma unroll
    for (int dc = 0; dc < 8; ++dc) kf[dc] = *reinterpret_cast<const bf16x8*>(kp + dc * 32);
  };
  // V staging: thread = 4 (key, 16-B dim chunk) pairs of the 32 x 32 chunks
  auto load_v = [&](int c, u32x4 (&vv)[4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int e = threadIdx.x + i * 256, kr = e >> 5, ch = e & 31;
      vv[i] = *reinterpret_cast<const u32x4*>(V + (int64_t)min(c * DA_KC + kr, nk - 1) * DA_HD + 8 * ch);
    }
  };
  const float inv_cap = a.cap > 0.f ? 1.f / a.cap : 0.f;
  f32x4 acc[4][2];  // O^T tiles: dim tile 4 * wave + i, row tile j (lane: dims 4 (lane >> 4) .. + 3, row lane & 15)
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // softmax ownership: row sr = threadIdx.x >> 3, keys 4 sq .. 4 sq + 3; (m, l) replicated in the row's 8 lanes
  const int sr = threadIdx.x >> 3, sq = threadIdx.x & 7;
  float m_run = -INFINITY, l_run = 0.f;
  bf16x8 kf[8], kn[8];
  u32x4 vv[4], vn[4];
  if (c0 < c1) {
    load_k(c0, kf);
    load_v(c0, vv);
  }
  for (int c = c0; c < c1; ++c) {
    const int j0 = c * DA_KC;
    // V(c) -> LDS image (the previous chunk's P.V reads ended at the loop-closing barrier)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int e = threadIdx.x + i * 256, kr = e >> 5, ch = e & 31;
      *reinterpret_cast<u32x4*>(Vimg + kr * 512 + (((2 * ch) ^ da_sw(kr)) << 3)) = vv[i];
    }
    {  // S^T tile
      f32x4 sv = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int dc = 0; dc < 8; ++dc) sv = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf[dc], qf[dc], sv, 0, 0, 0);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int kl = kt * 16 + 4 * g + e;
        float x = sv[e] * a.scale;
        if (a.cap > 0.f) x = a.cap * tanh_fast(x * inv_cap);
        const bool ok = rok && (masked ? da_allowed(qt, j0 + kl, nk, cnt, (int)a.prefix, (int)a.cond) : j0 + kl < nk);
        S[row - r0][kl] = ok ? x : -INFINITY;
      }
    }
    if (c + 1 < c1) {  // next chunk's K fragments and V rows in flight during this chunk's softmax / P.V
      load_k(c + 1, kn);
      load_v(c + 1, vn);
    }
    __syncthreads();
    {  // online softmax: 8 lanes per row
      float x[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) x[i] = S[sr][4 * sq + i];
      float m = fmaxf(fmaxf(x[0], x[1]), fmaxf(x[2], x[3]));
#pragma unroll
      for (int o = 1; o < 8; o <<= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
      m = fmaxf(m, m_run);
      const float al = m_run == -INFINITY ? 0.f : __expf(m_run - m);
      float p[4], l = 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        p[i] = m == -INFINITY ? 0.f : __expf(x[i] - m);
        l += p[i];
      }
#pragma unroll
      for (int o = 1; o < 8; o <<= 1) l += __shfl_xor(l, o, 64);
      l_run = l_run * al + l;
      m_run = m;
      *reinterpret_cast<u32x2*>(&Pm[sr][4 * sq]) = u32x2{pack2bf(p[0], p[1]), pack2bf(p[2], p[3])};
      if (sq == 0) alpha_s[sr] = al;
    }
    __syncthreads();
    {  // O^T += V^T P^T (rows rescaled by alpha first)
      bf16x8 pb[2];
#pragma unroll
      for (int j = 0; j < 2; ++j) pb[j] = *reinterpret_cast<const bf16x8*>(&Pm[j * 16 + (lane & 15)][8 * g]);
      const float al0 = alpha_s[lane & 15], al1 = alpha_s[16 + (lane & 15)];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const bf16x8 vf = da_vfrag(Vimg, 4 * wave + i, lane);
        acc[i][0] *= al0;
        acc[i][1] *= al1;
        acc[i][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pb[0], acc[i][0], 0, 0, 0);
        acc[i][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pb[1], acc[i][1], 0, 0, 0);
      }
    }
#pragma unroll
    for (int dc = 0; dc < 8; ++dc) kf[dc] = kn[dc];
#pragma unroll
    for (int i = 0; i < 4; ++i) vv[i] = vn[i];
    __syncthreads();  // S, P, alpha and the V image are rewritten by the next chunk
  }
  if (sq == 0) {
    ml_s[sr][0] = m_run;
    ml_s[sr][1] = l_run;
  }
  __syncthreads();
  const bool direct = gridDim.x == 1;
  float* ws = direct ? nullptr : a.ws + (((int64_t)b * gridDim.x + grp) * Rpad + r0) * DA_RS;
  if (!direct && threadIdx.x < DA_R) {
    ws[threadIdx.x * DA_RS + DA_HD] = ml_s[threadIdx.x][0];
    ws[threadIdx.x * DA_RS + DA_HD + 1] = ml_s[threadIdx.x][1];
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int rl = j * 16 + (lane & 15), rr = r0 + rl;
    if (rr >= R) continue;
    if (direct) {
      const float l = ml_s[rl][1], il = l > 0.f ? 1.f / l : 0.f;
      const int tt = rr / nh, hh = rr % nh;
      bf16_t* out = (bf16_t*)a.o + ((int64_t)b * a.T + tt) * a.ldo + (int64_t)hh * DA_HD;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int d0 = (4 * wave + i) * 16 + 4 * g;
        *reinterpret_cast<u32x2*>(out + d0) =
            u32x2{pack2bf(acc[i][j][0] * il, acc[i][j][1] * il), pack2bf(acc[i][j][2] * il, acc[i][j][3] * il)};
      }
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int d0 = (4 * wave + i) * 16 + 4 * g;
        *reinterpret_cast<f32x4*>(ws + rl * DA_RS + d0) = acc[i][j];
      }
    }
  }
}

}  // namespace

extern "C" int64_t pz_decode_attn_ws_bytes(int64_t B, int64_t rows, int64_t nk) {
  const int64_t rpad = (rows + DA_R - 1) / DA_R * DA_R;
  return B * ((nk + DA_KC - 1) / DA_KC) * rpad * DA_RS * (int64_t)sizeof(float);
}

extern "C" int pz_decode_attn(const pz_decode_attn_args* a, void* stream) {
  PZ_CHECK_ARG(a && a->q && a->k && a->v && a->o && a->ws && a->B > 0 && a->nh > 0, "decode_attn: bad args");
  PZ_CHECK_ARG(a->head_dim == DA_HD && a->T >= 1 && a->T * a->nh <= DA_RMAX && a->nk >= 1,
               "decode_attn: head_dim 256 and tokens x heads <= 1024 query rows per sample");
  PZ_CHECK_ARG(a->ws_bytes >= pz_decode_attn_ws_bytes(a->B, a->T * a->nh, a->nk), "decode_attn: workspace too small");
  PZ_CHECK_ARG(PZ_ALIGNED(a->q, 16) && PZ_ALIGNED(a->k, 16) && PZ_ALIGNED(a->v, 16) && PZ_ALIGNED(a->o, 2) &&
                   PZ_ALIGNED(a->ws, 16) && a->ldq % 8 == 0 && a->k_bstride % 8 == 0 && a->v_bstride % 8 == 0,
               "decode_attn: alignment");
  const int nchunks = (int)((a->nk + DA_KC - 1) / DA_KC);
  hipStream_t st = (hipStream_t)stream;
  const int64_t rtiles = (a->T * a->nh + DA_R - 1) / DA_R;
  PZ_CHECK_ARG(a->B * rtiles < 65536, "decode_attn: grid too large");
  // chunks per workgroup: one (C4: 9 workgroups) until the (chunk, row tile) grid passes 256 workgroups,
  // then groups of nch chunks (fewer partial rows for the merge).  One workgroup walking every chunk (no merge
  // launch) measured slower for C4: 15.21 vs 12.81 ms per chunk (profiles/r03/decode_grouping_ab.txt)
  const int64_t wg1 = (int64_t)nchunks * a->B * rtiles;
  const char* e = getenv("PZ_DECODE_WG");  // target workgroups (A/B; read per call)
  const int64_t target = e && atoll(e) > 0 ? atoll(e) : 256;
  int nch = (int)((wg1 + target - 1) / target);
  int ngroups = (nchunks + nch - 1) / nch;
  const bool o_vec = PZ_ALIGNED(a->o, 8) && a->ldo % 4 == 0;
  if (ngroups == 1 && !o_vec) {  // the direct-O path stores 8 B per lane
    PZ_CHECK_ARG(nchunks > 1, "decode_attn: a single key chunk needs an aligned O (8 B, ldo %% 4 == 0)");
    nch = (nchunks + 1) / 2;
    ngroups = (nchunks + nch - 1) / nch;
  }
  hipLaunchKernelGGL(decode_attn_mfma, dim3((unsigned)ngroups, (unsigned)(a->B * rtiles)), dim3(256), 0, st, *a, nch);
  PZ_CHECK_LAUNCH();
  if (ngroups == 1) return PZ_OK;  // the kernel wrote O
  hipLaunchKernelGGL(decode_attn_combine, dim3((unsigned)(a->T * a->nh), (unsigned)a->B), dim3(256), 0, st, *a,
                     ngroups);
  PZ_CHECK_LAUNCH();
  return PZ_OK;
}
