// Fused (flash) attention for the two attention shapes of the Pi0 path, forward and backward:
//
//   * SigLIP self-attention (siglip.py:108-166): 16 heads x 72, 256 tokens, no mask, fp32 softmax;
//     Q/K/V read in place from the fused q|k|v projection output, O written in place for out_proj.
//   * the joint mixture attention (joint_model.py:130-304): MQA with ONE shared K/V head of 256 and
//     the 8 query heads stacked as rows (row r = token * 8 + head, no repeat_kv copy), Gemma
//     soft-cap 50*tanh(s/50) (joint_model.py:265-268) and the Pi0 block mask regenerated from the
//     per-sample prefix count (pizero.py:271-306); O rows are scattered straight into the per-
//     mixture buffers that feed each mixture's o_proj.
//
// Nothing of size L x L touches HBM: the forward keeps S/P in registers and saves one fp32
// log-sum-exp per query row; the backward recomputes P from it.  K/V (forward) and Q/dO
// (backward) tiles are staged in LDS; MFMA v_mfma_f32_16x16x32_bf16 throughout.
//
// Orientation (per wave, 64-lane wave64): the forward computes S^T = K Q^T so each lane owns one
// query column and 4 consecutive keys per 16x16 block; P^T then feeds O^T = V^T P^T directly as the
// B operand (no LDS round trip), with the MFMA k order permuted to keys {4g..4g+3, 16+4g..16+4g+3}
// for lane group g and the matching V^T fragment fetched by two ds_read_b64_tr_b16 (4 keys each).
// The backward mirrors it with S = Q K^T (key on the lane), so dV^T = dO^T P and dK^T = Q^T dS take
// P / dS from registers and dO^T / Q^T through transposed LDS reads; dQ = dS K is a separate
// query-parallel pass (no atomics: deterministic).
#include "pz_common.h"

#include <type_traits>

namespace {

constexpr int FA_KB = 64;   // keys per staged block (forward, dQ) / per dK-dV workgroup
constexpr int FA_NW = 4;    // waves per workgroup (backward)
constexpr int FA_QS = 32;   // query rows per staged step of the dK/dV pass

template <int HD>
struct FaDims {
  static constexpr int HDK = (HD + 31) / 32 * 32;  // contraction over head_dim, in 32-steps
  static constexpr int HDV = (HD + 15) / 16 * 16;  // head_dim as 16-wide output blocks
  static constexpr int NKS = HDK / 32;
  static constexpr int NDB = HDV / 16;
  // LDS row stride (elements): >= HDK, 16-B rows, and chosen so the 4 rows of a transposed read
  // land on disjoint banks (HD 256: 272 = 136 dwords = 8 mod 64; HD 72: 112; small test heads: HDK + 16)
  static constexpr int ROW = HD == 256 ? 272 : (HD == 72 ? 112 : HDK + 16);
  // forward geometry: 128 query rows per workgroup; HD 256 keeps one 16-row block per wave (8 waves,
  // <= 256 registers so two workgroups share a CU and one stages while the other computes)
  static constexpr int FNW = HD == 256 ? 8 : 4;
  static constexpr int FNQB = HD == 256 ? 1 : 2;
};

__device__ __forceinline__ bool fa_allowed(int64_t i, int64_t j, int64_t cnt, int64_t P, int64_t C) {
  if (i < P) return i < cnt && j < cnt;
  if (i < P + C) return j < cnt || (j >= P && j < P + C);
  return j < cnt || j >= P;
}

__device__ __forceinline__ s16x4 lds_tr4(const bf16_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p));
}

// V^T / dO^T / Q^T fragment for MFMA A (m = column c0 + (lane & 15), k-slot 8g + e) taken from a
// row-major LDS tile T[row][col]: k-slots 0..3 <- rows r0 + 4g + e, 4..7 <- rows r0 + 16 + 4g + e.
template <int ROW>
__device__ __forceinline__ bf16x8 frag_tr(const bf16_t* T, int r0, int c0, int lane) {
  const int g = lane >> 4, w = lane & 15, q = w >> 2, p = w & 3;
  const s16x4 a = lds_tr4(T + (r0 + 4 * g + q) * ROW + c0 + 4 * p);
  const s16x4 b = lds_tr4(T + (r0 + 16 + 4 * g + q) * ROW + c0 + 4 * p);
  s16x8 o;
  o[0] = a[0]; o[1] = a[1]; o[2] = a[2]; o[3] = a[3];
  o[4] = b[0]; o[5] = b[1]; o[6] = b[2]; o[7] = b[3];
  return __builtin_bit_cast(bf16x8, o);
}

// row fragment (MFMA A with m = row, or B with n = row): T[r0 + (lane & 15)][c0 + 8g .. +7]
template <int ROW>
__device__ __forceinline__ bf16x8 frag_row(const bf16_t* T, int r0, int c0, int lane) {
  return *reinterpret_cast<const bf16x8*>(T + (r0 + (lane & 15)) * ROW + c0 + 8 * (lane >> 4));
}

__device__ __forceinline__ bf16x8 pack8(const f32x4& a, const f32x4& b) {
  s16x8 o;
  const unsigned u0 = pack2bf(a[0], a[1]), u1 = pack2bf(a[2], a[3]);
  const unsigned u2 = pack2bf(b[0], b[1]), u3 = pack2bf(b[2], b[3]);
  o[0] = (short)(u0 & 0xffff); o[1] = (short)(u0 >> 16); o[2] = (short)(u1 & 0xffff); o[3] = (short)(u1 >> 16);
  o[4] = (short)(u2 & 0xffff); o[5] = (short)(u2 >> 16); o[6] = (short)(u3 & 0xffff); o[7] = (short)(u3 >> 16);
  return __builtin_bit_cast(bf16x8, o);
}

__device__ __forceinline__ f32x4 mfma(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// Register-staged prefetch of a ROWS x HD tile: load() issues the global loads of the NEXT tile
// before the current tile's MFMAs, store() writes them to the other LDS buffer afterwards, so the
// HBM/L2 latency hides behind the compute (one barrier per step).
template <int HD, int ROW, int ROWS, int NT>
struct TileStager {
  static constexpr int CH = HD / 8, TOT = ROWS * CH, PER = (TOT + NT - 1) / NT;
  u32x4 v[PER];
  __device__ __forceinline__ void load(const bf16_t* src, int64_t ld, int64_t j0, int64_t n) {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = threadIdx.x + i * NT, r = c / CH, ch = c % CH;
      v[i] = u32x4{0u, 0u, 0u, 0u};
      if (c < TOT && j0 + r < n) v[i] = *reinterpret_cast<const u32x4*>(src + (j0 + r) * ld + ch * 8);
    }
  }
  // query-side rows [r0, r0 + ROWS) of Q (q strides) or dO (output-group layout)
  __device__ __forceinline__ void load_q(const pz_flash_args& a, const bf16_t* Q, int64_t b, int64_t h, int64_t r0,
                                         bool is_do);
  __device__ __forceinline__ void store(bf16_t* T) const {
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = threadIdx.x + i * NT, r = c / CH, ch = c % CH;
      if (c < TOT) *reinterpret_cast<u32x4*>(T + r * ROW + ch * 8) = v[i];
    }
  }
};

// zero the padding columns [HD, PADTO) of a staged tile once (loads never write them)
template <int HD, int PADTO, int ROW, int ROWS, int NT>
__device__ __forceinline__ void zero_pad_cols(bf16_t* T) {
  if constexpr (PADTO > HD) {
    constexpr int CH = (PADTO - HD) / 8;
    for (int c = threadIdx.x; c < ROWS * CH; c += NT) {
      const int r = c / CH, ch = c % CH;
      *reinterpret_cast<u32x4*>(T + r * ROW + HD + ch * 8) = u32x4{0u, 0u, 0u, 0u};
    }
  }
}

struct FaRow {  // where O / dO row r of unit (b, h) lives
  const pz_flash_args* a;
  __device__ __forceinline__ int grp(int64_t r) const {
    int gi = 0;
    for (int i = 1; i < a->n_groups; ++i)
      if (r >= a->g_row0[i]) gi = i;
    return gi;
  }
  __device__ __forceinline__ int64_t off(int64_t b, int64_t h, int64_t r, int gi) const {
    return b * a->g_bstride[gi] + (r - a->g_row0[gi]) * a->g_ld[gi] + h * a->o_hstride;
  }
};

template <int HD, int ROW, int ROWS, int NT>
__device__ __forceinline__ void TileStager<HD, ROW, ROWS, NT>::load_q(const pz_flash_args& a, const bf16_t* Q,
                                                                      int64_t b, int64_t h, int64_t r0, bool is_do) {
  const FaRow fr{&a};
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int c = threadIdx.x + i * NT, rr = c / CH, ch = c % CH;
    const int64_t r = r0 + rr;
    v[i] = u32x4{0u, 0u, 0u, 0u};
    if (c < TOT && r < a.nq) {
      const bf16_t* src;
      if (is_do) {
        const int gi = fr.grp(r);
        src = (const bf16_t*)a.g_do[gi] + fr.off(b, h, r, gi);
      } else {
        src = Q + r * a.ldq;
      }
      v[i] = *reinterpret_cast<const u32x4*>(src + ch * 8);
    }
  }
}

// Mask / logit context in 32-bit registers (token of a query row by a float reciprocal: exact for
// nq < 2^22, checked on the host) -- no 64-bit division in the inner loops
struct FaMask {
  int mode, nk, P, C, cnt, row0;
  float inv_rpt, scale, cap, inv_cap;
  __device__ __forceinline__ FaMask(const pz_flash_args& a, int64_t b) {
    mode = a.mask_mode;
    nk = (int)a.nk;
    P = (int)a.prefix;
    C = (int)a.cond;
    cnt = mode == 1 ? a.cnt[b] : 0;
    inv_rpt = mode == 1 ? 1.f / (float)a.rows_per_token : 0.f;
    row0 = (int)a.mask_row0;
    scale = a.scale;
    cap = a.cap;
    inv_cap = a.cap > 0.f ? 1.f / a.cap : 0.f;
  }
  __device__ __forceinline__ int token(int r) const { return (int)(((float)(r + row0) + 0.5f) * inv_rpt); }
  __device__ __forceinline__ bool dead(int t) const { return mode == 1 && t < P && t >= cnt; }
  __device__ __forceinline__ bool allowed(int t, int j) const {
    if (j >= nk) return false;
    if (mode != 1) return true;
    if (t < P) return t < cnt && j < cnt;
    if (t < P + C) return j < cnt || (j >= P && j < P + C);
    return j < cnt || j >= P;
  }
};

// 1-D grid of nblk workgroups per unit: the nblk workgroups of one unit get ids of one residue mod 8,
// i.e. land on one XCD (blocks are dealt round-robin over the 8 XCDs) and share its L2 for the
// unit's resident operand, which every one of them stages
__device__ __forceinline__ void fa_unit_block(int nblk, int units, int64_t& zh, int& blk) {
  const int id = blockIdx.x;
  if (units % 8 == 0) {
    const int xcd = id & 7, local = id >> 3;
    zh = (int64_t)(local / nblk) * 8 + xcd;
    blk = local % nblk;
  } else {
    zh = id / nblk;
    blk = id % nblk;
  }
}

// logits with soft-cap and mask for key j of a query row of token t; dead rows (pad tokens of the
// prefix, pizero.py:291: finfo.min absorbs s) attend uniformly to every key
__device__ __forceinline__ float fa_logit(const FaMask& mk, float s, int t, int j) {
  if (j >= mk.nk) return -INFINITY;
  if (mk.dead(t)) return 0.f;
  if (!mk.allowed(t, j)) return -INFINITY;
  float x = s * mk.scale;
  if (mk.cap > 0.f) x = mk.cap * tanh_fast(x * mk.inv_cap);
  return x;
}

// ------------------------------------------------------------------ forward --
// grid (ceil(nq / 128), Z * H), FNW waves: wave w owns query rows q0 + 16*FNQB*w .. + 16*FNQB - 1
template <int HD>
__global__ void __launch_bounds__(FaDims<HD>::FNW * 64) flash_fwd_kernel(pz_flash_args a) {
  using D = FaDims<HD>;
  constexpr int NQB = D::FNQB, NT = D::FNW * 64;
  __shared__ __attribute__((aligned(16))) bf16_t Ks2[2][FA_KB * D::ROW];  // double-buffered K / V tiles
  __shared__ __attribute__((aligned(16))) bf16_t Vs2[2][FA_KB * D::ROW];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4;
  const int64_t zh = blockIdx.y, b = zh / a.H, h = zh % a.H;
  const int64_t q0 = (int64_t)blockIdx.x * (D::FNW * 16 * NQB) + wave * 16 * NQB;
  const bf16_t* Q = (const bf16_t*)a.q + b * a.q_bstride + h * a.q_hstride;
  const bf16_t* K = (const bf16_t*)a.k + b * a.k_bstride + h * a.k_hstride;
  const bf16_t* V = (const bf16_t*)a.v + b * a.v_bstride + h * a.v_hstride;
  const FaMask mk(a, b);

#pragma unroll
  for (int bi = 0; bi < 2; ++bi) {
    zero_pad_cols<HD, D::HDK, D::ROW, FA_KB, NT>(Ks2[bi]);
    zero_pad_cols<HD, D::HDV, D::ROW, FA_KB, NT>(Vs2[bi]);
  }
  // key split (gridDim.z > 1, few query blocks: inference): key blocks [kb_begin, kb_end) only,
  // unnormalised O + (m, l) partials to the workspace, merged by flash_fwd_combine_kernel
  const int nkb = (int)((a.nk + FA_KB - 1) / FA_KB);
  const int per = (nkb + (int)gridDim.z - 1) / (int)gridDim.z;
  const int kb_begin = (int)blockIdx.z * per, kb_end = min(nkb, kb_begin + per);
  TileStager<HD, D::ROW, FA_KB, NT> stk, stv;
  stk.load(K, a.ldk, (int64_t)kb_begin * FA_KB, a.nk);
  stv.load(V, a.ldv, (int64_t)kb_begin * FA_KB, a.nk);

  // Q^T fragments (B operand: k = head dim, n = query) straight from HBM, zero past HD / nq
  bf16x8 qf[NQB][D::NKS];
#pragma unroll
  for (int qb = 0; qb < NQB; ++qb) {
    const int64_t r = q0 + qb * 16 + (lane & 15);
#pragma unroll
    for (int ks = 0; ks < D::NKS; ++ks) {
      const int c = ks * 32 + 8 * g;
      qf[qb][ks] = (r < a.nq && c < HD) ? *reinterpret_cast<const bf16x8*>(Q + r * a.ldq + c) : bf16x8{};
    }
  }
  f32x4 o[D::NDB][NQB];
#pragma unroll
  for (int db = 0; db < D::NDB; ++db)
#pragma unroll
    for (int qb = 0; qb < NQB; ++qb) o[db][qb] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m[NQB], l[NQB];
#pragma unroll
  for (int qb = 0; qb < NQB; ++qb) {
    m[qb] = -INFINITY;
    l[qb] = 0.f;
  }

  __syncthreads();  // pad columns zeroed
  stk.store(Ks2[0]);
  stv.store(Vs2[0]);
  __syncthreads();
  for (int kb = kb_begin; kb < kb_end; ++kb) {
    const bf16_t* Ks = Ks2[(kb - kb_begin) & 1];
    const bf16_t* Vs = Vs2[(kb - kb_begin) & 1];
    const bool more = kb + 1 < kb_end;
    if (more) {  // next K/V tile in flight during this tile's MFMAs
      stk.load(K, a.ldk, (int64_t)(kb + 1) * FA_KB, a.nk);
      stv.load(V, a.ldv, (int64_t)(kb + 1) * FA_KB, a.nk);
    }
    // S^T[key][q] for 64 keys x 16*NQB queries
    f32x4 s[4][NQB];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int qb = 0; qb < NQB; ++qb) s[i][qb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < D::NKS; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const bf16x8 kf = frag_row<D::ROW>(Ks, i * 16, ks * 32, lane);
#pragma unroll
        for (int qb = 0; qb < NQB; ++qb) s[i][qb] = mfma(kf, qf[qb][ks], s[i][qb]);
      }
    // logits, online softmax (each lane: one query column, 16 of the block's 64 keys)
    bf16x8 pf[2][NQB];  // [k-step of 32 keys][query block]
#pragma unroll
    for (int qb = 0; qb < NQB; ++qb) {
      const int t = mk.token((int)(q0 + qb * 16 + (lane & 15)));
      float mx = -INFINITY;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int j = kb * FA_KB + i * 16 + 4 * g + e;
          const float x = fa_logit(mk, s[i][qb][e], t, j);
          s[i][qb][e] = x;
          mx = fmaxf(mx, x);
        }
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float mn = fmaxf(m[qb], mx);
      const float alpha = mn == -INFINITY ? 1.f : __expf(m[qb] - mn);
      float sum = 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float p = mn == -INFINITY ? 0.f : __expf(s[i][qb][e] - mn);
          s[i][qb][e] = p;
          sum += p;
        }
      sum += __shfl_xor(sum, 16, 64);
      sum += __shfl_xor(sum, 32, 64);
      l[qb] = l[qb] * alpha + sum;
      m[qb] = mn;
#pragma unroll
      for (int db = 0; db < D::NDB; ++db) o[db][qb] *= alpha;
      pf[0][qb] = pack8(s[0][qb], s[1][qb]);
      pf[1][qb] = pack8(s[2][qb], s[3][qb]);
    }
    // O^T[d][q] += V^T[d][key] P^T[key][q]
#pragma unroll
    for (int k2 = 0; k2 < 2; ++k2)
#pragma unroll
      for (int db = 0; db < D::NDB; ++db) {
        const bf16x8 vf = frag_tr<D::ROW>(Vs, k2 * 32, db * 16, lane);
#pragma unroll
        for (int qb = 0; qb < NQB; ++qb) o[db][qb] = mfma(vf, pf[k2][qb], o[db][qb]);
      }
    if (more) {
      stk.store(Ks2[(kb + 1 - kb_begin) & 1]);
      stv.store(Vs2[(kb + 1 - kb_begin) & 1]);
    }
    __syncthreads();
  }
  if (gridDim.z > 1) {
    float* pO = (float*)a.ws;
    float* pml = pO + (int64_t)gridDim.z * gridDim.y * a.nq * HD;
#pragma unroll
    for (int qb = 0; qb < NQB; ++qb) {
      const int64_t r = q0 + qb * 16 + (lane & 15);
      if (r >= a.nq) continue;
      const int64_t row = ((int64_t)blockIdx.z * gridDim.y + zh) * a.nq + r;
#pragma unroll
      for (int db = 0; db < D::NDB; ++db) {
        const int d = db * 16 + 4 * g;
        if (d < HD) *reinterpret_cast<f32x4*>(pO + row * HD + d) = o[db][qb];
      }
      if (g == 0) {
        pml[2 * row] = m[qb];
        pml[2 * row + 1] = l[qb];
      }
    }
    return;
  }
  // O[r][d..d+3] = O^T / l; lse
  const FaRow fr{&a};
#pragma unroll
  for (int qb = 0; qb < NQB; ++qb) {
    const int64_t r = q0 + qb * 16 + (lane & 15);
    if (r >= a.nq) continue;
    const float inv = l[qb] > 0.f ? 1.f / l[qb] : 0.f;
    const int gi = fr.grp(r);
    bf16_t* O = (bf16_t*)a.g_o[gi] + fr.off(b, h, r, gi);
#pragma unroll
    for (int db = 0; db < D::NDB; ++db) {
      const int d = db * 16 + 4 * g;
      if (d < HD)
        *reinterpret_cast<u32x2*>(O + d) =
            u32x2{pack2bf(o[db][qb][0] * inv, o[db][qb][1] * inv), pack2bf(o[db][qb][2] * inv, o[db][qb][3] * inv)};
    }
    if (g == 0 && a.lse) a.lse[zh * a.nq + r] = m[qb] + __logf(l[qb]);
  }
}

// key-split merge: one thread per (unit, query row, 4 head dims); fixed split order
template <int HD>
__global__ void __launch_bounds__(256) flash_fwd_combine_kernel(pz_flash_args a, int nsp) {
  const int64_t ZH = a.Z * a.H;
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= ZH * a.nq * (HD / 4)) return;
  const int d = (int)(i % (HD / 4)) * 4;
  const int64_t zr = i / (HD / 4), r = zr % a.nq, zh = zr / a.nq;
  const float* pO = (const float*)a.ws;
  const float* pml = pO + (int64_t)nsp * ZH * a.nq * HD;
  // every split's (m, l, O[d..d+3]) loaded before any is consumed (nsp <= 16, host-checked): one round
  // of independent loads instead of a dependent chain per split
  constexpr int SMAX = 16;
  float mv[SMAX], lv[SMAX];
  f32x4 ov[SMAX];
#pragma unroll
  for (int s = 0; s < SMAX; ++s) {
    const bool ok = s < nsp;
    const int64_t row = ((int64_t)(ok ? s : 0) * ZH + zh) * a.nq + r;
    mv[s] = ok ? pml[2 * row] : -INFINITY;
    lv[s] = ok ? pml[2 * row + 1] : 0.f;
    ov[s] = ok ? *reinterpret_cast<const f32x4*>(pO + row * HD + d) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  float M = -INFINITY;
#pragma unroll
  for (int s = 0; s < SMAX; ++s) M = fmaxf(M, mv[s]);
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  float L = 0.f;
#pragma unroll
  for (int s = 0; s < SMAX; ++s) {
    const float w = mv[s] == -INFINITY ? 0.f : __expf(mv[s] - M);
    L += w * lv[s];
    acc += w * ov[s];
  }
  const float inv = L > 0.f ? 1.f / L : 0.f;
  const FaRow fr{&a};
  const int gi = fr.grp(r);
  bf16_t* O = (bf16_t*)a.g_o[gi] + fr.off(zh / a.H, zh % a.H, r, gi);
  *reinterpret_cast<u32x2*>(O + d) = u32x2{pack2bf(acc[0] * inv, acc[1] * inv), pack2bf(acc[2] * inv, acc[3] * inv)};
  if (d == 0 && a.lse) a.lse[zh * a.nq + r] = M + __logf(L);
}

// ----------------------------------------------------------------- backward --
// logit x of raw score s and dx/ds (scale, soft-cap); masked -> x = -inf
struct FaLogit {
  float x, dxds;
};
__device__ __forceinline__ FaLogit fa_logit_d(const FaMask& mk, float s, int t, int j) {
  FaLogit o{-INFINITY, 0.f};
  const bool dead = mk.dead(t);
  if (j >= mk.nk || (!dead && !mk.allowed(t, j))) return o;
  float x = s * mk.scale, d = mk.scale;
  if (mk.cap > 0.f) {
    const float th = tanh_fast(x * mk.inv_cap);
    x = mk.cap * th;
    d *= 1.f - th * th;
  }
  o.x = dead ? 0.f : x;  // dead rows: finfo.min absorbed the value, autograd still passes through
  o.dxds = d;
  return o;
}

// ---- fast element-wise path of the joint backward (soft-cap and/or the Pi0 block mask) ----------
// The per-score vector work bounds the step-staged backward kernels as much as their MFMAs do, so
// each score costs: exp2(s k2) -> rcp -> th (soft-cap tanh), exp2(th * crow - lse2) = P, the mask as
// one bit test (and only in key blocks that reach past the valid prefix), dS' = P (dP - delta)
// (1 - th^2); the softmax scale is applied once to dQ / dK instead of per score.
//   key class kc(j): 0 j < cnt, 1 cond token, 2 action token, 3 prefix padding, 4 j >= nk
//   row bits rb(t) over key classes: valid prefix 0x1, cond 0x3, action 0x7, dead prefix row 0xF
//   (dead rows attend every key with logit 0: crow = 0); no mask: every row 0xF
__device__ __forceinline__ int fa_row_bits(const FaMask& mk, int t) {
  if (mk.mode != 1) return 0xF;
  if (t < mk.P) return t < mk.cnt ? 0x1 : 0xF;
  return t < mk.P + mk.C ? 0x3 : 0x7;
}
__device__ __forceinline__ int fa_key_class(const FaMask& mk, int j) {
  if (j >= mk.nk) return 4;
  if (mk.mode != 1 || j < mk.cnt) return 0;
  if (j < mk.P) return 3;
  return j < mk.P + mk.C ? 1 : 2;
}
// keys [0, fa_full_keys) are class 0: allowed for every row
__device__ __forceinline__ int fa_full_keys(const FaMask& mk) { return mk.mode == 1 ? min(mk.cnt, mk.nk) : mk.nk; }

struct FaFast {
  float k2, crow_live, scale;  // exp2 argument of tanh's exp(2u), log2-domain logit factor
  __device__ __forceinline__ FaFast(const pz_flash_args& a) {
    scale = a.scale;
    k2 = a.cap > 0.f ? 2.f * a.scale / a.cap * 1.4426950408889634f : 0.f;
    crow_live = (a.cap > 0.f ? a.cap : a.scale) * 1.4426950408889634f;
  }
  // P and dS' (dS / scale) of raw score s and dP; masked -> 0
  template <bool CAP>
  __device__ __forceinline__ void eval(float s, float dp, float lse2, float crow, float del, bool ok, float& p,
                                       float& ds) const {
    float pe, dd;
    if constexpr (CAP) {
      const float e2 = __builtin_amdgcn_exp2f(s * k2);
      const float th = fmaf(-2.f, __builtin_amdgcn_rcpf(e2 + 1.f), 1.f);
      pe = __builtin_amdgcn_exp2f(fmaf(th, crow, -lse2));
      dd = fmaf(-th, th, 1.f);
    } else {
      pe = __builtin_amdgcn_exp2f(fmaf(s, crow, -lse2));
      dd = 1.f;
    }
    pe = ok ? pe : 0.f;
    p = pe;
    ds = pe * (dp - del) * dd;
  }
};

// delta[z][r] = sum_d dO[r][d] O[r][d]: one wave per row
template <int HD>
__global__ void __launch_bounds__(256) flash_bwd_prep_kernel(pz_flash_args a) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= a.Z * a.H * a.nq) return;
  const int64_t zh = row / a.nq, r = row % a.nq, b = zh / a.H, h = zh % a.H;
  const FaRow fr{&a};
  const int gi = fr.grp(r);
  const int64_t off = fr.off(b, h, r, gi);
  const bf16_t* O = (const bf16_t*)a.g_o[gi] + off;
  const bf16_t* dO = (const bf16_t*)a.g_do[gi] + off;
  float acc = 0.f;
  for (int d = lane * 4; d < HD; d += 256) {
    float x[4], y[4];
    const u32x2 u = *reinterpret_cast<const u32x2*>(O + d), w = *reinterpret_cast<const u32x2*>(dO + d);
    x[0] = __uint_as_float(u[0] << 16); x[1] = __uint_as_float(u[0] & 0xffff0000u);
    x[2] = __uint_as_float(u[1] << 16); x[3] = __uint_as_float(u[1] & 0xffff0000u);
    y[0] = __uint_as_float(w[0] << 16); y[1] = __uint_as_float(w[0] & 0xffff0000u);
    y[2] = __uint_as_float(w[1] << 16); y[3] = __uint_as_float(w[1] & 0xffff0000u);
    acc += x[0] * y[0] + x[1] * y[1] + x[2] * y[2] + x[3] * y[3];
  }
  acc = warp_sum(acc);
  if (lane == 0) a.delta[zh * a.nq + r] = acc;
}

// dK, dV: grid (ceil(nk / 64), Z * H), 4 waves; wave w owns keys kb*64 + 16w + (lane & 15) and
// sweeps every query row of the unit in staged steps of 32 (Q, dO, lse, delta in LDS)
// FM: 1 fast element-wise path (FaFast), 2 the same with the soft-cap.
// 1-D grid of nkb x (units x splits) workgroups, the key blocks of one (unit, split) on one XCD.
template <int HD, int FM>
__global__ void __launch_bounds__(FA_NW * 64, HD == 256 ? 1 : 2) flash_bwd_kv_kernel(pz_flash_args a, int splits) {
  using D = FaDims<HD>;
  constexpr int NT = FA_NW * 64;
  __shared__ __attribute__((aligned(16))) bf16_t Qs2[2][FA_QS * D::ROW];  // double-buffered Q / dO steps
  __shared__ __attribute__((aligned(16))) bf16_t Ds2[2][FA_QS * D::ROW];
  __shared__ float lse2[2][FA_QS], del2[2][FA_QS], crw2[2][FA_QS];
  __shared__ int rbw2[2][FA_QS];
  __shared__ __attribute__((aligned(16))) bf16_t Kk[FA_KB * D::ROW];  // this workgroup's 64 keys / values
  __shared__ __attribute__((aligned(16))) bf16_t Vk[FA_KB * D::ROW];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4;
  const int64_t ZH = a.Z * a.H;
  int64_t grp;
  int kblk;
  fa_unit_block((int)((a.nk + FA_KB - 1) / FA_KB), (int)(ZH * splits), grp, kblk);
  const int64_t zh = grp % ZH, b = zh / a.H, h = zh % a.H;
  const int split = (int)(grp / ZH);
  const int k0 = kblk * FA_KB;
  const int key = k0 + wave * 16 + (lane & 15);
  const bf16_t* Q = (const bf16_t*)a.q + b * a.q_bstride + h * a.q_hstride;
  const bf16_t* K = (const bf16_t*)a.k + b * a.k_bstride + h * a.k_hstride;
  const bf16_t* V = (const bf16_t*)a.v + b * a.v_bstride + h * a.v_hstride;
  const FaMask mk(a, b);

#pragma unroll
  for (int bi = 0; bi < 2; ++bi) {  // row reads reach HDK, transposed reads HDV <= HDK
    zero_pad_cols<HD, D::HDK, D::ROW, FA_QS, NT>(Qs2[bi]);
    zero_pad_cols<HD, D::HDK, D::ROW, FA_QS, NT>(Ds2[bi]);
  }
  // query split: this workgroup sweeps query steps [qs0, qs1)
  const int nqs_all = (int)((a.nq + FA_QS - 1) / FA_QS);
  const int per = (nqs_all + splits - 1) / splits;
  const int qs0 = min(nqs_all, split * per), qs1 = min(nqs_all, qs0 + per);
  const FaFast ff(a);
  // fast path: this lane's key class and whether the wave's 16 keys are all class 0 (no mask test)
  const int kcl = fa_key_class(mk, key);
  const bool wfull = k0 + wave * 16 + 16 <= fa_full_keys(mk);
  TileStager<HD, D::ROW, FA_QS, NT> stq, std_;
  stq.load_q(a, Q, b, h, (int64_t)qs0 * FA_QS, false);
  std_.load_q(a, Q, b, h, (int64_t)qs0 * FA_QS, true);
  float lse_v = 0.f, del_v = 0.f, crw_v = 0.f;  // threads < FA_QS carry one row's lse / delta / mask
  int rbw_v = 0;
  auto load_rows = [&](int64_t r0) {
    const int64_t rr = r0 + threadIdx.x;
    lse_v = threadIdx.x < FA_QS && rr < a.nq ? a.lse[zh * a.nq + rr] : 0.f;
    del_v = threadIdx.x < FA_QS && rr < a.nq ? a.delta[zh * a.nq + rr] : 0.f;
    const int t = mk.token((int)rr);
    lse_v *= 1.4426950408889634f;
    rbw_v = fa_row_bits(mk, t);
    crw_v = mk.dead(t) ? 0.f : ff.crow_live;
  };
  load_rows((int64_t)qs0 * FA_QS);
  // this workgroup's keys / values, read as B operands (n = key, k = head dim) from LDS:
  // K for S = Q K^T, V for dP = dO V^T (in LDS rather than registers: the accumulators need them)
  zero_pad_cols<HD, D::HDK, D::ROW, FA_KB, NT>(Kk);
  zero_pad_cols<HD, D::HDK, D::ROW, FA_KB, NT>(Vk);
  {
    TileStager<HD, D::ROW, FA_KB, NT> sk;
    sk.load(K, a.ldk, k0, a.nk);
    sk.store(Kk);
    sk.load(V, a.ldv, k0, a.nk);
    sk.store(Vk);
  }
  f32x4 dk[D::NDB], dv[D::NDB];
#pragma unroll
  for (int db = 0; db < D::NDB; ++db) dk[db] = dv[db] = f32x4{0.f, 0.f, 0.f, 0.f};

  __syncthreads();  // pad columns zeroed
  stq.store(Qs2[0]);
  std_.store(Ds2[0]);
  if (threadIdx.x < FA_QS) {
    lse2[0][threadIdx.x] = lse_v;
    del2[0][threadIdx.x] = del_v;
    crw2[0][threadIdx.x] = crw_v;
    rbw2[0][threadIdx.x] = rbw_v;
  }
  __syncthreads();
  for (int qs = qs0; qs < qs1; ++qs) {
    const int64_t r0 = (int64_t)qs * FA_QS;
    const int cur = (qs - qs0) & 1;
    const bf16_t* Qs = Qs2[cur];
    const bf16_t* Ds = Ds2[cur];
    const float* lse_s = lse2[cur];
    const float* del_s = del2[cur];
    const float* crw_s = crw2[cur];
    const int* rbw_s = rbw2[cur];
    const bool more = qs + 1 < qs1;
    if (more) {  // next query step in flight during this step's MFMAs
      stq.load_q(a, Q, b, h, r0 + FA_QS, false);
      std_.load_q(a, Q, b, h, r0 + FA_QS, true);
      load_rows(r0 + FA_QS);
    }
    f32x4 p[2], ds[2];  // [16-row query block]: lane holds rows 16i + 4g + e, key = lane's key
    bf16x8 kfr[D::NKS], vfr[D::NKS];
#pragma unroll
    for (int ks = 0; ks < D::NKS; ++ks) {
      kfr[ks] = frag_row<D::ROW>(Kk, wave * 16, ks * 32, lane);
      vfr[ks] = frag_row<D::ROW>(Vk, wave * 16, ks * 32, lane);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      f32x4 sv = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
      bf16x8 qa[D::NKS], da[D::NKS];  // LDS reads issued ahead of the MFMAs
#pragma unroll
      for (int ks = 0; ks < D::NKS; ++ks) {
        qa[ks] = frag_row<D::ROW>(Qs, i * 16, ks * 32, lane);
        da[ks] = frag_row<D::ROW>(Ds, i * 16, ks * 32, lane);
      }
#pragma unroll
      for (int ks = 0; ks < D::NKS; ++ks) {
        sv = mfma(qa[ks], kfr[ks], sv);
        dp = mfma(da[ks], vfr[ks], dp);
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int rr = i * 16 + 4 * g + e;
        float pe = 0.f, dse = 0.f;
        // (rows past nq: zero Q / dO rows and delta, no contribution)
        const bool ok = wfull || ((rbw_s[rr] >> kcl) & 1);
        ff.eval<FM == 2>(sv[e], dp[e], lse_s[rr], crw_s[rr], del_s[rr], ok, pe, dse);
        p[i][e] = pe;
        ds[i][e] = dse;
      }
    }
    // dV^T[d][key] += dO^T[d][q] P[q][key];  dK^T[d][key] += Q^T[d][q] dS[q][key]
    const bf16x8 pb = pack8(p[0], p[1]);
    const bf16x8 sb = pack8(ds[0], ds[1]);
    constexpr int HB = (D::NDB + 1) / 2;  // transposed reads in two batches ahead of their MFMAs
#pragma unroll
    for (int hb = 0; hb < 2; ++hb) {
      bf16x8 dt[HB], qt[HB];
#pragma unroll
      for (int x = 0; x < HB; ++x) {
        const int db = hb * HB + x;
        if (db < D::NDB) {
          dt[x] = frag_tr<D::ROW>(Ds, 0, db * 16, lane);
          qt[x] = frag_tr<D::ROW>(Qs, 0, db * 16, lane);
        }
      }
#pragma unroll
      for (int x = 0; x < HB; ++x) {
        const int db = hb * HB + x;
        if (db < D::NDB) {
          dv[db] = mfma(dt[x], pb, dv[db]);
          dk[db] = mfma(qt[x], sb, dk[db]);
        }
      }
    }
    if (more) {
      stq.store(Qs2[cur ^ 1]);
      std_.store(Ds2[cur ^ 1]);
      if (threadIdx.x < FA_QS) {
        lse2[cur ^ 1][threadIdx.x] = lse_v;
        del2[cur ^ 1][threadIdx.x] = del_v;
        crw2[cur ^ 1][threadIdx.x] = crw_v;
        rbw2[cur ^ 1][threadIdx.x] = rbw_v;
      }
    }
    __syncthreads();
  }
  if (key >= a.nk) return;
#pragma unroll
  for (int db = 0; db < D::NDB; ++db) dk[db] *= ff.scale;  // the fast path's dS' excludes the softmax scale
  if (splits > 1) {  // fp32 partial sums of this query split -> ws[split][unit][key][HD] (dK), then dV
    const int64_t slab = ZH * a.nk * HD;
    float* pk = a.ws + ((int64_t)split * ZH + zh) * a.nk * HD + (int64_t)key * HD;
    float* pv = pk + (int64_t)splits * slab;
#pragma unroll
    for (int db = 0; db < D::NDB; ++db) {
      const int d = db * 16 + 4 * g;
      if (d < HD) {
        *reinterpret_cast<f32x4*>(pk + d) = dk[db];
        *reinterpret_cast<f32x4*>(pv + d) = dv[db];
      }
    }
    return;
  }
  bf16_t* dK = (bf16_t*)a.dk + b * a.k_bstride + h * a.k_hstride + (int64_t)key * a.ldk;
  bf16_t* dV = (bf16_t*)a.dv + b * a.v_bstride + h * a.v_hstride + (int64_t)key * a.ldv;
#pragma unroll
  for (int db = 0; db < D::NDB; ++db) {
    const int d = db * 16 + 4 * g;
    if (d < HD) {
      *reinterpret_cast<u32x2*>(dK + d) = u32x2{pack2bf(dk[db][0], dk[db][1]), pack2bf(dk[db][2], dk[db][3])};
      *reinterpret_cast<u32x2*>(dV + d) = u32x2{pack2bf(dv[db][0], dv[db][1]), pack2bf(dv[db][2], dv[db][3])};
    }
  }
}

// sum of the query-split partials (fixed order) -> bf16 dK / dV; one thread per 4 elements
template <int HD>
__global__ void __launch_bounds__(256) flash_bwd_kv_reduce_kernel(pz_flash_args a, int splits) {
  const int64_t units = a.Z * a.H, per_unit = a.nk * (HD / 4);
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= 2 * units * per_unit) return;
  const bool is_v = idx >= units * per_unit;
  const int64_t i = is_v ? idx - units * per_unit : idx;
  const int64_t zh = i / per_unit, rem = i % per_unit, key = rem / (HD / 4), d = (rem % (HD / 4)) * 4;
  const int64_t slab = units * a.nk * HD;
  const float* src = a.ws + (is_v ? (int64_t)splits * slab : 0) + zh * a.nk * HD + key * HD + d;
  f32x4 acc = *reinterpret_cast<const f32x4*>(src);
  for (int sp = 1; sp < splits; ++sp) acc += *reinterpret_cast<const f32x4*>(src + sp * slab);
  const int64_t b = zh / a.H, h = zh % a.H;
  bf16_t* dst = is_v ? (bf16_t*)a.dv + b * a.v_bstride + h * a.v_hstride + key * a.ldv
                     : (bf16_t*)a.dk + b * a.k_bstride + h * a.k_hstride + key * a.ldk;
  *reinterpret_cast<u32x2*>(dst + d) = u32x2{pack2bf(acc[0], acc[1]), pack2bf(acc[2], acc[3])};
}

// dQ (+ delta): 4 waves x 32 query rows (two 16-row blocks per K / V fragment read), 32-key blocks double-buffered in LDS (70 KiB), the
// query blocks of one unit on one XCD (its K / V served from that L2).  1-D grid.
constexpr int JQ_NW = 4, JQ_KB = 32;
template <int HD, bool CAP>
__global__ void __launch_bounds__(JQ_NW * 64, 1) flash_bwd_q2_kernel(pz_flash_args a) {
  using D = FaDims<HD>;
  constexpr int NT = JQ_NW * 64, RPW = JQ_NW * 32;
  __shared__ __attribute__((aligned(16))) bf16_t Ks2[2][JQ_KB * D::ROW];
  __shared__ __attribute__((aligned(16))) bf16_t Vs2[2][JQ_KB * D::ROW];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4;
  int64_t zh;
  int qblk;
  fa_unit_block((int)((a.nq + RPW - 1) / RPW), (int)(a.Z * a.H), zh, qblk);
  const int64_t b = zh / a.H, h = zh % a.H;
  const bf16_t* Q = (const bf16_t*)a.q + b * a.q_bstride + h * a.q_hstride;
  const bf16_t* K = (const bf16_t*)a.k + b * a.k_bstride + h * a.k_hstride;
  const bf16_t* V = (const bf16_t*)a.v + b * a.v_bstride + h * a.v_hstride;
  const FaMask mk(a, b);
  const FaFast ff(a);
  const FaRow fr{&a};
#pragma unroll
  for (int bi = 0; bi < 2; ++bi) {
    zero_pad_cols<HD, D::HDK, D::ROW, JQ_KB, NT>(Ks2[bi]);
    zero_pad_cols<HD, D::HDK, D::ROW, JQ_KB, NT>(Vs2[bi]);
  }
  const int nkb = (int)((a.nk + JQ_KB - 1) / JQ_KB);
  const int full_keys = fa_full_keys(mk);
  TileStager<HD, D::ROW, JQ_KB, NT> stk, stv;
  stk.load(K, a.ldk, 0, a.nk);
  stv.load(V, a.ldv, 0, a.nk);
  bf16x8 qf[2][D::NKS], df[2][D::NKS];
  float del[2], lse2[2], crow[2];
  int rb[2];
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    const int64_t r = (int64_t)qblk * RPW + wave * 32 + qb * 16 + (lane & 15);
    const bool live = r < a.nq;
    const bf16_t* dOr = nullptr;
    const bf16_t* Or = nullptr;
    if (live) {
      const int gi = fr.grp(r);
      dOr = (const bf16_t*)a.g_do[gi] + fr.off(b, h, r, gi);
      Or = (const bf16_t*)a.g_o[gi] + fr.off(b, h, r, gi);
    }
    float dl = 0.f;
#pragma unroll
    for (int ks = 0; ks < D::NKS; ++ks) {
      const int c = ks * 32 + 8 * g;
      const bool ok = live && c < HD;
      qf[qb][ks] = ok ? *reinterpret_cast<const bf16x8*>(Q + r * a.ldq + c) : bf16x8{};
      df[qb][ks] = ok ? *reinterpret_cast<const bf16x8*>(dOr + c) : bf16x8{};
      if (ok) {
        const bf16x8 ov = *reinterpret_cast<const bf16x8*>(Or + c);
#pragma unroll
        for (int e = 0; e < 8; ++e) dl += (float)df[qb][ks][e] * (float)ov[e];
      }
    }
    dl += __shfl_xor(dl, 16, 64);
    dl += __shfl_xor(dl, 32, 64);
    del[qb] = dl;
    if (live && g == 0) a.delta[zh * a.nq + r] = dl;
    lse2[qb] = live ? a.lse[zh * a.nq + r] * 1.4426950408889634f : 0.f;
    const int t = mk.token((int)r);
    rb[qb] = fa_row_bits(mk, t);
    crow[qb] = mk.dead(t) ? 0.f : ff.crow_live;
  }
  f32x4 dq[D::NDB][2];
#pragma unroll
  for (int db = 0; db < D::NDB; ++db) dq[db][0] = dq[db][1] = f32x4{0.f, 0.f, 0.f, 0.f};

  __syncthreads();  // pad columns zeroed
  stk.store(Ks2[0]);
  stv.store(Vs2[0]);
  __syncthreads();
  for (int kb = 0; kb < nkb; ++kb) {
    const bf16_t* Ks = Ks2[kb & 1];
    const bf16_t* Vs = Vs2[kb & 1];
    const bool more = kb + 1 < nkb;
    if (more) {
      stk.load(K, a.ldk, (int64_t)(kb + 1) * JQ_KB, a.nk);
      stv.load(V, a.ldv, (int64_t)(kb + 1) * JQ_KB, a.nk);
    }
    const bool full = (kb + 1) * JQ_KB <= full_keys;
    f32x4 ds[2][2];  // dS'^T[key 16i + 4g + e][query of block qb]
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      bf16x8 kfr[D::NKS], vfr[D::NKS];
#pragma unroll
      for (int ks = 0; ks < D::NKS; ++ks) {
        kfr[ks] = frag_row<D::ROW>(Ks, i * 16, ks * 32, lane);
        vfr[ks] = frag_row<D::ROW>(Vs, i * 16, ks * 32, lane);
      }
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) {
        f32x4 sv = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < D::NKS; ++ks) {
          sv = mfma(kfr[ks], qf[qb][ks], sv);
          dp = mfma(vfr[ks], df[qb][ks], dp);
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const bool ok = full || ((rb[qb] >> fa_key_class(mk, kb * JQ_KB + i * 16 + 4 * g + e)) & 1);
          float pe, dse;
          ff.eval<CAP>(sv[e], dp[e], lse2[qb], crow[qb], del[qb], ok, pe, dse);
          ds[i][qb][e] = dse;
        }
      }
    }
    const bf16x8 sb0 = pack8(ds[0][0], ds[1][0]), sb1 = pack8(ds[0][1], ds[1][1]);
    constexpr int HB = (D::NDB + 1) / 2;  // transposed K reads in two batches ahead of their MFMAs
#pragma unroll
    for (int hb = 0; hb < 2; ++hb) {
      bf16x8 kt[HB];
#pragma unroll
      for (int x = 0; x < HB; ++x)
        if (hb * HB + x < D::NDB) kt[x] = frag_tr<D::ROW>(Ks, 0, (hb * HB + x) * 16, lane);
#pragma unroll
      for (int x = 0; x < HB; ++x) {
        const int db = hb * HB + x;
        if (db < D::NDB) {
          dq[db][0] = mfma(kt[x], sb0, dq[db][0]);
          dq[db][1] = mfma(kt[x], sb1, dq[db][1]);
        }
      }
    }
    if (more) {
      stk.store(Ks2[(kb + 1) & 1]);
      stv.store(Vs2[(kb + 1) & 1]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    const int64_t r = (int64_t)qblk * RPW + wave * 32 + qb * 16 + (lane & 15);
    if (r >= a.nq) continue;
    bf16_t* dQ = (bf16_t*)a.dq + b * a.q_bstride + h * a.q_hstride + r * a.ldq;
#pragma unroll
    for (int db = 0; db < D::NDB; ++db) {
      const int d = db * 16 + 4 * g;
      if (d < HD)
        *reinterpret_cast<u32x2*>(dQ + d) = u32x2{pack2bf(dq[db][qb][0] * ff.scale, dq[db][qb][1] * ff.scale),
                                                  pack2bf(dq[db][qb][2] * ff.scale, dq[db][qb][3] * ff.scale)};
    }
  }
}

// ---- joint attention with the softmax probabilities exported (training default): see flash_fwd_probs_dma_kernel
constexpr int JP_NW = 8, JP_MAXKB = 5;

// ---- resident variants (SigLIP: nq, nk <= 256) ---------------------------------
// The whole key side (forward, dQ) or query side (dK/dV) of a unit is staged in LDS once, by
// loads all in flight together: one global-latency round per workgroup instead of one per
// 64-key / 32-query step, which the step-staged kernels above expose at SigLIP's small per-step
// work (16 heads x 72).  8 waves per workgroup (two per SIMD), dynamic LDS up to 142 KiB.
constexpr int FR_MAX = 256, FR_NW = 8;

template <int HD>
__global__ void __launch_bounds__(FR_NW * 64) flash_fwd_res_kernel(pz_flash_args a) {
  using D = FaDims<HD>;
  constexpr int NT = FR_NW * 64;
  extern __shared__ __attribute__((aligned(16))) char fa_smem[];
  bf16_t* Kall = reinterpret_cast<bf16_t*>(fa_smem);
  bf16_t* Vall = Kall + FR_MAX * D::ROW;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4;
  int64_t zh;
  int qblk;
  fa_unit_block((int)((a.nq + FR_NW * 16 - 1) / (FR_NW * 16)), (int)(a.Z * a.H), zh, qblk);
  const int64_t b = zh / a.H, h = zh % a.H;
  const int64_t q0 = (int64_t)qblk * (FR_NW * 16) + wave * 16;
  const bf16_t* Q = (const bf16_t*)a.q + b * a.q_bstride + h * a.q_hstride;
  const bf16_t* K = (const bf16_t*)a.k + b * a.k_bstride + h * a.k_hstride;
  const bf16_t* V = (const bf16_t*)a.v + b * a.v_bstride + h * a.v_hstride;
  const FaMask mk(a, b);
  {
    TileStager<HD, D::ROW, FR_MAX, NT> stk, stv;
    stk.load(K, a.ldk, 0, a.nk);
    stv.load(V, a.ldv, 0, a.nk);
    zero_pad_cols<HD, D::HDK, D::ROW, FR_MAX, NT>(Kall);
    zero_pad_cols<HD, D::HDK, D::ROW, FR_MAX, NT>(Vall);
    stk.store(Kall);
    stv.store(Vall);
  }
  bf16x8 qf[D::NKS];
  const int64_t rq = q0 + (lane & 15);
#pragma unroll
  for (int ks = 0; ks < D::NKS; ++ks) {
    const int c = ks * 32 + 8 * g;
    qf[ks] = (rq < a.nq && c < HD) ? *reinterpret_cast<const bf16x8*>(Q + rq * a.ldq + c) : bf16x8{};
  }
  f32x4 o[D::NDB];
#pragma unroll
  for (int db = 0; db < D::NDB; ++db) o[db] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, l = 0.f;
  const int t = mk.token((int)rq);
  const int nkb = (int)((a.nk + FA_KB - 1) / FA_KB);
  __syncthreads();
  for (int kb = 0; kb < nkb; ++kb) {
    const bf16_t* Ks = Kall + kb * FA_KB * D::ROW;
    const bf16_t* Vs = Vall + kb * FA_KB * D::ROW;
    f32x4 sc[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) sc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < D::NKS; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i) sc[i] = mfma(frag_row<D::ROW>(Ks, i * 16, ks * 32, lane), qf[ks], sc[i]);
    float mx = -INFINITY;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float x = fa_logit(mk, sc[i][e], t, kb * FA_KB + i * 16 + 4 * g + e);
        sc[i][e] = x;
        mx = fmaxf(mx, x);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float mn = fmaxf(m, mx);
    const float alpha = mn == -INFINITY ? 1.f : __expf(m - mn);
    float sum = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float pv = mn == -INFINITY ? 0.f : __expf(sc[i][e] - mn);
        sc[i][e] = pv;
        sum += pv;
      }
    sum += __shfl_xor(sum, 16, 64);
    sum += __shfl_xor(sum, 32, 64);
    l = l * alpha + sum;
    m = mn;
#pragma unroll
    for (int db = 0; db < D::NDB; ++db) o[db] *= alpha;
    const bf16x8 pf0 = pack8(sc[0], sc[1]), pf1 = pack8(sc[2], sc[3]);
#pragma unroll
    for (int db = 0; db < D::NDB; ++db) {
      o[db] = mfma(frag_tr<D::ROW>(Vs, 0, db * 16, lane), pf0, o[db]);
      o[db] = mfma(frag_tr<D::ROW>(Vs, 32, db * 16, lane), pf1, o[db]);
    }
  }
  if (rq >= a.nq) return;
  const float inv = l > 0.f ? 1.f / l : 0.f;
  const FaRow fr{&a};
  const int gi = fr.grp(rq);
  bf16_t* O = (bf16_t*)a.g_o[gi] + fr.off(b, h, rq, gi);
#pragma unroll
  for (int db = 0; db < D::NDB; ++db) {
    const int d = db * 16 + 4 * g;
    if (d < HD)
      *reinterpret_cast<u32x2*>(O + d) =
          u32x2{pack2bf(o[db][0] * inv, o[db][1] * inv), pack2bf(o[db][2] * inv, o[db][3] * inv)};
  }
  if (g == 0 && a.lse) a.lse[zh * a.nq + rq] = m + __logf(l);
}

// dQ (+ delta) with every key / value of the unit resident: grid (ceil(nq / 128), Z * H)
template <int HD>
__global__ void __launch_bounds__(FR_NW * 64) flash_bwd_q_res_kernel(pz_flash_args a) {
  using D = FaDims<HD>;
  constexpr int NT = FR_NW * 64;
  extern __shared__ __attribute__((aligned(16))) char fa_smem[];
  bf16_t* Kall = reinterpret_cast<bf16_t*>(fa_smem);
  bf16_t* Vall = Kall + FR_MAX * D::ROW;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4;
  int64_t zh;
  int qblk;
  fa_unit_block((int)((a.nq + FR_NW * 16 - 1) / (FR_NW * 16)), (int)(a.Z * a.H), zh, qblk);
  const int64_t b = zh / a.H, h = zh % a.H;
  const int64_t r = (int64_t)qblk * (FR_NW * 16) + wave * 16 + (lane & 15);
  const bf16_t* Q = (const bf16_t*)a.q + b * a.q_bstride + h * a.q_hstride;
  const bf16_t* K = (const bf16_t*)a.k + b * a.k_bstride + h * a.k_hstride;
  const bf16_t* V = (const bf16_t*)a.v + b * a.v_bstride + h * a.v_hstride;
  const FaMask mk(a, b);
  const FaRow fr{&a};
  {
    TileStager<HD, D::ROW, FR_MAX, NT> stk, stv;
    stk.load(K, a.ldk, 0, a.nk);
    stv.load(V, a.ldv, 0, a.nk);
    zero_pad_cols<HD, D::HDK, D::ROW, FR_MAX, NT>(Kall);
    zero_pad_cols<HD, D::HDK, D::ROW, FR_MAX, NT>(Vall);
    stk.store(Kall);
    stv.store(Vall);
  }
  bf16x8 qf[D::NKS], df[D::NKS];
  const bool live = r < a.nq;
  const bf16_t* dOr = nullptr;
  const bf16_t* Or = nullptr;
  if (live) {
    const int gi = fr.grp(r);
    dOr = (const bf16_t*)a.g_do[gi] + fr.off(b, h, r, gi);
    Or = (const bf16_t*)a.g_o[gi] + fr.off(b, h, r, gi);
  }
  float del = 0.f;
#pragma unroll
  for (int ks = 0; ks < D::NKS; ++ks) {
    const int c = ks * 32 + 8 * g;
    const bool ok = live && c < HD;
    qf[ks] = ok ? *reinterpret_cast<const bf16x8*>(Q + r * a.ldq + c) : bf16x8{};
    df[ks] = ok ? *reinterpret_cast<const bf16x8*>(dOr + c) : bf16x8{};
    if (ok) {
      const bf16x8 ov = *reinterpret_cast<const bf16x8*>(Or + c);
#pragma unroll
      for (int e = 0; e < 8; ++e) del += (float)df[ks][e] * (float)ov[e];
    }
  }
  del += __shfl_xor(del, 16, 64);
  del += __shfl_xor(del, 32, 64);
  if (live && g == 0) a.delta[zh * a.nq + r] = del;
  const float lse = live ? a.lse[zh * a.nq + r] : 0.f;
  const int tq = mk.token((int)r);
  f32x4 dq[D::NDB];
#pragma unroll
  for (int db = 0; db < D::NDB; ++db) dq[db] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nkb = (int)((a.nk + FA_KB - 1) / FA_KB);
  __syncthreads();
  for (int kb = 0; kb < nkb; ++kb) {
    const bf16_t* Ks = Kall + kb * FA_KB * D::ROW;
    const bf16_t* Vs = Vall + kb * FA_KB * D::ROW;
    f32x4 ds[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      f32x4 sv = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
      bf16x8 kfr[D::NKS], vfr[D::NKS];
#pragma unroll
      for (int ks = 0; ks < D::NKS; ++ks) {
        kfr[ks] = frag_row<D::ROW>(Ks, i * 16, ks * 32, lane);
        vfr[ks] = frag_row<D::ROW>(Vs, i * 16, ks * 32, lane);
      }
#pragma unroll
      for (int ks = 0; ks < D::NKS; ++ks) {
        sv = mfma(kfr[ks], qf[ks], sv);
        dp = mfma(vfr[ks], df[ks], dp);
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int j = kb * FA_KB + i * 16 + 4 * g + e;
        float dse = 0.f;
        if (live) {
          const FaLogit lg = fa_logit_d(mk, sv[e], tq, j);
          const float pe = lg.x == -INFINITY ? 0.f : __expf(lg.x - lse);
          dse = pe * (dp[e] - del) * lg.dxds;
        }
        ds[i][e] = dse;
      }
    }
#pragma unroll
    for (int k2 = 0; k2 < 2; ++k2) {
      const bf16x8 sb = pack8(ds[2 * k2], ds[2 * k2 + 1]);
      bf16x8 kt[D::NDB];
#pragma unroll
      for (int db = 0; db < D::NDB; ++db) kt[db] = frag_tr<D::ROW>(Ks, k2 * 32, db * 16, lane);
#pragma unroll
      for (int db = 0; db < D::NDB; ++db) dq[db] = mfma(kt[db], sb, dq[db]);
    }
  }
  if (!live) return;
  bf16_t* dQ = (bf16_t*)a.dq + b * a.q_bstride + h * a.q_hstride + r * a.ldq;
#pragma unroll
  for (int db = 0; db < D::NDB; ++db) {
    const int d = db * 16 + 4 * g;
    if (d < HD) *reinterpret_cast<u32x2*>(dQ + d) = u32x2{pack2bf(dq[db][0], dq[db][1]), pack2bf(dq[db][2], dq[db][3])};
  }
}

// dK, dV with every query row (Q, dO, lse, delta) of the unit resident: grid (ceil(nk / 64), Z * H);
// wave w owns keys 16 (w & 3).. of the block and sweeps query half (w >> 2); halves summed in LDS
template <int HD>
__global__ void __launch_bounds__(FR_NW * 64) flash_bwd_kv_res_kernel(pz_flash_args a) {
  using D = FaDims<HD>;
  constexpr int NT = FR_NW * 64;
  extern __shared__ __attribute__((aligned(16))) char fa_smem[];
  bf16_t* Qall = reinterpret_cast<bf16_t*>(fa_smem);
  bf16_t* Dall = Qall + FR_MAX * D::ROW;
  bf16_t* Kk = Dall + FR_MAX * D::ROW;
  bf16_t* Vk = Kk + FA_KB * D::ROW;
  float* lse_all = reinterpret_cast<float*>(Vk + FA_KB * D::ROW);
  float* del_all = lse_all + FR_MAX;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4;
  const int kw = wave & 3, qh = wave >> 2;
  int64_t zh;
  int kblk;
  fa_unit_block((int)((a.nk + FA_KB - 1) / FA_KB), (int)(a.Z * a.H), zh, kblk);
  const int64_t b = zh / a.H, h = zh % a.H;
  const int k0 = kblk * FA_KB;
  const int key = k0 + kw * 16 + (lane & 15);
  const bf16_t* Q = (const bf16_t*)a.q + b * a.q_bstride + h * a.q_hstride;
  const bf16_t* K = (const bf16_t*)a.k + b * a.k_bstride + h * a.k_hstride;
  const bf16_t* V = (const bf16_t*)a.v + b * a.v_bstride + h * a.v_hstride;
  const FaMask mk(a, b);
  {
    TileStager<HD, D::ROW, FR_MAX, NT> stq, std_;
    TileStager<HD, D::ROW, FA_KB, NT> sk, sv;
    stq.load_q(a, Q, b, h, 0, false);
    std_.load_q(a, Q, b, h, 0, true);
    sk.load(K, a.ldk, k0, a.nk);
    sv.load(V, a.ldv, k0, a.nk);
    const int tr = threadIdx.x;
    const float lv = tr < FR_MAX && tr < a.nq ? a.lse[zh * a.nq + tr] : 0.f;
    const float dv_ = tr < FR_MAX && tr < a.nq ? a.delta[zh * a.nq + tr] : 0.f;
    zero_pad_cols<HD, D::HDK, D::ROW, FR_MAX, NT>(Qall);
    zero_pad_cols<HD, D::HDK, D::ROW, FR_MAX, NT>(Dall);
    zero_pad_cols<HD, D::HDK, D::ROW, FA_KB, NT>(Kk);
    zero_pad_cols<HD, D::HDK, D::ROW, FA_KB, NT>(Vk);
    stq.store(Qall);
    std_.store(Dall);
    sk.store(Kk);
    sv.store(Vk);
    if (tr < FR_MAX) {
      lse_all[tr] = lv;
      del_all[tr] = dv_;
    }
  }
  f32x4 dk[D::NDB], dv[D::NDB];
#pragma unroll
  for (int db = 0; db < D::NDB; ++db) dk[db] = dv[db] = f32x4{0.f, 0.f, 0.f, 0.f};
  __syncthreads();
  bf16x8 kfr[D::NKS], vfr[D::NKS];
#pragma unroll
  for (int ks = 0; ks < D::NKS; ++ks) {
    kfr[ks] = frag_row<D::ROW>(Kk, kw * 16, ks * 32, lane);
    vfr[ks] = frag_row<D::ROW>(Vk, kw * 16, ks * 32, lane);
  }
  const int nqs = (int)((a.nq + FA_QS - 1) / FA_QS);
  const int half = (nqs + 1) / 2;
  const int qs0 = qh * half, qs1 = min(nqs, qs0 + half);
  for (int qs = qs0; qs < qs1; ++qs) {
    const int r0 = qs * FA_QS;
    const bf16_t* Qs = Qall + r0 * D::ROW;
    const bf16_t* Ds = Dall + r0 * D::ROW;
    f32x4 p[2], ds[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      f32x4 sv = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
      bf16x8 qa[D::NKS], da[D::NKS];
#pragma unroll
      for (int ks = 0; ks < D::NKS; ++ks) {
        qa[ks] = frag_row<D::ROW>(Qs, i * 16, ks * 32, lane);
        da[ks] = frag_row<D::ROW>(Ds, i * 16, ks * 32, lane);
      }
#pragma unroll
      for (int ks = 0; ks < D::NKS; ++ks) {
        sv = mfma(qa[ks], kfr[ks], sv);
        dp = mfma(da[ks], vfr[ks], dp);
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int rr = r0 + i * 16 + 4 * g + e;
        float pe = 0.f, dse = 0.f;
        if (rr < a.nq) {
          const FaLogit lg = fa_logit_d(mk, sv[e], mk.token(rr), key);
          pe = lg.x == -INFINITY ? 0.f : __expf(lg.x - lse_all[rr]);
          dse = pe * (dp[e] - del_all[rr]) * lg.dxds;
        }
        p[i][e] = pe;
        ds[i][e] = dse;
      }
    }
    const bf16x8 pb = pack8(p[0], p[1]);
    const bf16x8 sb = pack8(ds[0], ds[1]);
#pragma unroll
    for (int db = 0; db < D::NDB; ++db) {
      dv[db] = mfma(frag_tr<D::ROW>(Ds, 0, db * 16, lane), pb, dv[db]);
      dk[db] = mfma(frag_tr<D::ROW>(Qs, 0, db * 16, lane), sb, dk[db]);
    }
  }
  // query halves: waves 4..7 hand their partial sums to waves 0..3 through LDS (Q image reused)
  __syncthreads();
  f32x4* red = reinterpret_cast<f32x4*>(fa_smem);
  if (qh == 1) {
#pragma unroll
    for (int db = 0; db < D::NDB; ++db) {
      red[((kw * D::NDB + db) * 2 + 0) * 64 + lane] = dk[db];
      red[((kw * D::NDB + db) * 2 + 1) * 64 + lane] = dv[db];
    }
  }
  __syncthreads();
  if (qh == 1 || key >= a.nk) return;
#pragma unroll
  for (int db = 0; db < D::NDB; ++db) {
    dk[db] += red[((kw * D::NDB + db) * 2 + 0) * 64 + lane];
    dv[db] += red[((kw * D::NDB + db) * 2 + 1) * 64 + lane];
  }
  bf16_t* dK = (bf16_t*)a.dk + b * a.k_bstride + h * a.k_hstride + (int64_t)key * a.ldk;
  bf16_t* dV = (bf16_t*)a.dv + b * a.v_bstride + h * a.v_hstride + (int64_t)key * a.ldv;
#pragma unroll
  for (int db = 0; db < D::NDB; ++db) {
    const int d = db * 16 + 4 * g;
    if (d < HD) {
      *reinterpret_cast<u32x2*>(dK + d) = u32x2{pack2bf(dk[db][0], dk[db][1]), pack2bf(dk[db][2], dk[db][3])};
      *reinterpret_cast<u32x2*>(dV + d) = u32x2{pack2bf(dv[db][0], dv[db][1]), pack2bf(dv[db][2], dv[db][3])};
    }
  }
}

constexpr int FR_SMEM_KQ = 2 * FR_MAX * FaDims<72>::ROW * 2;  // forward / dQ: K + V images
constexpr int FR_SMEM_KV = 2 * FR_MAX * FaDims<72>::ROW * 2 + 2 * FA_KB * FaDims<72>::ROW * 2 + 2 * FR_MAX * 4;

// ---- one workgroup per unit (SigLIP: 16 heads x 72, 256 tokens) -----------------------------
// The resident kernels above give each unit 2 (forward, dQ) or 4 (dK/dV) workgroups, and every one
// of them stages the unit's whole resident side (114 KiB) before its first MFMA: at one workgroup
// per CU the staging is most of their time (dK/dV: 585 MB staged per micro-batch layer).  Here one
// workgroup of 8 waves owns the whole unit, each wave 32 rows (queries) or 32 keys, so each
// resident operand is staged once per unit, every LDS fragment read feeds two MFMAs (two 16-row
// blocks), and the dK/dV pass takes its K/V fragments straight from global memory into registers
// (no K/V image, no query-half reduction).  Grid = Z * H workgroups (1024 per micro-batch layer).
// unit of this workgroup: the H heads of one image on one XCD (workgroups are dealt round-robin over
// the 8 XCDs), so the 128-B lines that adjacent heads' 144-B q / k / v / O / dO segments share are fetched
// into one L2 (the default order puts consecutive heads on different XCDs); Z % 8 != 0: linear
__device__ __forceinline__ int64_t fa_unit_of(const pz_flash_args& a) {
  const int64_t id = blockIdx.x;
  if (a.Z % 8 != 0) return id;
  const int64_t xcd = id & 7, local = id >> 3;
  return ((local / a.H) * 8 + xcd) * a.H + local % a.H;
}

constexpr int FU_NW = 8;

// PLAIN (no mask, no soft-cap: SigLIP): the element-wise softmax in the log2 domain with the scale
// folded into one multiply and no mask / -inf guards -- the per-score VALU work, not the MFMAs,
// bounds these head-72 kernels (5 instead of ~17 vector instructions per score)
constexpr float FA_LOG2E = 1.4426950408889634f, FA_LN2 = 0.6931471805599453f;

template <int HD, bool PLAIN>
__global__ void __launch_bounds__(FU_NW * 64) flash_fwd_unit_kernel(pz_flash_args a) {
  using D = FaDims<HD>;
  constexpr int NT = FU_NW * 64;
  extern __shared__ __attribute__((aligned(16))) char fa_smem[];
  bf16_t* Kall = reinterpret_cast<bf16_t*>(fa_smem);
  bf16_t* Vall = Kall + FR_MAX * D::ROW;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4;
  const int64_t zh = fa_unit_of(a), b = zh / a.H, h = zh % a.H;
  const bf16_t* Q = (const bf16_t*)a.q + b * a.q_bstride + h * a.q_hstride;
  const bf16_t* K = (const bf16_t*)a.k + b * a.k_bstride + h * a.k_hstride;
  const bf16_t* V = (const bf16_t*)a.v + b * a.v_bstride + h * a.v_hstride;
  const FaMask mk(a, b);
  {
    TileStager<HD, D::ROW, FR_MAX, NT> stk, stv;
    stk.load(K, a.ldk, 0, a.nk);
    stv.load(V, a.ldv, 0, a.nk);
    zero_pad_cols<HD, D::HDK, D::ROW, FR_MAX, NT>(Kall);
    zero_pad_cols<HD, D::HDK, D::ROW, FR_MAX, NT>(Vall);
    stk.store(Kall);
    stv.store(Vall);
  }
  bf16x8 qf[2][D::NKS];
  int t[2];
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    const int64_t rq = wave * 32 + qb * 16 + (lane & 15);
    t[qb] = mk.token((int)rq);
#pragma unroll
    for (int ks = 0; ks < D::NKS; ++ks) {
      const int c = ks * 32 + 8 * g;
      qf[qb][ks] = (rq < a.nq && c < HD) ? *reinterpret_cast<const bf16x8*>(Q + rq * a.ldq + c) : bf16x8{};
    }
  }
  f32x4 o[D::NDB][2];
#pragma unroll
  for (int db = 0; db < D::NDB; ++db) o[db][0] = o[db][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m[2] = {-INFINITY, -INFINITY}, l[2] = {0.f, 0.f};
  const float sl2 = a.scale * FA_LOG2E;
  const int nkb = (int)((a.nk + FA_KB - 1) / FA_KB);
  __syncthreads();
  for (int kb = 0; kb < nkb; ++kb) {
    const bf16_t* Ks = Kall + kb * FA_KB * D::ROW;
    const bf16_t* Vs = Vall + kb * FA_KB * D::ROW;
    f32x4 sc[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i) sc[i][0] = sc[i][1] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < D::NKS; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const bf16x8 kf = frag_row<D::ROW>(Ks, i * 16, ks * 32, lane);
        sc[i][0] = mfma(kf, qf[0][ks], sc[i][0]);
        sc[i][1] = mfma(kf, qf[1][ks], sc[i][1]);
      }
    bf16x8 pf[2][2];  // [k-step of 32 keys][query block]
    const bool full = (kb + 1) * FA_KB <= (int)a.nk;
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) {
      float mx = -INFINITY;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int j = kb * FA_KB + i * 16 + 4 * g + e;
          float x;
          if constexpr (PLAIN) {
            x = sc[i][qb][e] * sl2;  // log2-domain logit
            if (!full && j >= (int)a.nk) x = -INFINITY;
          } else {
            x = fa_logit(mk, sc[i][qb][e], t[qb], j);
          }
          sc[i][qb][e] = x;
          mx = fmaxf(mx, x);
        }
      mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
      mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
      const float mn = fmaxf(m[qb], mx);
      float sum = 0.f, alpha;
      if constexpr (PLAIN) {  // key 0 is valid: mn is finite from the first block on; exp2(-inf) = 0
        alpha = __builtin_amdgcn_exp2f(m[qb] - mn);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float pv = __builtin_amdgcn_exp2f(sc[i][qb][e] - mn);
            sc[i][qb][e] = pv;
            sum += pv;
          }
      } else {
        alpha = mn == -INFINITY ? 1.f : __expf(m[qb] - mn);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float pv = mn == -INFINITY ? 0.f : __expf(sc[i][qb][e] - mn);
            sc[i][qb][e] = pv;
            sum += pv;
          }
      }
      sum += __shfl_xor(sum, 16, 64);
      sum += __shfl_xor(sum, 32, 64);
      l[qb] = l[qb] * alpha + sum;
      m[qb] = mn;
#pragma unroll
      for (int db = 0; db < D::NDB; ++db) o[db][qb] *= alpha;
      pf[0][qb] = pack8(sc[0][qb], sc[1][qb]);
      pf[1][qb] = pack8(sc[2][qb], sc[3][qb]);
    }
#pragma unroll
    for (int k2 = 0; k2 < 2; ++k2)
#pragma unroll
      for (int db = 0; db < D::NDB; ++db) {
        const bf16x8 vf = frag_tr<D::ROW>(Vs, k2 * 32, db * 16, lane);
        o[db][0] = mfma(vf, pf[k2][0], o[db][0]);
        o[db][1] = mfma(vf, pf[k2][1], o[db][1]);
      }
  }
  const FaRow fr{&a};
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    const int64_t rq = wave * 32 + qb * 16 + (lane & 15);
    if (rq >= a.nq) continue;
    const float inv = l[qb] > 0.f ? 1.f / l[qb] : 0.f;
    const int gi = fr.grp(rq);
    bf16_t* O = (bf16_t*)a.g_o[gi] + fr.off(b, h, rq, gi);
#pragma unroll
    for (int db = 0; db < D::NDB; ++db) {
      const int d = db * 16 + 4 * g;
      if (d < HD)
        *reinterpret_cast<u32x2*>(O + d) =
            u32x2{pack2bf(o[db][qb][0] * inv, o[db][qb][1] * inv), pack2bf(o[db][qb][2] * inv, o[db][qb][3] * inv)};
    }
    if (g == 0 && a.lse) a.lse[zh * a.nq + rq] = PLAIN ? m[qb] * FA_LN2 + __logf(l[qb]) : m[qb] + __logf(l[qb]);
  }
}

// dQ (+ delta): one workgroup per unit, K / V resident, wave w owns query rows 32w .. 32w + 31
template <int HD, bool PLAIN>
__global__ void __launch_bounds__(FU_NW * 64) flash_bwd_q_unit_kernel(pz_flash_args a) {
  using D = FaDims<HD>;
  constexpr int NT = FU_NW * 64;
  extern __shared__ __attribute__((aligned(16))) char fa_smem[];
  bf16_t* Kall = reinterpret_cast<bf16_t*>(fa_smem);
  bf16_t* Vall = Kall + FR_MAX * D::ROW;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4;
  const int64_t zh = fa_unit_of(a), b = zh / a.H, h = zh % a.H;
  const bf16_t* Q = (const bf16_t*)a.q + b * a.q_bstride + h * a.q_hstride;
  const bf16_t* K = (const bf16_t*)a.k + b * a.k_bstride + h * a.k_hstride;
  const bf16_t* V = (const bf16_t*)a.v + b * a.v_bstride + h * a.v_hstride;
  const FaMask mk(a, b);
  const FaRow fr{&a};
  {
    TileStager<HD, D::ROW, FR_MAX, NT> stk, stv;
    stk.load(K, a.ldk, 0, a.nk);
    stv.load(V, a.ldv, 0, a.nk);
    zero_pad_cols<HD, D::HDK, D::ROW, FR_MAX, NT>(Kall);
    zero_pad_cols<HD, D::HDK, D::ROW, FR_MAX, NT>(Vall);
    stk.store(Kall);
    stv.store(Vall);
  }
  bf16x8 qf[2][D::NKS], df[2][D::NKS];
  float del[2], lse[2];
  int tq[2];
  bool live[2];
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    const int64_t r = wave * 32 + qb * 16 + (lane & 15);
    live[qb] = r < a.nq;
    tq[qb] = mk.token((int)r);
    const bf16_t* dOr = nullptr;
    const bf16_t* Or = nullptr;
    if (live[qb]) {
      const int gi = fr.grp(r);
      dOr = (const bf16_t*)a.g_do[gi] + fr.off(b, h, r, gi);
      Or = (const bf16_t*)a.g_o[gi] + fr.off(b, h, r, gi);
    }
    float dl = 0.f;
#pragma unroll
    for (int ks = 0; ks < D::NKS; ++ks) {
      const int c = ks * 32 + 8 * g;
      const bool ok = live[qb] && c < HD;
      qf[qb][ks] = ok ? *reinterpret_cast<const bf16x8*>(Q + r * a.ldq + c) : bf16x8{};
      df[qb][ks] = ok ? *reinterpret_cast<const bf16x8*>(dOr + c) : bf16x8{};
      if (ok) {
        const bf16x8 ov = *reinterpret_cast<const bf16x8*>(Or + c);
#pragma unroll
        for (int e = 0; e < 8; ++e) dl += (float)df[qb][ks][e] * (float)ov[e];
      }
    }
    dl += __shfl_xor(dl, 16, 64);
    dl += __shfl_xor(dl, 32, 64);
    del[qb] = dl;
    if (live[qb] && g == 0) a.delta[zh * a.nq + r] = dl;
    lse[qb] = live[qb] ? a.lse[zh * a.nq + r] : 0.f;
    if constexpr (PLAIN) lse[qb] *= FA_LOG2E;
  }
  const float sl2 = a.scale * FA_LOG2E;
  f32x4 dq[D::NDB][2];
#pragma unroll
  for (int db = 0; db < D::NDB; ++db) dq[db][0] = dq[db][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int nkb = (int)((a.nk + FA_KB - 1) / FA_KB);
  __syncthreads();
  for (int kb = 0; kb < nkb; ++kb) {
    const bf16_t* Ks = Kall + kb * FA_KB * D::ROW;
    const bf16_t* Vs = Vall + kb * FA_KB * D::ROW;
    f32x4 ds[4][2];  // dS^T[key 16i + 4g + e][query of block qb]
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      bf16x8 kfr[D::NKS], vfr[D::NKS];
#pragma unroll
      for (int ks = 0; ks < D::NKS; ++ks) {
        kfr[ks] = frag_row<D::ROW>(Ks, i * 16, ks * 32, lane);
        vfr[ks] = frag_row<D::ROW>(Vs, i * 16, ks * 32, lane);
      }
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) {
        f32x4 sv = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < D::NKS; ++ks) {
          sv = mfma(kfr[ks], qf[qb][ks], sv);
          dp = mfma(vfr[ks], df[qb][ks], dp);
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int j = kb * FA_KB + i * 16 + 4 * g + e;
          float dse = 0.f;
          if constexpr (PLAIN) {  // keys past nk are zero rows of the K / V images: no contribution;
            // dS without the scale (applied to dQ once, in the epilogue)
            dse = __builtin_amdgcn_exp2f(sv[e] * sl2 - lse[qb]) * (dp[e] - del[qb]);
          } else if (live[qb]) {
            const FaLogit lg = fa_logit_d(mk, sv[e], tq[qb], j);
            const float pe = lg.x == -INFINITY ? 0.f : __expf(lg.x - lse[qb]);
            dse = pe * (dp[e] - del[qb]) * lg.dxds;
          }
          ds[i][qb][e] = dse;
        }
      }
    }
#pragma unroll
    for (int k2 = 0; k2 < 2; ++k2) {
      const bf16x8 sb0 = pack8(ds[2 * k2][0], ds[2 * k2 + 1][0]);
      const bf16x8 sb1 = pack8(ds[2 * k2][1], ds[2 * k2 + 1][1]);
#pragma unroll
      for (int db = 0; db < D::NDB; ++db) {
        const bf16x8 kt = frag_tr<D::ROW>(Ks, k2 * 32, db * 16, lane);
        dq[db][0] = mfma(kt, sb0, dq[db][0]);
        dq[db][1] = mfma(kt, sb1, dq[db][1]);
      }
    }
  }
#pragma unroll
  for (int qb = 0; qb < 2; ++qb) {
    if (!live[qb]) continue;
    const int64_t r = wave * 32 + qb * 16 + (lane & 15);
    bf16_t* dQ = (bf16_t*)a.dq + b * a.q_bstride + h * a.q_hstride + r * a.ldq;
    const float f = PLAIN ? a.scale : 1.f;
#pragma unroll
    for (int db = 0; db < D::NDB; ++db) {
      const int d = db * 16 + 4 * g;
      if (d < HD)
        *reinterpret_cast<u32x2*>(dQ + d) =
            u32x2{pack2bf(dq[db][qb][0] * f, dq[db][qb][1] * f), pack2bf(dq[db][qb][2] * f, dq[db][qb][3] * f)};
    }
  }
}

// dK, dV: one workgroup per unit, Q / dO / lse / delta resident; wave w owns keys 32w .. 32w + 31,
// their K / V fragments loaded once from global memory into registers
template <int HD, bool PLAIN>
__global__ void __launch_bounds__(FU_NW * 64) flash_bwd_kv_unit_kernel(pz_flash_args a) {
  using D = FaDims<HD>;
  constexpr int NT = FU_NW * 64;
  extern __shared__ __attribute__((aligned(16))) char fa_smem[];
  bf16_t* Qall = reinterpret_cast<bf16_t*>(fa_smem);
  bf16_t* Dall = Qall + FR_MAX * D::ROW;
  float* lse_all = reinterpret_cast<float*>(Dall + FR_MAX * D::ROW);
  float* del_all = lse_all + FR_MAX;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4;
  const int64_t zh = fa_unit_of(a), b = zh / a.H, h = zh % a.H;
  const bf16_t* Q = (const bf16_t*)a.q + b * a.q_bstride + h * a.q_hstride;
  const bf16_t* K = (const bf16_t*)a.k + b * a.k_bstride + h * a.k_hstride;
  const bf16_t* V = (const bf16_t*)a.v + b * a.v_bstride + h * a.v_hstride;
  const FaMask mk(a, b);
  {
    TileStager<HD, D::ROW, FR_MAX, NT> stq, std_;
    stq.load_q(a, Q, b, h, 0, false);
    std_.load_q(a, Q, b, h, 0, true);
    const int tr = threadIdx.x;
    const float lv = tr < FR_MAX && tr < a.nq ? a.lse[zh * a.nq + tr] : 0.f;
    const float dv_ = tr < FR_MAX && tr < a.nq ? a.delta[zh * a.nq + tr] : 0.f;
    zero_pad_cols<HD, D::HDK, D::ROW, FR_MAX, NT>(Qall);
    zero_pad_cols<HD, D::HDK, D::ROW, FR_MAX, NT>(Dall);
    stq.store(Qall);
    std_.store(Dall);
    if (tr < FR_MAX) {
      lse_all[tr] = PLAIN ? lv * FA_LOG2E : lv;
      del_all[tr] = dv_;
    }
  }
  const float sl2 = a.scale * FA_LOG2E;
  // B operands of S = Q K^T / dP = dO V^T: n = key (lane & 15), k = head dim 32 ks + 8g ..
  bf16x8 kfr[2][D::NKS], vfr[2][D::NKS];
  int key[2];
#pragma unroll
  for (int kb2 = 0; kb2 < 2; ++kb2) {
    key[kb2] = wave * 32 + kb2 * 16 + (lane & 15);
#pragma unroll
    for (int ks = 0; ks < D::NKS; ++ks) {
      const int c = ks * 32 + 8 * g;
      const bool ok = key[kb2] < a.nk && c < HD;
      kfr[kb2][ks] = ok ? *reinterpret_cast<const bf16x8*>(K + (int64_t)key[kb2] * a.ldk + c) : bf16x8{};
      vfr[kb2][ks] = ok ? *reinterpret_cast<const bf16x8*>(V + (int64_t)key[kb2] * a.ldv + c) : bf16x8{};
    }
  }
  f32x4 dk[D::NDB][2], dv[D::NDB][2];
#pragma unroll
  for (int db = 0; db < D::NDB; ++db) dk[db][0] = dk[db][1] = dv[db][0] = dv[db][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  __syncthreads();
  const int nqs = (int)((a.nq + FA_QS - 1) / FA_QS);
  for (int qs = 0; qs < nqs; ++qs) {
    const int r0 = qs * FA_QS;
    const bf16_t* Qs = Qall + r0 * D::ROW;
    const bf16_t* Ds = Dall + r0 * D::ROW;
    f32x4 p[2][2], ds[2][2];  // [16-row query block][key block of the wave]
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      float l2r[4], dlr[4];  // this lane's 4 rows of the block (shared by both key blocks)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        l2r[e] = lse_all[r0 + i * 16 + 4 * g + e];
        dlr[e] = del_all[r0 + i * 16 + 4 * g + e];
      }
      bf16x8 qa[D::NKS], da[D::NKS];
#pragma unroll
      for (int ks = 0; ks < D::NKS; ++ks) {
        qa[ks] = frag_row<D::ROW>(Qs, i * 16, ks * 32, lane);
        da[ks] = frag_row<D::ROW>(Ds, i * 16, ks * 32, lane);
      }
#pragma unroll
      for (int kb2 = 0; kb2 < 2; ++kb2) {
        f32x4 sv = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < D::NKS; ++ks) {
          sv = mfma(qa[ks], kfr[kb2][ks], sv);
          dp = mfma(da[ks], vfr[kb2][ks], dp);
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int rr = r0 + i * 16 + 4 * g + e;
          float pe = 0.f, dse = 0.f;
          if constexpr (PLAIN) {  // query rows past nq are zero rows of the Q / dO images: no contribution;
            // dS without the scale (applied to dK once, in the epilogue)
            pe = __builtin_amdgcn_exp2f(sv[e] * sl2 - l2r[e]);
            dse = pe * (dp[e] - dlr[e]);
          } else if (rr < a.nq) {
            const FaLogit lg = fa_logit_d(mk, sv[e], mk.token(rr), key[kb2]);
            pe = lg.x == -INFINITY ? 0.f : __expf(lg.x - l2r[e]);
            dse = pe * (dp[e] - dlr[e]) * lg.dxds;
          }
          p[i][kb2][e] = pe;
          ds[i][kb2][e] = dse;
        }
      }
    }
    const bf16x8 pb0 = pack8(p[0][0], p[1][0]), pb1 = pack8(p[0][1], p[1][1]);
    const bf16x8 sb0 = pack8(ds[0][0], ds[1][0]), sb1 = pack8(ds[0][1], ds[1][1]);
#pragma unroll
    for (int db = 0; db < D::NDB; ++db) {
      const bf16x8 dt = frag_tr<D::ROW>(Ds, 0, db * 16, lane);
      const bf16x8 qt = frag_tr<D::ROW>(Qs, 0, db * 16, lane);
      dv[db][0] = mfma(dt, pb0, dv[db][0]);
      dv[db][1] = mfma(dt, pb1, dv[db][1]);
      dk[db][0] = mfma(qt, sb0, dk[db][0]);
      dk[db][1] = mfma(qt, sb1, dk[db][1]);
    }
  }
#pragma unroll
  for (int kb2 = 0; kb2 < 2; ++kb2) {
    if (key[kb2] >= a.nk) continue;
    bf16_t* dK = (bf16_t*)a.dk + b * a.k_bstride + h * a.k_hstride + (int64_t)key[kb2] * a.ldk;
    bf16_t* dV = (bf16_t*)a.dv + b * a.v_bstride + h * a.v_hstride + (int64_t)key[kb2] * a.ldv;
    const float f = PLAIN ? a.scale : 1.f;
#pragma unroll
    for (int db = 0; db < D::NDB; ++db) {
      const int d = db * 16 + 4 * g;
      if (d < HD) {
        *reinterpret_cast<u32x2*>(dK + d) = u32x2{pack2bf(dk[db][kb2][0] * f, dk[db][kb2][1] * f),
                                                  pack2bf(dk[db][kb2][2] * f, dk[db][kb2][3] * f)};
        *reinterpret_cast<u32x2*>(dV + d) =
            u32x2{pack2bf(dv[db][kb2][0], dv[db][kb2][1]), pack2bf(dv[db][kb2][2], dv[db][kb2][3])};
      }
    }
  }
}

constexpr int FU_SMEM_KV = 2 * FR_MAX * FaDims<72>::ROW * 2 + 2 * FR_MAX * 4;

// ---- SigLIP attention, persistent and pipelined (training: 16 heads x 72, 256 tokens, no mask) ----------
// PMC of the one-workgroup-per-unit kernels above (profiles/r05/pmc_attn_*.json): the waves spend 43-62 % of
// their cycles parked at s_waitcnt / barriers -- each unit's 114 KiB LDS image holds one workgroup per CU, so
// the staging of every unit's resident operand is exposed -- and the forward issues ~7 vector instructions
// per MFMA (mask selects on full key blocks, a separate scale multiply).  Here a grid of one workgroup per CU
// walks its units in turn with the resident operand images double-buffered: LDS-DMA (no VGPR staging) brings
// unit i+1's images while unit i computes.  The images use an 80-element (160-B) row pitch, so two units'
// K and V (or Q and dO) fit the CU's 160 KiB, and both the 16-row ds_read_b128 fragments and the 4-row
// ds_read_b64_tr_b16 fragments are bank-conflict free (row r starts at dword 40 r: 16 consecutive rows tile
// the 64 banks).  Each row's tenth 16-B chunk (head dims 72..79) repeats the ninth (or, in the dK / dV kernel's
// Q / dO images, carries lse / delta): the transposed reads that meet it land in discarded output columns, and
// the 32-wide k step's lanes past dim 71 re-read dims 64..71 of their own row (fs_frag) against zeroed fragments.
// reductions over the 4 lanes l, l ^ 16, l ^ 32, l ^ 48 (the 4 lane groups of a 16 x 16 MFMA column) with gfx950's
// v_permlane16_swap / v_permlane32_swap (VALU, no LDS round trip as __shfl_xor's ds_bpermute); every lane gets the
// same value, combined in the same order
__device__ __forceinline__ float fs_max4(float x) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  x = fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
  const auto r2 = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r2[0]), __uint_as_float(r2[1]));
}
__device__ __forceinline__ float fs_sum4(float x) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  x = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  const auto r2 = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r2[0]) + __uint_as_float(r2[1]);
}

constexpr int FS_N = 256, FS_ROW = 80, FS_IMG = FS_N * FS_ROW * 2, FS_SMEM = 4 * FS_IMG;
constexpr int FS_NW = 8, FS_PER = FS_N * 10 / 64 / FS_NW;  // DMA instructions per wave per image (5)

__device__ __forceinline__ void fs_glds16(const bf16_t* src, char* lds) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}

// ---- dynamic unit assignment of the persistent SigLIP kernels ------------------------------------------------------
// A workgroup takes its next unit from a ticket counter instead of a fixed list, so units flow to whichever CUs run:
// with statically dealt units a workgroup whose CU is held by another stream's kernel (RCCL under data parallelism)
// delays all of its units -- measured x1.7-1.8 for these kernels with 8 or 32 CUs held, against the ideal x1.03 / x1.14
// (tools/contention_probe.py, profiles/r06/contention_r6b.log).  Results per unit do not depend on which workgroup
// computes it, so the output stays bitwise deterministic.
//   * one counter per XCD (workgroup i runs on XCD i % 8): XCD x hands out the units of images x, x + 8, x + 16, ...,
//     ticket k = head k % H of its (k / H)-th image, so the heads of an image run together on one XCD and share its L2
//     (their 144-B q / k / v segments share lines), as the static order did;
//   * wave 0 / lane 0 takes the ticket of the unit after next (inline-asm returning atomic, retired by the vmcnt(0)
//     that ends every unit) and publishes it through 4 bytes of LDS that no read uses -- the tenth 16-B chunk of row
//     0 (K image; the dK / dV kernel: row 1 of the Q image, whose chunk carries an lse copy nobody reads), whose only
//     readers are the transposed reads of head dims 72..79 into discarded output rows -- before the barrier that ends
//     the unit;
//   * self-resetting: every workgroup takes tickets until one is past its XCD's units, so exactly units_x + G_x tickets
//     are handed out; the workgroup that receives the last one resets the counter for the next launch (stream order,
//     hipGraph replays included).  The kernels must not run concurrently with themselves (the engine runs SigLIP on
//     one stream).
__device__ unsigned g_fs_ctr[3][8];  // [kernel: 0 fwd, 1 dQ, 2 dK / dV][XCD]

struct FsTickets {
  unsigned* ctr;
  int64_t units_x, units;
  unsigned last;
  int x, nx, H;
  __device__ __forceinline__ FsTickets(const pz_flash_args& a, int kind) {
    const int G = (int)gridDim.x;
    nx = G % 8 == 0 ? 8 : 1;
    x = (int)blockIdx.x % nx;
    H = (int)a.H;
    units = a.Z * a.H;
    const int64_t zx = nx == 8 ? (a.Z > x ? (a.Z - x + 7) / 8 : 0) : a.Z;
    units_x = zx * a.H;
    last = (unsigned)(units_x + G / nx - 1);
    ctr = &g_fs_ctr[kind][x];
  }
  // unit of ticket k (>= units: no more work)
  __device__ __forceinline__ int64_t unit(unsigned k) const {
    if ((int64_t)k >= units_x) return units;
    return nx == 8 ? ((int64_t)(k / H) * 8 + x) * H + k % H : (int64_t)k;
  }
  // wave 0 / lane 0: take a ticket (returning atomic; the result lands with the caller's next vmcnt(0))
  __device__ __forceinline__ void take(unsigned& tk) const {
    asm volatile("global_atomic_add %0, %1, %2, off sc0" : "=v"(tk) : "v"(ctr), "v"(1u) : "memory");
  }
  // wave 0 / lane 0, after a vmcnt(0): publish the ticket to the slot; the receiver of the last ticket resets
  __device__ __forceinline__ void publish(unsigned& tk, char* slot) const {
    asm volatile("" : "+v"(tk));
    if (tk == last) asm volatile("global_store_dword %0, %1, off sc1" ::"v"(ctr), "v"(0u) : "memory");  // agent scope
    // (LDS by inline asm: a C++ store through the generic pointer compiles to a flat store, counted by vmcnt too)
    asm volatile("ds_write_b32 %0, %1" ::"v"((unsigned)(size_t)(__attribute__((address_space(3))) char*)slot), "v"(tk)
                 : "memory");
  }
  __device__ __forceinline__ unsigned read(const char* slot) const {
    unsigned v;
    asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)"
                 : "=v"(v)
                 : "v"((unsigned)(size_t)(const __attribute__((address_space(3))) char*)slot)
                 : "memory");
    return __builtin_amdgcn_readfirstlane(v);
  }
};
constexpr int FS_SLOT0 = 9 * 16;             // byte offset of row 0's tenth chunk in an image
constexpr int FS_SLOT1 = FS_ROW * 2 + 9 * 16;  // ... of row 1's

// per-lane element offsets of this wave's FS_PER DMA pieces of a [256][72] operand with row stride ld
__device__ __forceinline__ void fs_dma_offsets(int64_t ld, int wave, int lane, int (&off)[FS_PER]) {
#pragma unroll
  for (int s = 0; s < FS_PER; ++s) {
    const int c = (wave * FS_PER + s) * 64 + lane, row = c / 10, ch = c % 10;
    off[s] = row * (int)ld + 8 * (ch < 9 ? ch : 8);
  }
}

__device__ __forceinline__ void fs_dma(const bf16_t* base, const int (&off)[FS_PER], char* img, int wave) {
#pragma unroll
  for (int s = 0; s < FS_PER; ++s) fs_glds16(base + off[s], img + (wave * FS_PER + s) * 1024);
}

#define FS_WAIT_VM(n) asm volatile("s_waitcnt vmcnt(" #n ")" ::: "memory")

// 16-row fragment of a resident image (80-element rows), k step ks of the 72-dim contraction.  At ks 2 every lane
// group reads head dims 64..71 of its OWN row: groups g >= 1 stand for dims 72..95, which the other operand zeroes, so
// only finite, landed bytes may meet those zeros.  (Reading on past dim 79 runs into the NEXT row -- for row 255 of
// the second image of a buffer that is the other buffer's first image, whose DMA may still be in flight or which may
// hold stale LDS of an earlier kernel on this CU: 0 x NaN = NaN.  Round 5's dQ kernel did exactly that.)
__device__ __forceinline__ bf16x8 fs_frag(const bf16_t* T, int r0, int ks, int lane) {
  return *reinterpret_cast<const bf16x8*>(T + (r0 + (lane & 15)) * FS_ROW + (ks < 2 ? ks * 32 + 8 * (lane >> 4) : 64));
}

// ds_read_b64_tr_b16 by inline asm: NOT counted by hipcc's lgkmcnt tracking -- the caller waits with an asm
// that names the result (see the forward's V^T fragments)
template <int OFF>  // byte offset folded into the instruction
__device__ __forceinline__ s16x4 fs_tr(unsigned lds_addr) {
  s16x4 v;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(v) : "v"(lds_addr), "i"(OFF));
  return v;
}
__device__ __forceinline__ unsigned fs_lds_addr(const void* p) {
  return (unsigned)(size_t)(const __attribute__((address_space(3))) char*)p;
}
__device__ __forceinline__ bf16x8 fs_cat(const s16x4& a, const s16x4& b) {
  s16x8 o;
  o[0] = a[0]; o[1] = a[1]; o[2] = a[2]; o[3] = a[3];
  o[4] = b[0]; o[5] = b[1]; o[6] = b[2]; o[7] = b[3];
  return __builtin_bit_cast(bf16x8, o);
}
// workgroup barrier without __syncthreads()'s release fence (which drains vmcnt, i.e. the next unit's
// LDS-DMA): this wave's LDS reads are done (lgkmcnt) and its DMA pieces waited for by FS_WAIT_VM
#define FS_BARRIER()                                   \
  do {                                                 \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); \
    __builtin_amdgcn_s_barrier();                      \
    asm volatile("" ::: "memory");                     \
  } while (0)

// forward: QB 16-row query blocks per wave (QB = 2: 8 waves, two blocks share each K / V fragment read, 2 waves per
// SIMD; QB = 1: 16 waves of 16 rows, 4 waves per SIMD at <= 128 VGPRs -- twice the LDS fragment reads per MFMA but
// twice the waves to hide the softmax chains and LDS latencies); log2-domain online softmax over four 64-key blocks
// with the scale folded into the exponent's FMA (max over raw scores: scale > 0)
template <int QB>
__global__ void __launch_bounds__(16 / QB * 64, 1) flash_fwd_sig_kernel(pz_flash_args a, int G) {
  constexpr int NW = 16 / QB;
  extern __shared__ __attribute__((aligned(16))) char fa_smem[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4;
  const int64_t units = a.Z * a.H;
  // DMA pieces: QB = 2 -- each wave 5 pieces of K and 5 of V; QB = 1 -- waves 0..7 the K image, 8..15 the V image
  int offk[FS_PER], offv[FS_PER];
  fs_dma_offsets(QB == 1 && wave >= 8 ? a.ldv : a.ldk, wave & 7, lane, offk);
  fs_dma_offsets(a.ldv, wave & 7, lane, offv);
  const float sl2 = a.scale * FA_LOG2E;
  // Pipeline (per workgroup, unit t in buffer t & 1): the Q fragments of unit t + 1 (inline-asm loads into
  // qn: hipcc would drain every in-flight LDS-DMA with vmcnt(0) at the first use of an ordinary load) and its
  // K / V images are issued before unit t's compute; one vmcnt(0) after the compute (long landed by then),
  // before unit t's O stores, and the barrier that ends unit t publish them, so no wait stalls in steady state.
  (void)G;
  const FsTickets tix(a, 0);
  const bool w0 = wave == 0 && lane == 0;
  unsigned tk = 0;
  bf16x8 qn[QB][3];
  auto issue = [&](int64_t un, int t1) {  // Q fragments + K / V images of unit un into buffer t1 & 1
    const int64_t bn = un / a.H, hn = un % a.H;
    const bf16_t* Q = (const bf16_t*)a.q + bn * a.q_bstride + hn * a.q_hstride;
#pragma unroll
    for (int qb = 0; qb < QB; ++qb)
#pragma unroll
      for (int ks = 0; ks < 3; ++ks) {  // head dims 72..95 (g >= 1 at ks 2) re-read dims 64..71, zeroed below
        const bf16_t* src =
            Q + (wave * 16 * QB + qb * 16 + (lane & 15)) * a.ldq + (ks < 2 || g == 0 ? ks * 32 + 8 * g : 64);
        asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(qn[qb][ks]) : "v"(src) : "memory");
      }
    char* nxt = fa_smem + (t1 & 1) * 2 * FS_IMG;
    const bf16_t* Kn = (const bf16_t*)a.k + bn * a.k_bstride + hn * a.k_hstride;
    const bf16_t* Vn = (const bf16_t*)a.v + bn * a.v_bstride + hn * a.v_hstride;
    if constexpr (QB == 2) {
      fs_dma(Kn, offk, nxt, wave);
      fs_dma(Vn, offv, nxt + FS_IMG, wave);
    } else {
      fs_dma(wave < 8 ? Kn : Vn, offk, nxt + (wave < 8 ? 0 : FS_IMG), wave & 7);
    }
  };
  // the first unit's ticket through buffer 1's slot (no DMA reaches buffer 1 before the loop), the second's through
  // buffer 0's (after wave 0's own DMA of that chunk landed)
  if (w0) tix.take(tk);
  FS_WAIT_VM(0);
  if (w0) tix.publish(tk, fa_smem + 2 * FS_IMG + FS_SLOT0);
  FS_BARRIER();
  int64_t u = tix.unit(tix.read(fa_smem + 2 * FS_IMG + FS_SLOT0));
  if (u < units) {
    issue(u, 0);
    if (w0) tix.take(tk);
  }
  FS_WAIT_VM(0);
  if (u < units && w0) tix.publish(tk, fa_smem + FS_SLOT0);
  FS_BARRIER();
  for (int t = 0; u < units; ++t) {
    const int64_t b = u / a.H, h = u % a.H;
    bf16x8 qf[QB][3];
#pragma unroll
    for (int qb = 0; qb < QB; ++qb) {
#pragma unroll
      for (int ks = 0; ks < 3; ++ks) {
        asm volatile("" : "+v"(qn[qb][ks]));  // landed (the vmcnt(0) before the previous barrier)
        qf[qb][ks] = qn[qb][ks];
      }
      if (g != 0) qf[qb][2] = bf16x8{};
    }
    const int64_t un = tix.unit(tix.read(fa_smem + (t & 1) * 2 * FS_IMG + FS_SLOT0));  // uniform
    if (un < units) {
      issue(un, t + 1);
      if (w0) tix.take(tk);  // the unit after next
    }
    const char* cur = fa_smem + (t & 1) * 2 * FS_IMG;
    const bf16_t* Kall = reinterpret_cast<const bf16_t*>(cur);
    const bf16_t* Vall = reinterpret_cast<const bf16_t*>(cur + FS_IMG);
    f32x4 o[5][QB];
#pragma unroll
    for (int db = 0; db < 5; ++db)
#pragma unroll
      for (int qb = 0; qb < QB; ++qb) o[db][qb] = f32x4{0.f, 0.f, 0.f, 0.f};
    float m[QB], l[QB];  // m: running max of the RAW scores
#pragma unroll
    for (int qb = 0; qb < QB; ++qb) {
      m[qb] = -INFINITY;
      l[qb] = 0.f;
    }
    // software pipeline over the four 64-key blocks: block kb + 1's S MFMAs are issued before block kb's softmax
    // (independent vector work the SIMD issues while they run), then block kb's P V
    auto scores = [&](int kb, f32x4 (&sc)[4][QB]) {
      const bf16_t* Ks = Kall + kb * FA_KB * FS_ROW;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int qb = 0; qb < QB; ++qb) sc[i][qb] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 3; ++ks)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const bf16x8 kf = fs_frag(Ks, i * 16, ks, lane);
#pragma unroll
          for (int qb = 0; qb < QB; ++qb) sc[i][qb] = mfma(kf, qf[qb][ks], sc[i][qb]);
        }
    };
    auto soft_pv = [&](int kb, f32x4 (&sc)[4][QB]) {
      const bf16_t* Vs = Vall + kb * FA_KB * FS_ROW;
      bf16x8 pf[2][QB];  // [k-step of 32 keys][query block]
#pragma unroll
      for (int qb = 0; qb < QB; ++qb) {
        float mx = fmaxf(fmaxf(sc[0][qb][0], sc[0][qb][1]), fmaxf(sc[0][qb][2], sc[0][qb][3]));
#pragma unroll
        for (int i = 1; i < 4; ++i)
          mx = fmaxf(fmaxf(mx, fmaxf(sc[i][qb][0], sc[i][qb][1])), fmaxf(sc[i][qb][2], sc[i][qb][3]));
        mx = fs_max4(mx);
        const float mn = fmaxf(m[qb], mx), nb = -mn * sl2;
        const float alpha = __builtin_amdgcn_exp2f((m[qb] - mn) * sl2);  // exp2(-inf) = 0 on the first block
        float sum = 0.f;
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float pv = __builtin_amdgcn_exp2f(fmaf(sc[i][qb][e], sl2, nb));
            sc[i][qb][e] = pv;
            sum += pv;
          }
        sum = fs_sum4(sum);
        l[qb] = fmaf(l[qb], alpha, sum);
        m[qb] = mn;
#pragma unroll
        for (int db = 0; db < 5; ++db) o[db][qb] *= alpha;
        pf[0][qb] = pack8(sc[0][qb], sc[1][qb]);
        pf[1][qb] = pack8(sc[2][qb], sc[3][qb]);
      }
      // V^T fragments by inline-asm transposed reads (with the builtin hipcc drains the in-flight LDS-DMA
      // before each); the waits name the fragments so the consuming MFMAs stay behind them
      const unsigned va = fs_lds_addr(Vs + (4 * g + ((lane & 15) >> 2)) * FS_ROW + 4 * (lane & 3));
#pragma unroll
      for (int k2 = 0; k2 < 2; ++k2) {
        s16x4 tv[5][2];
        if (k2 == 0) {
#define FS_TR(db, hf) tv[db][hf] = fs_tr<(16 * (hf)) * FS_ROW * 2 + (db) * 32>(va)
          FS_TR(0, 0); FS_TR(0, 1); FS_TR(1, 0); FS_TR(1, 1); FS_TR(2, 0); FS_TR(2, 1); FS_TR(3, 0); FS_TR(3, 1);
          FS_TR(4, 0); FS_TR(4, 1);
#undef FS_TR
        } else {
#define FS_TR(db, hf) tv[db][hf] = fs_tr<(32 + 16 * (hf)) * FS_ROW * 2 + (db) * 32>(va)
          FS_TR(0, 0); FS_TR(0, 1); FS_TR(1, 0); FS_TR(1, 1); FS_TR(2, 0); FS_TR(2, 1); FS_TR(3, 0); FS_TR(3, 1);
          FS_TR(4, 0); FS_TR(4, 1);
#undef FS_TR
        }
        asm volatile("s_waitcnt lgkmcnt(0)"
                     : "+v"(tv[0][0]), "+v"(tv[0][1]), "+v"(tv[1][0]), "+v"(tv[1][1]), "+v"(tv[2][0]), "+v"(tv[2][1]),
                       "+v"(tv[3][0]), "+v"(tv[3][1]), "+v"(tv[4][0]), "+v"(tv[4][1]));
#pragma unroll
        for (int db = 0; db < 5; ++db) {
          const bf16x8 vf = fs_cat(tv[db][0], tv[db][1]);
#pragma unroll
          for (int qb = 0; qb < QB; ++qb) o[db][qb] = mfma(vf, pf[k2][qb], o[db][qb]);
        }
      }
    };
    f32x4 scA[4][QB], scB[4][QB];
    scores(0, scA);
    scores(1, scB);
    soft_pv(0, scA);
    scores(2, scA);
    soft_pv(1, scB);
    scores(3, scB);
    soft_pv(2, scA);
    soft_pv(3, scB);
    FS_WAIT_VM(0);  // the next unit's Q fragments and images (issued before this unit's compute)
#pragma unroll
    for (int qb = 0; qb < QB; ++qb) {  // one output group (host-checked)
      const int64_t rq = wave * 16 * QB + qb * 16 + (lane & 15);
      const float inv = 1.f / l[qb];
      bf16_t* O = (bf16_t*)a.g_o[0] + b * a.g_bstride[0] + rq * a.g_ld[0] + h * a.o_hstride;
#pragma unroll
      for (int db = 0; db < 5; ++db) {
        const int d = db * 16 + 4 * g;
        if (d < 72)
          *reinterpret_cast<u32x2*>(O + d) =
              u32x2{pack2bf(o[db][qb][0] * inv, o[db][qb][1] * inv), pack2bf(o[db][qb][2] * inv, o[db][qb][3] * inv)};
      }
      if (g == 0 && a.lse) a.lse[u * FS_N + rq] = m[qb] * a.scale + __logf(l[qb]);
    }
    if (un < units && w0) tix.publish(tk, fa_smem + ((t + 1) & 1) * 2 * FS_IMG + FS_SLOT0);
    FS_BARRIER();  // this buffer's readers are done; the next unit's pieces landed in every wave
    u = un;
  }
}

// row fragment loads (Q / dO / O rows of one 16-row block) by inline asm; head dims 72..95 (g >= 1 at
// ks 2) re-read dims 64..71 and are zeroed by the consumer
__device__ __forceinline__ void fs_load_rows(bf16x8 (&f)[3], const bf16_t* row, int g) {
#pragma unroll
  for (int ks = 0; ks < 3; ++ks) {
    const bf16_t* src = row + (ks < 2 || g == 0 ? ks * 32 + 8 * g : 64);
    asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(f[ks]) : "v"(src) : "memory");
  }
}

// dQ with K / V resident (delta = rowsum(dO O) from flash_bwd_prep_kernel): wave w owns query rows 32w ..
// 32w + 31; the next unit's Q / dO rows, lse and delta (inline-asm loads) and K / V images (LDS-DMA) are issued
// before this unit's compute
template <bool DELTA>  // DELTA: delta = rowsum(dO O) computed here from O rows loaded at the unit's start (and written
                       // for the dK / dV pass) instead of read from flash_delta72_kernel's output
__global__ void __launch_bounds__(FS_NW * 64, 1) flash_bwd_q_sig_kernel(pz_flash_args a, int G) {
  extern __shared__ __attribute__((aligned(16))) char fa_smem[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4;
  const int64_t units = a.Z * a.H;
  int offk[FS_PER], offv[FS_PER];
  fs_dma_offsets(a.ldk, wave, lane, offk);
  fs_dma_offsets(a.ldv, wave, lane, offv);
  const float sl2 = a.scale * FA_LOG2E;
  (void)G;
  const FsTickets tix(a, 1);
  const bool w0 = wave == 0 && lane == 0;
  unsigned tk = 0;
  bf16x8 qn[2][3], dn[2][3];
  float ln[2], dln[2];
  auto issue = [&](int64_t un, int t1) {
    const int64_t bn = un / a.H, hn = un % a.H;
    const bf16_t* Q = (const bf16_t*)a.q + bn * a.q_bstride + hn * a.q_hstride;
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) {
      const int64_t r = wave * 32 + qb * 16 + (lane & 15);
      fs_load_rows(qn[qb], Q + r * a.ldq, g);
      fs_load_rows(dn[qb], (const bf16_t*)a.g_do[0] + bn * a.g_bstride[0] + r * a.g_ld[0] + hn * a.o_hstride, g);
      asm volatile("global_load_dword %0, %1, off" : "=v"(ln[qb]) : "v"(a.lse + un * FS_N + r) : "memory");
      if (!DELTA) asm volatile("global_load_dword %0, %1, off" : "=v"(dln[qb]) : "v"(a.delta + un * FS_N + r) : "memory");
    }
    char* nxt = fa_smem + (t1 & 1) * 2 * FS_IMG;
    fs_dma((const bf16_t*)a.k + bn * a.k_bstride + hn * a.k_hstride, offk, nxt, wave);
    fs_dma((const bf16_t*)a.v + bn * a.v_bstride + hn * a.v_hstride, offv, nxt + FS_IMG, wave);
  };
  if (w0) tix.take(tk);  // the first two tickets as in the forward
  FS_WAIT_VM(0);
  if (w0) tix.publish(tk, fa_smem + 2 * FS_IMG + FS_SLOT0);
  FS_BARRIER();
  int64_t u = tix.unit(tix.read(fa_smem + 2 * FS_IMG + FS_SLOT0));
  if (u < units) {
    issue(u, 0);
    if (w0) tix.take(tk);
  }
  FS_WAIT_VM(0);
  if (u < units && w0) tix.publish(tk, fa_smem + FS_SLOT0);
  FS_BARRIER();
  for (int t = 0; u < units; ++t) {
    const int64_t b = u / a.H, h = u % a.H;
    const int64_t un = tix.unit(tix.read(fa_smem + (t & 1) * 2 * FS_IMG + FS_SLOT0));  // uniform
    bf16x8 qf[2][3], df[2][3];
    float del[2], lse2[2];
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) {
#pragma unroll
      for (int ks = 0; ks < 3; ++ks) {
        asm volatile("" : "+v"(qn[qb][ks]), "+v"(dn[qb][ks]));  // landed (vmcnt(0) + barrier)
        qf[qb][ks] = qn[qb][ks];
        df[qb][ks] = dn[qb][ks];
      }
      if (g != 0) qf[qb][2] = df[qb][2] = bf16x8{};
      asm volatile("" : "+v"(ln[qb]), "+v"(dln[qb]));
      lse2[qb] = ln[qb] * FA_LOG2E;
      del[qb] = dln[qb];
    }
    if constexpr (DELTA) {  // O rows by ordinary loads, before the next unit's DMA is issued (nothing else in flight)
#pragma unroll
      for (int qb = 0; qb < 2; ++qb) {
        const int64_t r = wave * 32 + qb * 16 + (lane & 15);
        const bf16_t* Or = (const bf16_t*)a.g_o[0] + b * a.g_bstride[0] + r * a.g_ld[0] + h * a.o_hstride;
        float dl = 0.f;
        bf16x8 ov[3];
#pragma unroll
        for (int ks = 0; ks < 3; ++ks)  // dims 72..95 re-read 64..71 against the zeroed dO fragment (no branch)
          ov[ks] = *reinterpret_cast<const bf16x8*>(Or + (ks < 2 || g == 0 ? ks * 32 + 8 * g : 64));
#pragma unroll
        for (int ks = 0; ks < 3; ++ks)
#pragma unroll
          for (int e = 0; e < 8; ++e) dl = fmaf((float)df[qb][ks][e], (float)ov[ks][e], dl);
        dl = fs_sum4(dl);
        del[qb] = dl;
        if (g == 0) a.delta[u * FS_N + r] = dl;
      }
    }
    if (un < units) {
      issue(un, t + 1);
      if (w0) tix.take(tk);
    }
    const char* cur = fa_smem + (t & 1) * 2 * FS_IMG;
    const bf16_t* Kall = reinterpret_cast<const bf16_t*>(cur);
    const bf16_t* Vall = reinterpret_cast<const bf16_t*>(cur + FS_IMG);
    f32x4 dq[5][2];
#pragma unroll
    for (int db = 0; db < 5; ++db) dq[db][0] = dq[db][1] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
    for (int kb = 0; kb < FS_N / FA_KB; ++kb) {
      const bf16_t* Ks = Kall + kb * FA_KB * FS_ROW;
      const bf16_t* Vs = Vall + kb * FA_KB * FS_ROW;
      const unsigned ka = fs_lds_addr(Ks + (4 * g + ((lane & 15) >> 2)) * FS_ROW + 4 * (lane & 3));
#pragma unroll
      for (int k2 = 0; k2 < 2; ++k2) {
        f32x4 dsv[2][2];  // dS^T (without the scale) [16-key block of the k-step][query block]
#pragma unroll
        for (int i2 = 0; i2 < 2; ++i2) {
          const int i = 2 * k2 + i2;
          bf16x8 kfr[3], vfr[3];
#pragma unroll
          for (int ks = 0; ks < 3; ++ks) {
            kfr[ks] = fs_frag(Ks, i * 16, ks, lane);
            vfr[ks] = fs_frag(Vs, i * 16, ks, lane);
          }
#pragma unroll
          for (int qb = 0; qb < 2; ++qb) {
            f32x4 sv = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int ks = 0; ks < 3; ++ks) {
              sv = mfma(kfr[ks], qf[qb][ks], sv);
              dp = mfma(vfr[ks], df[qb][ks], dp);
            }
#pragma unroll
            for (int e = 0; e < 4; ++e)
              dsv[i2][qb][e] = __builtin_amdgcn_exp2f(fmaf(sv[e], sl2, -lse2[qb])) * (dp[e] - del[qb]);
          }
        }
        const bf16x8 sb0 = pack8(dsv[0][0], dsv[1][0]), sb1 = pack8(dsv[0][1], dsv[1][1]);
        // dQ^T += K^T dS^T over these 32 keys: K^T fragments by inline-asm transposed reads (see the forward)
        s16x4 tk[5][2];
#define FS_TR(db, hf) tk[db][hf] = fs_tr<(16 * (hf)) * FS_ROW * 2 + (db) * 32>(ka + k2 * 32 * FS_ROW * 2)
        FS_TR(0, 0); FS_TR(0, 1); FS_TR(1, 0); FS_TR(1, 1); FS_TR(2, 0); FS_TR(2, 1); FS_TR(3, 0); FS_TR(3, 1);
        FS_TR(4, 0); FS_TR(4, 1);
#undef FS_TR
        asm volatile("s_waitcnt lgkmcnt(0)"
                     : "+v"(tk[0][0]), "+v"(tk[0][1]), "+v"(tk[1][0]), "+v"(tk[1][1]), "+v"(tk[2][0]), "+v"(tk[2][1]),
                       "+v"(tk[3][0]), "+v"(tk[3][1]), "+v"(tk[4][0]), "+v"(tk[4][1]));
#pragma unroll
        for (int db = 0; db < 5; ++db) {
          const bf16x8 kt = fs_cat(tk[db][0], tk[db][1]);
          dq[db][0] = mfma(kt, sb0, dq[db][0]);
          dq[db][1] = mfma(kt, sb1, dq[db][1]);
        }
      }
    }
    FS_WAIT_VM(0);  // the next unit's rows and images (issued before this unit's compute)
#pragma unroll
    for (int qb = 0; qb < 2; ++qb) {
      const int64_t r = wave * 32 + qb * 16 + (lane & 15);
      bf16_t* dQ = (bf16_t*)a.dq + b * a.q_bstride + h * a.q_hstride + r * a.ldq;
#pragma unroll
      for (int db = 0; db < 5; ++db) {
        const int d = db * 16 + 4 * g;
        if (d < 72)
          *reinterpret_cast<u32x2*>(dQ + d) = u32x2{pack2bf(dq[db][qb][0] * a.scale, dq[db][qb][1] * a.scale),
                                                    pack2bf(dq[db][qb][2] * a.scale, dq[db][qb][3] * a.scale)};
      }
    }
    if (un < units && w0) tix.publish(tk, fa_smem + ((t + 1) & 1) * 2 * FS_IMG + FS_SLOT0);
    FS_BARRIER();
    u = un;
  }
}

// dK, dV with Q and dO resident: wave w owns keys 32w .. 32w + 31 and sweeps the unit's query rows in steps of
// 32.  Each Q / dO image row's tenth chunk carries lse / delta instead (rows 4j .. 4j + 3 of the row's group of
// four, so a lane's four rows of a 16-row block come with ONE 16-B read); the head-dim-72..95 fragments that
// would meet them are zeroed after the read.  The next unit's K / V fragments (inline-asm loads) and images
// (LDS-DMA) are issued before this unit's compute.
__global__ void __launch_bounds__(FS_NW * 64, 1) flash_bwd_kv_sig_kernel(pz_flash_args a, int G) {
  extern __shared__ __attribute__((aligned(16))) char fa_smem[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4;
  const int64_t units = a.Z * a.H;
  int offq[FS_PER], offd[FS_PER], offl[FS_PER];
  bool side[FS_PER];
  {
    const FaRow fr{&a};
    (void)fr;
#pragma unroll
    for (int s2 = 0; s2 < FS_PER; ++s2) {
      const int c = (wave * FS_PER + s2) * 64 + lane, row = c / 10, ch = c % 10;
      side[s2] = ch == 9;
      offq[s2] = row * (int)a.ldq + 8 * (ch < 9 ? ch : 0);
      offd[s2] = row * (int)a.g_ld[0] + 8 * (ch < 9 ? ch : 0);
      offl[s2] = row & ~3;
    }
  }
  const float sl2 = a.scale * FA_LOG2E;
  (void)G;
  const FsTickets tix(a, 2);
  const bool w0 = wave == 0 && lane == 0;
  unsigned tk = 0;
  bf16x8 kfr[2][3], vfr[2][3];
  // the wave's K / V fragments of unit un (inline-asm loads into kfr / vfr): issued in the last query step of
  // the previous unit, right after the last products that read kfr / vfr
  auto issue_kv = [&](int64_t un) {
    const int64_t bn = un / a.H, hn = un % a.H;
    const bf16_t* K = (const bf16_t*)a.k + bn * a.k_bstride + hn * a.k_hstride;
    const bf16_t* V = (const bf16_t*)a.v + bn * a.v_bstride + hn * a.v_hstride;
#pragma unroll
    for (int kb2 = 0; kb2 < 2; ++kb2) {
      const int key = wave * 32 + kb2 * 16 + (lane & 15);
      fs_load_rows(kfr[kb2], K + key * a.ldk, g);
      fs_load_rows(vfr[kb2], V + key * a.ldv, g);
    }
  };
  auto issue = [&](int64_t un, int t1) {  // the Q / dO (+ lse / delta) images of unit un into buffer t1 & 1
    const int64_t bn = un / a.H, hn = un % a.H;
    const bf16_t* Q = (const bf16_t*)a.q + bn * a.q_bstride + hn * a.q_hstride;
    const bf16_t* dO = (const bf16_t*)a.g_do[0] + bn * a.g_bstride[0] + hn * a.o_hstride;
    const float* L = a.lse + un * FS_N;
    const float* D = a.delta + un * FS_N;
    char* nxt = fa_smem + (t1 & 1) * 2 * FS_IMG;
#pragma unroll
    for (int s2 = 0; s2 < FS_PER; ++s2)
      fs_glds16(side[s2] ? (const bf16_t*)(L + offl[s2]) : Q + offq[s2], nxt + (wave * FS_PER + s2) * 1024);
#pragma unroll
    for (int s2 = 0; s2 < FS_PER; ++s2)
      fs_glds16(side[s2] ? (const bf16_t*)(D + offl[s2]) : dO + offd[s2], nxt + FS_IMG + (wave * FS_PER + s2) * 1024);
  };
  // tickets through row 1's tenth chunk of the Q image (an lse copy that no read uses)
  if (w0) tix.take(tk);
  FS_WAIT_VM(0);
  if (w0) tix.publish(tk, fa_smem + 2 * FS_IMG + FS_SLOT1);
  FS_BARRIER();
  int64_t u = tix.unit(tix.read(fa_smem + 2 * FS_IMG + FS_SLOT1));
  if (u < units) {
    issue_kv(u);
    issue(u, 0);
    if (w0) tix.take(tk);
  }
  FS_WAIT_VM(0);
  if (u < units && w0) tix.publish(tk, fa_smem + FS_SLOT1);
  FS_BARRIER();
  for (int t = 0; u < units; ++t) {
    const int64_t b = u / a.H, h = u % a.H;
#pragma unroll
    for (int kb2 = 0; kb2 < 2; ++kb2) {
#pragma unroll
      for (int ks = 0; ks < 3; ++ks) asm volatile("" : "+v"(kfr[kb2][ks]), "+v"(vfr[kb2][ks]));  // landed
      if (g != 0) kfr[kb2][2] = vfr[kb2][2] = bf16x8{};
    }
    const int64_t un = tix.unit(tix.read(fa_smem + (t & 1) * 2 * FS_IMG + FS_SLOT1));  // uniform
    if (un < units) {
      issue(un, t + 1);
      if (w0) tix.take(tk);
    }
    const char* cur = fa_smem + (t & 1) * 2 * FS_IMG;
    const bf16_t* Qall = reinterpret_cast<const bf16_t*>(cur);
    const bf16_t* Dall = reinterpret_cast<const bf16_t*>(cur + FS_IMG);
    f32x4 dk[5][2], dv[5][2];
#pragma unroll
    for (int db = 0; db < 5; ++db) dk[db][0] = dk[db][1] = dv[db][0] = dv[db][1] = f32x4{0.f, 0.f, 0.f, 0.f};
    auto step = [&](int qs, bool last) {
      const int r0 = qs * FA_QS;
      const bf16_t* Qs = Qall + r0 * FS_ROW;
      const bf16_t* Ds = Dall + r0 * FS_ROW;
      unsigned pp[2][2][2], dd[2][2][2];  // bf16 pairs of P / dS [16-row query block][key block][pair]
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        // lse / delta of rows r0 + 16 i + 4g .. + 3 from the tenth chunk of row r0 + 16 i + 4g
        const f32x4 l2r = *reinterpret_cast<const f32x4*>(Qs + (i * 16 + 4 * g) * FS_ROW + 72) * FA_LOG2E;
        const f32x4 dlr = *reinterpret_cast<const f32x4*>(Ds + (i * 16 + 4 * g) * FS_ROW + 72);
        bf16x8 qa[3], da[3];
#pragma unroll
        for (int ks = 0; ks < 3; ++ks) {
          qa[ks] = fs_frag(Qs, i * 16, ks, lane);
          da[ks] = fs_frag(Ds, i * 16, ks, lane);
        }
        // (dims 72..95: these lanes re-read dims 64..71 of their own row -- finite -- against the zeroed kfr / vfr)
#pragma unroll
        for (int kb2 = 0; kb2 < 2; ++kb2) {
          f32x4 sv = {0.f, 0.f, 0.f, 0.f}, dp = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int ks = 0; ks < 3; ++ks) {
            sv = mfma(qa[ks], kfr[kb2][ks], sv);
            dp = mfma(da[ks], vfr[kb2][ks], dp);
          }
          float pe[4], de[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            pe[e] = __builtin_amdgcn_exp2f(fmaf(sv[e], sl2, -l2r[e]));
            de[e] = pe[e] * (dp[e] - dlr[e]);  // dS without the scale (applied to dK once)
          }
          pp[i][kb2][0] = pack2bf(pe[0], pe[1]);
          pp[i][kb2][1] = pack2bf(pe[2], pe[3]);
          dd[i][kb2][0] = pack2bf(de[0], de[1]);
          dd[i][kb2][1] = pack2bf(de[2], de[3]);
        }
      }
      if (last && un < units) issue_kv(un);  // kfr / vfr are dead from here on in this unit
      auto cat4 = [](unsigned x0, unsigned x1, unsigned x2, unsigned x3) {
        return __builtin_bit_cast(bf16x8, u32x4{x0, x1, x2, x3});
      };
      const bf16x8 pb0 = cat4(pp[0][0][0], pp[0][0][1], pp[1][0][0], pp[1][0][1]);
      const bf16x8 pb1 = cat4(pp[0][1][0], pp[0][1][1], pp[1][1][0], pp[1][1][1]);
      const bf16x8 sb0 = cat4(dd[0][0][0], dd[0][0][1], dd[1][0][0], dd[1][0][1]);
      const bf16x8 sb1 = cat4(dd[0][1][0], dd[0][1][1], dd[1][1][0], dd[1][1][1]);
      // dV^T += dO^T P, dK^T += Q^T dS: dO^T / Q^T fragments by inline-asm transposed reads (see the forward)
      const unsigned da0 = fs_lds_addr(Ds + (4 * g + ((lane & 15) >> 2)) * FS_ROW + 4 * (lane & 3));
      const unsigned qa0 = fs_lds_addr(Qs + (4 * g + ((lane & 15) >> 2)) * FS_ROW + 4 * (lane & 3));
      s16x4 td[5][2], tq[5][2];
#define FS_TR(db, hf)                                             \
  td[db][hf] = fs_tr<(16 * (hf)) * FS_ROW * 2 + (db) * 32>(da0); \
  tq[db][hf] = fs_tr<(16 * (hf)) * FS_ROW * 2 + (db) * 32>(qa0)
#define FS_MM(db)                                                                \
  {                                                                              \
    const bf16x8 dt = fs_cat(td[db][0], td[db][1]), qt = fs_cat(tq[db][0], tq[db][1]); \
    dv[db][0] = mfma(dt, pb0, dv[db][0]);                                        \
    dv[db][1] = mfma(dt, pb1, dv[db][1]);                                        \
    dk[db][0] = mfma(qt, sb0, dk[db][0]);                                        \
    dk[db][1] = mfma(qt, sb1, dk[db][1]);                                        \
  }
      FS_TR(0, 0); FS_TR(0, 1); FS_TR(1, 0); FS_TR(1, 1);
      asm volatile("s_waitcnt lgkmcnt(0)"
                   : "+v"(td[0][0]), "+v"(td[0][1]), "+v"(td[1][0]), "+v"(td[1][1]), "+v"(tq[0][0]), "+v"(tq[0][1]),
                     "+v"(tq[1][0]), "+v"(tq[1][1]));
      FS_TR(2, 0); FS_TR(2, 1); FS_TR(3, 0); FS_TR(3, 1);
      FS_MM(0) FS_MM(1)
      asm volatile("s_waitcnt lgkmcnt(0)"
                   : "+v"(td[2][0]), "+v"(td[2][1]), "+v"(td[3][0]), "+v"(td[3][1]), "+v"(tq[2][0]), "+v"(tq[2][1]),
                     "+v"(tq[3][0]), "+v"(tq[3][1]));
      FS_TR(4, 0); FS_TR(4, 1);
      FS_MM(2) FS_MM(3)
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(td[4][0]), "+v"(td[4][1]), "+v"(tq[4][0]), "+v"(tq[4][1]));
      FS_MM(4)
#undef FS_MM
#undef FS_TR
    };
#pragma unroll 1
    for (int qs = 0; qs < FS_N / FA_QS - 1; ++qs) step(qs, false);
    step(FS_N / FA_QS - 1, true);
    FS_WAIT_VM(0);  // the next unit's fragments and images (issued before this unit's compute)
#pragma unroll
    for (int kb2 = 0; kb2 < 2; ++kb2) {
      const int key = wave * 32 + kb2 * 16 + (lane & 15);
      bf16_t* dK = (bf16_t*)a.dk + b * a.k_bstride + h * a.k_hstride + (int64_t)key * a.ldk;
      bf16_t* dV = (bf16_t*)a.dv + b * a.v_bstride + h * a.v_hstride + (int64_t)key * a.ldv;
#pragma unroll
      for (int db = 0; db < 5; ++db) {
        const int d = db * 16 + 4 * g;
        if (d < 72) {
          *reinterpret_cast<u32x2*>(dK + d) = u32x2{pack2bf(dk[db][kb2][0] * a.scale, dk[db][kb2][1] * a.scale),
                                                    pack2bf(dk[db][kb2][2] * a.scale, dk[db][kb2][3] * a.scale)};
          *reinterpret_cast<u32x2*>(dV + d) =
              u32x2{pack2bf(dv[db][kb2][0], dv[db][kb2][1]), pack2bf(dv[db][kb2][2], dv[db][kb2][3])};
        }
      }
    }
    if (un < units && w0) tix.publish(tk, fa_smem + ((t + 1) & 1) * 2 * FS_IMG + FS_SLOT1);
    FS_BARRIER();
    u = un;
  }
}

// ---- joint forward with the softmax exported: LDS-DMA key / value ring (training default) -----------------------
// flash_fwd_probs_kernel's math and contract (P, tanh(cap), O) with the staging and the element-wise work rebuilt
// after its PMC (profiles/r05/pmc_attn_*.json: waves parked 45 % of their cycles, 11 vector instructions per
// MFMA, most of them the register staging's address arithmetic / LDS stores and per-score mask selects):
//   * the 5 K blocks then the 5 V blocks of 64 keys stream by LDS-DMA into a 4-slot ring of 32 KiB images,
//     three blocks ahead (stage s in slot s % 4; s + 3 issued once every wave has passed stage s's barrier);
//     512-B rows XOR-swizzled through the global source address: K chunk c of row r at c ^ (r & 15) (16-row
//     ds_read_b128 fragments conflict-free), V chunk c at c ^ 2 (r & 7) (4-row transposed reads conflict-free);
//   * key blocks wholly below the valid prefix (every key allowed for every row) in a wave without dead / past-
//     the-end rows skip the mask and the dead-row selects;
//   * Q fragments and the V^T fragments by inline-asm loads (hipcc would drain the in-flight DMA before the first
//     use of an ordinary global load or a transposed-read builtin).
// Keys past nk read the last key row (finite) and are masked; the schedule always runs 5 + 5 stages (nk <= 320).
constexpr int JD_SLOT = 64 * 512, JD_SMEM = 4 * JD_SLOT;

struct JdDma {  // this lane's part of the wave's 4 LDS-DMA instructions of a 64-key block image (recomputed per
               // issue: a few vector instructions instead of 8 live registers)
  int wave, lane;
  bool trs;
  __device__ __forceinline__ JdDma(int wave_, int lane_, bool trs_) : wave(wave_), lane(lane_), trs(trs_) {}
  __device__ __forceinline__ void issue(const bf16_t* X, int64_t ld, int kb, int nk, char* slot, int) const {
    int ln = lane;
    asm volatile("" : "+v"(ln));  // keeps hipcc from hoisting every stage's 64-bit addresses (80 live VGPRs)
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int r = 2 * (wave * 4 + s) + (ln >> 5), pch = ln & 31;
      const int coff = 8 * (pch ^ (trs ? 2 * (r & 7) : (r & 15)));
      int key = kb * 64 + r;
      key = key < nk ? key : nk - 1;
      fs_glds16(X + (int64_t)key * ld + coff, slot + (wave * 4 + s) * 1024);
    }
  }
};

// O^T += V^T P^T for head-dim blocks 4 DG .. 4 DG + 3 over the 32 keys of k-step K2: 8 transposed reads, one
// wait naming them, 4 MFMAs
template <int K2, int DG>
__device__ __forceinline__ void jd_pv_group(f32x4 (&o)[16], const unsigned (&vs)[8], const bf16x8& pk) {
  s16x4 tv[4][2];
#define JD_TR(u, hf) tv[u][hf] = fs_tr<(K2 * 32 + 16 * (hf)) * 512 + ((DG * 4 + (u)) & 8) * 32>(vs[(DG * 4 + (u)) & 7])
  JD_TR(0, 0); JD_TR(0, 1); JD_TR(1, 0); JD_TR(1, 1); JD_TR(2, 0); JD_TR(2, 1); JD_TR(3, 0); JD_TR(3, 1);
#undef JD_TR
  asm volatile("s_waitcnt lgkmcnt(0)"
               : "+v"(tv[0][0]), "+v"(tv[0][1]), "+v"(tv[1][0]), "+v"(tv[1][1]), "+v"(tv[2][0]), "+v"(tv[2][1]),
                 "+v"(tv[3][0]), "+v"(tv[3][1]));
#pragma unroll
  for (int u = 0; u < 4; ++u) o[DG * 4 + u] = mfma(fs_cat(tv[u][0], tv[u][1]), pk, o[DG * 4 + u]);
}

template <bool CAP>
__global__ void __launch_bounds__(JP_NW * 64, 1) flash_fwd_probs_dma_kernel(pz_flash_args a, bf16_t* P, bf16_t* TC,
                                                                         int64_t ldp) {
  extern __shared__ __attribute__((aligned(16))) char fa_smem[];
  constexpr int RPW = JP_NW * 16;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, l15 = lane & 15;
  int64_t zh;
  int qblk;
  fa_unit_block((int)((a.nq + RPW - 1) / RPW), (int)(a.Z * a.H), zh, qblk);
  const int64_t b = zh / a.H, h = zh % a.H;
  const int64_t r = (int64_t)qblk * RPW + wave * 16 + l15;  // this lane's query row
  const bool live = r < a.nq;
  const bf16_t* Q = (const bf16_t*)a.q + b * a.q_bstride + h * a.q_hstride;
  const bf16_t* K = (const bf16_t*)a.k + b * a.k_bstride + h * a.k_hstride;
  const bf16_t* V = (const bf16_t*)a.v + b * a.v_bstride + h * a.v_hstride;
  const FaMask mk(a, b);
  const FaFast ff(a);
  const int nk = (int)a.nk;
  const JdDma dmk(wave, lane, false), dmv(wave, lane, true);
  bf16x8 qf[8];
  {
    const bf16_t* qrow = Q + (live ? r : 0) * a.ldq + 8 * g;
#define JD_QLD(ks) asm volatile("global_load_dwordx4 %0, %1, off offset:%2" : "=v"(qf[ks]) : "v"(qrow), "i"((ks) * 64) : "memory")
    JD_QLD(0); JD_QLD(1); JD_QLD(2); JD_QLD(3); JD_QLD(4); JD_QLD(5); JD_QLD(6); JD_QLD(7);
#undef JD_QLD
  }
  auto issue = [&](int s) {  // stage s: K block s (s < 5) or V block s - 5, into slot s % 4
    char* slot = fa_smem + (s % 4) * JD_SLOT;
    if (s < 5) dmk.issue(K, a.ldk, s, nk, slot, wave);
    else dmv.issue(V, a.ldv, s - 5, nk, slot, wave);
  };
  issue(0);
  issue(1);
  issue(2);
  const int t = mk.token((int)r);
  const bool dead = mk.dead(t);
  const int rb = fa_row_bits(mk, t), full_keys = fa_full_keys(mk);
  const bool clean = __ballot(dead || !live) == 0ull;  // wave-uniform
  // pass 1: S^T[key][q] for every key of the row block (stage kb = K block kb); the element-wise logits of block
  // kb - 1 (soft-cap tanh, mask) are computed in stage kb beside its MFMAs (independent work the SIMD issues while
  // the MFMAs run), tanh(cap) kept packed in registers and exported after the pass
  f32x4 sc[JP_MAXKB][4];
  u32x2 tcv[JP_MAXKB][4];
  float mx = -INFINITY;
  auto logits_blk = [&](int kb) {
    // uniform per block: every key allowed and every row live (no mask, no dead-row selects)
    auto logits = [&](auto FAST) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float tv[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float sv = sc[kb][i][e];
          float th = 0.f, x2;
          if constexpr (CAP) {
            th = fmaf(-2.f, __builtin_amdgcn_rcpf(__builtin_amdgcn_exp2f(sv * ff.k2) + 1.f), 1.f);
            x2 = th * ff.crow_live;
          } else {
            x2 = sv * ff.crow_live;
          }
          if constexpr (!decltype(FAST)::value) {
            const int j = kb * FA_KB + i * 16 + 4 * g + e;
            const bool ok = j < nk && (j < full_keys || ((rb >> fa_key_class(mk, j)) & 1));
            x2 = ok ? x2 : -INFINITY;
            th = (dead || j >= nk) ? 0.f : th;
          }
          sc[kb][i][e] = x2;
          mx = fmaxf(mx, x2);
          tv[e] = th;
        }
        tcv[kb][i] = u32x2{pack2bf(tv[0], tv[1]), pack2bf(tv[2], tv[3])};
      }
    };
    if (clean && (kb + 1) * 64 <= full_keys) logits(std::true_type{});
    else logits(std::false_type{});
  };
#pragma unroll
  for (int kb = 0; kb < JP_MAXKB; ++kb) {
    FS_WAIT_VM(8);  // stage kb landed (stages kb + 1, kb + 2 in flight; the Q loads precede stage 0)
    FS_BARRIER();
    if (kb == 0)
      asm volatile("" : "+v"(qf[0]), "+v"(qf[1]), "+v"(qf[2]), "+v"(qf[3]), "+v"(qf[4]), "+v"(qf[5]), "+v"(qf[6]),
                   "+v"(qf[7]));
    issue(kb + 3);
    const char* slot = fa_smem + (kb % 4) * JD_SLOT + l15 * 512;
#pragma unroll
    for (int i = 0; i < 4; ++i) sc[kb][i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      const char* kp = slot + 16 * ((4 * ks + g) ^ l15);
#pragma unroll
      for (int i = 0; i < 4; ++i) sc[kb][i] = mfma(*reinterpret_cast<const bf16x8*>(kp + i * 8192), qf[ks], sc[kb][i]);
    }
    if (kb >= 1) logits_blk(kb - 1);
  }
  logits_blk(JP_MAXKB - 1);
  FS_WAIT_VM(4);  // V blocks 0, 1 (stages 5, 6) landed by this wave; stage 7 in flight
  bf16_t* prow = P + (b * a.nq + (live ? r : 0)) * ldp;
  if (TC) {  // uniform: the tanh(cap) export (zeros past nk and for dead rows)
    bf16_t* trow = TC + (b * a.nq + (live ? r : 0)) * ldp;
#pragma unroll
    for (int kb = 0; kb < JP_MAXKB; ++kb)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int j0 = kb * FA_KB + i * 16 + 4 * g;
        if (clean && (kb + 1) * 64 <= full_keys) *reinterpret_cast<u32x2*>(trow + j0) = tcv[kb][i];
        else if (live && j0 < ldp) *reinterpret_cast<u32x2*>(trow + j0) = tcv[kb][i];
      }
  }
  mx = fs_max4(mx);
  float sum = 0.f;
#pragma unroll
  for (int kb = 0; kb < JP_MAXKB; ++kb)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float pv = __builtin_amdgcn_exp2f(sc[kb][i][e] - mx);  // exp2(-inf) = 0
        sc[kb][i][e] = pv;
        sum += pv;
      }
  sum = fs_sum4(sum);
  // fully masked (dead) rows: uniform over the N keys (the finfo.min mask absorbs the logits)
  const float inv = 1.f / sum, uni = 1.f / (float)nk;
  bf16x8 pf[JP_MAXKB][2];
#pragma unroll
  for (int kb = 0; kb < JP_MAXKB; ++kb) {
    unsigned pk[4][2];
    auto probs = [&](auto FAST) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if constexpr (decltype(FAST)::value) {
          pk[i][0] = pack2bf(sc[kb][i][0] * inv, sc[kb][i][1] * inv);
          pk[i][1] = pack2bf(sc[kb][i][2] * inv, sc[kb][i][3] * inv);
        } else {
          float pv[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int j = kb * FA_KB + i * 16 + 4 * g + e;
            pv[e] = dead ? (j < nk ? uni : 0.f) : sc[kb][i][e] * inv;
          }
          pk[i][0] = pack2bf(pv[0], pv[1]);
          pk[i][1] = pack2bf(pv[2], pv[3]);
        }
        const int j0 = kb * FA_KB + i * 16 + 4 * g;
        if (decltype(FAST)::value || (live && j0 < ldp)) *reinterpret_cast<u32x2*>(prow + j0) = u32x2{pk[i][0], pk[i][1]};
      }
    };
    if (clean && (kb + 1) * 64 <= full_keys) probs(std::true_type{});
    else probs(std::false_type{});
    pf[kb][0] = __builtin_bit_cast(bf16x8, u32x4{pk[0][0], pk[0][1], pk[1][0], pk[1][1]});
    pf[kb][1] = __builtin_bit_cast(bf16x8, u32x4{pk[2][0], pk[2][1], pk[3][0], pk[3][1]});
  }
  // pass 2: O^T[d][q] = V^T[d][key] P^T[key][q] with the bf16 P (stage 5 + kb = V block kb)
  f32x4 o[16];
#pragma unroll
  for (int db = 0; db < 16; ++db) o[db] = f32x4{0.f, 0.f, 0.f, 0.f};
  // V^T fragment of (k2, db): rows k2*32 + 16 hf + 4g + q, 8-B piece p of head dims 16 db .. : swizzled chunk
  // (2 db + (p >> 1)) ^ 2 (r & 7) = 2 (db ^ w) + (p >> 1) with w = 4 (g & 1) + q
  const int q4 = l15 >> 2, p4 = lane & 3, w = 4 * (g & 1) + q4;
  unsigned va[8];
#pragma unroll
  for (int d7 = 0; d7 < 8; ++d7) va[d7] = fs_lds_addr(fa_smem + (4 * g + q4) * 512 + 32 * (d7 ^ w) + 8 * p4);
#pragma unroll
  for (int kb = 0; kb < JP_MAXKB; ++kb) {
    const int s = 5 + kb;
    if (s == 7) FS_WAIT_VM(8);  // (this wave's stages 5, 6 were waited before the softmax)
    if (s == 8) FS_WAIT_VM(4);
    if (s == 9) FS_WAIT_VM(0);
    FS_BARRIER();
    if (s + 3 <= 9) issue(s + 3);
    const unsigned sb = (unsigned)((s % 4) * JD_SLOT);
    unsigned vs[8];
#pragma unroll
    for (int d7 = 0; d7 < 8; ++d7) vs[d7] = va[d7] + sb;
    jd_pv_group<0, 0>(o, vs, pf[kb][0]);
    jd_pv_group<0, 1>(o, vs, pf[kb][0]);
    jd_pv_group<0, 2>(o, vs, pf[kb][0]);
    jd_pv_group<0, 3>(o, vs, pf[kb][0]);
    jd_pv_group<1, 0>(o, vs, pf[kb][1]);
    jd_pv_group<1, 1>(o, vs, pf[kb][1]);
    jd_pv_group<1, 2>(o, vs, pf[kb][1]);
    jd_pv_group<1, 3>(o, vs, pf[kb][1]);
  }
  if (!live) return;
  const FaRow fr{&a};
  const int gi = fr.grp(r);
  bf16_t* O = (bf16_t*)a.g_o[gi] + fr.off(b, h, r, gi);
#pragma unroll
  for (int db = 0; db < 16; ++db) {
    const int d = db * 16 + 4 * g;
    *reinterpret_cast<u32x2*>(O + d) = u32x2{pack2bf(o[db][0], o[db][1]), pack2bf(o[db][2], o[db][3])};
  }
}

// ---- joint backward dS (+ dQ) from the exported softmax: LDS-DMA value / key ring -----------------------------
// flash_bwd_ds_kernel's math and contract with flash_fwd_probs_dma_kernel's staging: stages 0..4 = V blocks
// (16-row fragments: K-style swizzle), 5..9 = K blocks (transposed fragments) in the 4-slot ring, three ahead;
// the P / tanh(cap) rows (inline-asm loads) are issued with the last V block so they land under its MFMAs.
// Without dQ the K stages still stream (from V: every wave's DMA count stays what the counted waits assume).
__global__ void __launch_bounds__(JP_NW * 64, 1) flash_bwd_ds_dma_kernel(pz_flash_args a, const bf16_t* P,
                                                                      const bf16_t* TC, bf16_t* dS, int64_t ldp) {
  extern __shared__ __attribute__((aligned(16))) char fa_smem[];
  constexpr int RPW = JP_NW * 16;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, l15 = lane & 15;
  int64_t zh;
  int qblk;
  fa_unit_block((int)((a.nq + RPW - 1) / RPW), (int)(a.Z * a.H), zh, qblk);
  const int64_t b = zh / a.H, h = zh % a.H;
  const int64_t r = (int64_t)qblk * RPW + wave * 16 + l15;
  const bool live = r < a.nq;
  const bool want_dq = a.dq != nullptr;
  const bf16_t* V = (const bf16_t*)a.v + b * a.v_bstride + h * a.v_hstride;
  const bf16_t* K = want_dq ? (const bf16_t*)a.k + b * a.k_bstride + h * a.k_hstride : V;
  const int64_t ldk = want_dq ? a.ldk : a.ldv;
  const int nk = (int)a.nk;
  const JdDma dmv(wave, lane, false), dmk(wave, lane, true);
  auto issue = [&](int s) {  // stage s: V block s (s < 5) or K block s - 5, into slot s % 4
    char* slot = fa_smem + (s % 4) * JD_SLOT;
    if (s < 5) dmv.issue(V, a.ldv, s, nk, slot, wave);
    else dmk.issue(K, ldk, s - 5, nk, slot, wave);
  };
  // dO fragments (a mixture without dO contributes dP = 0)
  bf16x8 df[8];
  bool has_do;
  {
    const FaRow fr{&a};
    const int gi = live ? fr.grp(r) : 0;
    has_do = live && a.g_do[gi];
    const bf16_t* dOr = has_do ? (const bf16_t*)a.g_do[gi] + fr.off(b, h, r, gi) + 8 * g : V;
#define JD_DLD(ks) asm volatile("global_load_dwordx4 %0, %1, off offset:%2" : "=v"(df[ks]) : "v"(dOr), "i"((ks) * 64) : "memory")
    JD_DLD(0); JD_DLD(1); JD_DLD(2); JD_DLD(3); JD_DLD(4); JD_DLD(5); JD_DLD(6); JD_DLD(7);
#undef JD_DLD
  }
  issue(0);
  issue(1);
  issue(2);
  const bf16_t* prow = P + (b * a.nq + (live ? r : 0)) * ldp;
  const bf16_t* trow = TC ? TC + (b * a.nq + (live ? r : 0)) * ldp : prow;
  const bool clean = __ballot(!live) == 0ull;
  // pass 1 (stage kb = V block kb): dP^T[key][q] = V dO^T
  f32x4 dp[JP_MAXKB][4];
  u32x2 pw[JP_MAXKB][4], tw[JP_MAXKB][4];
#pragma unroll
  for (int kb = 0; kb < JP_MAXKB; ++kb) {
    FS_WAIT_VM(8);
    FS_BARRIER();
    if (kb == 0) {
      asm volatile("" : "+v"(df[0]), "+v"(df[1]), "+v"(df[2]), "+v"(df[3]), "+v"(df[4]), "+v"(df[5]), "+v"(df[6]),
                   "+v"(df[7]));
      if (!has_do) {
#pragma unroll
        for (int ks = 0; ks < 8; ++ks) df[ks] = bf16x8{};
      }
    }
    issue(kb + 3);
    const char* slot = fa_smem + (kb % 4) * JD_SLOT + l15 * 512;
#pragma unroll
    for (int i = 0; i < 4; ++i) dp[kb][i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      const char* vp = slot + 16 * ((4 * ks + g) ^ l15);
#pragma unroll
      for (int i = 0; i < 4; ++i) dp[kb][i] = mfma(*reinterpret_cast<const bf16x8*>(vp + i * 8192), df[ks], dp[kb][i]);
    }
  }
  // this row's P and tanh(cap) (issued once dO's fragments are dead; the tanh(cap) latency runs under the P . dP
  // row sum; columns past ldp are never read).  The opaque lane index keeps hipcc from computing the 40 addresses
  // up front.
  int gl = g;
  asm volatile("" : "+v"(gl));
#pragma unroll
  for (int k2 = 0; k2 < JP_MAXKB; ++k2)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int j0 = k2 * FA_KB + i * 16 + 4 * gl;
      const int jc = j0 < ldp ? j0 : 0;
      asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(pw[k2][i]) : "v"(prow + jc) : "memory");
    }
#pragma unroll
  for (int k2 = 0; k2 < JP_MAXKB; ++k2)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int j0 = k2 * FA_KB + i * 16 + 4 * gl;
      const int jc = j0 < ldp ? j0 : 0;
      asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(tw[k2][i]) : "v"(trow + jc) : "memory");
    }
  FS_WAIT_VM(20);  // P rows and K blocks 0..2 (stages 5..7) landed; the 20 tanh(cap) loads in flight
  // dS = P (dP - delta) scale (1 - tc^2) for the row (kept in dp as fp32; stored in bf16)
  bf16_t* orow = dS + (b * a.nq + (live ? r : 0)) * ldp;
  const bool cap = a.cap > 0.f;
  float dot = 0.f;
#pragma unroll
  for (int kb = 0; kb < JP_MAXKB; ++kb)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      asm volatile("" : "+v"(pw[kb][i]));
      const int j0 = kb * FA_KB + i * 16 + 4 * g;
      if (!(live && j0 < nk)) pw[kb][i] = u32x2{0u, 0u};  // P = 0 past N (and for rows past nq)
      const float p0 = __uint_as_float(pw[kb][i][0] << 16), p1 = __uint_as_float(pw[kb][i][0] & 0xffff0000u);
      const float p2 = __uint_as_float(pw[kb][i][1] << 16), p3 = __uint_as_float(pw[kb][i][1] & 0xffff0000u);
      dot += p0 * dp[kb][i][0] + p1 * dp[kb][i][1] + p2 * dp[kb][i][2] + p3 * dp[kb][i][3];
    }
  dot += __shfl_xor(dot, 16, 64);  // (fs_sum4's two extra registers make this kernel spill)
  dot += __shfl_xor(dot, 32, 64);
  FS_WAIT_VM(0);
#pragma unroll
  for (int kb = 0; kb < JP_MAXKB; ++kb)
#pragma unroll
    for (int i = 0; i < 4; ++i) asm volatile("" : "+v"(tw[kb][i]));
  bf16x8 dsf[JP_MAXKB][2];
#pragma unroll
  for (int kb = 0; kb < JP_MAXKB; ++kb) {
    unsigned pk[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int j0 = kb * FA_KB + i * 16 + 4 * g;
      const u32x2 tv2 = (cap && live && j0 < nk) ? tw[kb][i] : u32x2{0u, 0u};
      const float pv[4] = {__uint_as_float(pw[kb][i][0] << 16), __uint_as_float(pw[kb][i][0] & 0xffff0000u),
                           __uint_as_float(pw[kb][i][1] << 16), __uint_as_float(pw[kb][i][1] & 0xffff0000u)};
      const float tv[4] = {__uint_as_float(tv2[0] << 16), __uint_as_float(tv2[0] & 0xffff0000u),
                           __uint_as_float(tv2[1] << 16), __uint_as_float(tv2[1] & 0xffff0000u)};
      float x[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {  // pv = 0 past N: x = 0 there
        x[e] = pv[e] * (dp[kb][i][e] - dot) * a.scale;
        if (cap) x[e] *= fmaf(-tv[e], tv[e], 1.f);
      }
      pk[i][0] = pack2bf(x[0], x[1]);
      pk[i][1] = pack2bf(x[2], x[3]);
      if (clean ? j0 < ldp : (live && j0 < ldp)) *reinterpret_cast<u32x2*>(orow + j0) = u32x2{pk[i][0], pk[i][1]};
    }
    dsf[kb][0] = __builtin_bit_cast(bf16x8, u32x4{pk[0][0], pk[0][1], pk[1][0], pk[1][1]});
    dsf[kb][1] = __builtin_bit_cast(bf16x8, u32x4{pk[2][0], pk[2][1], pk[3][0], pk[3][1]});
  }
  // pass 2 (stage 5 + kb = K block kb): dQ^T[d][q] = K^T[d][key] dS^T[key][q] with the bf16 dS
  f32x4 dq[16];
#pragma unroll
  for (int db = 0; db < 16; ++db) dq[db] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int q4 = l15 >> 2, p4 = lane & 3, w = 4 * (g & 1) + q4;
  unsigned ka[8];
#pragma unroll
  for (int d7 = 0; d7 < 8; ++d7) ka[d7] = fs_lds_addr(fa_smem + (4 * g + q4) * 512 + 32 * (d7 ^ w) + 8 * p4);
#pragma unroll
  for (int kb = 0; kb < JP_MAXKB; ++kb) {
    const int s = 5 + kb;
    if (s == 8) FS_WAIT_VM(4);  // (stages 5..7 were waited before the dS phase; its stores precede stage 8)
    if (s == 9) FS_WAIT_VM(0);
    FS_BARRIER();
    if (s + 3 <= 9) issue(s + 3);
    if (want_dq) {  // uniform
      const unsigned sb = (unsigned)((s % 4) * JD_SLOT);
      unsigned ks_[8];
#pragma unroll
      for (int d7 = 0; d7 < 8; ++d7) ks_[d7] = ka[d7] + sb;
      jd_pv_group<0, 0>(dq, ks_, dsf[kb][0]);
      jd_pv_group<0, 1>(dq, ks_, dsf[kb][0]);
      jd_pv_group<0, 2>(dq, ks_, dsf[kb][0]);
      jd_pv_group<0, 3>(dq, ks_, dsf[kb][0]);
      jd_pv_group<1, 0>(dq, ks_, dsf[kb][1]);
      jd_pv_group<1, 1>(dq, ks_, dsf[kb][1]);
      jd_pv_group<1, 2>(dq, ks_, dsf[kb][1]);
      jd_pv_group<1, 3>(dq, ks_, dsf[kb][1]);
    }
  }
  if (!live || !want_dq) return;
  bf16_t* dQ = (bf16_t*)a.dq + b * a.q_bstride + h * a.q_hstride + r * a.ldq;
#pragma unroll
  for (int db = 0; db < 16; ++db) {
    const int d = db * 16 + 4 * g;
    *reinterpret_cast<u32x2*>(dQ + d) = u32x2{pack2bf(dq[db][0], dq[db][1]), pack2bf(dq[db][2], dq[db][3])};
  }
}

// ---- fp8 attention forward (C5 prefill, BASELINE.json configs[4] "fp8 MFMA attention") ---------------------------
// S = Q K^T and O = P V on v_mfma_f32_16x16x128_f8f6f4 (OCP e4m3 codes, head_dim 256): per-row scales for Q (sq) and
// the keys (sk), per-head-dim scales for V (sv: O[q][d] = sv_d sum_k P v_kd, exact factorisation), P quantised as
// e4m3(256 p) with p <= 1 from the online softmax, so O = sv_d / 256 sum_k e4m3(256 p_qk) v_kd / l.  Soft-cap, block
// mask and the online softmax are the bf16 kernel's (fa_logit on the dequantised score).  8 waves x 16 query rows per
// workgroup, 128-key blocks double-buffered through LDS (register-staged):
//   * K block [128 keys][256 codes]; MFMA row m of 16-key group i is key 32 (m >> 2) + 4 i + (m & 3), so lane group g
//     of the S^T result holds keys 32 g .. 32 g + 31 of the block -- exactly the 32-code k set lane group g of P^T
//     needs for ONE P V MFMA over the 128 keys; 16-B chunk c of key row r stored at c ^ ((r & 3) | (r >> 5) << 2):
//     every ds_read_b128 of a fragment conflict-free;
//   * V^T block [256 d][128 keys] (pz_fp8_quant_vt writes V^T codes), chunk c of row d at c ^ ((d & 6) | (d >> 3 & 1)):
//     conflict-free;
//   * key split over blockIdx.z with unnormalised fp32 partials (O sv / 256, m, l) merged by flash_fwd_combine_kernel.
constexpr int F8_KB = 128, F8_KT = F8_KB * 256, F8_VT = 256 * F8_KB;
constexpr int F8_SMEM = 2 * (F8_KT + F8_VT) + 2 * F8_KB * 4;

__device__ __forceinline__ int f8_kswz(int r) { return (r & 3) | ((r >> 5) << 2); }
__device__ __forceinline__ int f8_vswz(int d) { return (d & 6) | ((d >> 3) & 1); }
__device__ __forceinline__ i32x8 f8_cat(const u32x4& lo, const u32x4& hi) {
  return i32x8{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
}
__device__ __forceinline__ unsigned f8_enc4(float a, float b, float c, float d) {
  int v = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  v = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, v, true);
  return (unsigned)v;
}

__global__ void __launch_bounds__(512) flash_fwd_f8_kernel(pz_flash_args a, const uint8_t* __restrict__ qc,
                                                          const float* __restrict__ qs, const uint8_t* __restrict__ kc,
                                                          const float* __restrict__ ks, int64_t krows,
                                                          const uint8_t* __restrict__ vtc,
                                                          const float* __restrict__ vs, int64_t ldvt) {
  extern __shared__ __attribute__((aligned(16))) char fa_smem[];
  auto Kt = [&](int bi) { return fa_smem + bi * F8_KT; };
  auto Vt = [&](int bi) { return fa_smem + 2 * F8_KT + bi * F8_VT; };
  auto Sk = [&](int bi) { return reinterpret_cast<float*>(fa_smem + 2 * (F8_KT + F8_VT)) + bi * F8_KB; };
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, g = lane >> 4, l15 = lane & 15;
  const int64_t b = blockIdx.y;
  const int64_t q0 = (int64_t)blockIdx.x * 128 + wave * 16;
  const int64_t r = q0 + l15;  // this lane's query row
  const FaMask mk(a, b);
  const int nkb = (int)((a.nk + F8_KB - 1) / F8_KB);
  const int per = (nkb + (int)gridDim.z - 1) / (int)gridDim.z;
  const int kb_begin = (int)blockIdx.z * per, kb_end = min(nkb, kb_begin + per);
  // register-staged block loads: 4 K chunks, 4 V^T chunks, (threads < 128) one key scale
  u32x4 sk_[4], sv_[4];
  float sks = 0.f;
  auto load = [&](int kb) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = t + 512 * j;
      const int64_t kr = min((int64_t)kb * F8_KB + (c >> 4), krows - 1);
      sk_[j] = *reinterpret_cast<const u32x4*>(kc + (b * krows + kr) * 256 + (c & 15) * 16);
      sv_[j] = *reinterpret_cast<const u32x4*>(vtc + (b * 256 + (c >> 3)) * ldvt + (int64_t)kb * F8_KB + (c & 7) * 16);
    }
    if (t < F8_KB) sks = ks[b * krows + min((int64_t)kb * F8_KB + t, krows - 1)];
  };
  auto store = [&](int bi) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = t + 512 * j;
      const int kr = c >> 4, d = c >> 3;
      *reinterpret_cast<u32x4*>(Kt(bi) + kr * 256 + (((c & 15) ^ f8_kswz(kr)) << 4)) = sk_[j];
      *reinterpret_cast<u32x4*>(Vt(bi) + d * 128 + (((c & 7) ^ f8_vswz(d)) << 4)) = sv_[j];
    }
    if (t < F8_KB) Sk(bi)[t] = sks;
  };
  // Q^T fragments (B operand: codes 128 ks + 32 g .. + 31 of this lane's row) and the row scale
  i32x8 qf[2];
  float sq = 0.f;
  {
    const bool ok = r < a.nq;
    const uint8_t* qr = qc + (b * a.nq + (ok ? r : 0)) * 256 + 32 * g;
#pragma unroll
    for (int k2 = 0; k2 < 2; ++k2) {
      const u32x4 lo = ok ? *reinterpret_cast<const u32x4*>(qr + 128 * k2) : u32x4{0u, 0u, 0u, 0u};
      const u32x4 hi = ok ? *reinterpret_cast<const u32x4*>(qr + 128 * k2 + 16) : u32x4{0u, 0u, 0u, 0u};
      qf[k2] = f8_cat(lo, hi);
    }
    if (ok) sq = qs[b * a.nq + r];
  }
  const int tq = mk.token((int)r);
  f32x4 o[16];
#pragma unroll
  for (int db = 0; db < 16; ++db) o[db] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY, l = 0.f;
  if (kb_begin < kb_end) {
    load(kb_begin);
    store(0);
  }
  __syncthreads();
  // this lane's K fragment rows (key within the block) per 16-key group: 32 (l15 >> 2) + 4 i + (l15 & 3)
  const int krow0 = 32 * (l15 >> 2) + (l15 & 3);
  for (int kb = kb_begin; kb < kb_end; ++kb) {
    const int bi = (kb - kb_begin) & 1;
    const bool more = kb + 1 < kb_end;
    if (more) load(kb + 1);
    const char* K = Kt(bi);
    f32x4 sc[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      sc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
      const int kr = krow0 + 4 * i, sw = f8_kswz(kr);
#pragma unroll
      for (int k2 = 0; k2 < 2; ++k2) {
        const int c0 = 8 * k2 + 2 * g;
        const u32x4 lo = *reinterpret_cast<const u32x4*>(K + kr * 256 + ((c0 ^ sw) << 4));
        const u32x4 hi = *reinterpret_cast<const u32x4*>(K + kr * 256 + (((c0 + 1) ^ sw) << 4));
        sc[i] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(f8_cat(lo, hi), qf[k2], sc[i], 0, 0, 0, 0, 0, 0);
      }
    }
    // dequantised logits of keys 32 g + 4 i + e, online softmax over the block
    float mx = -INFINITY;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const f32x4 skv = *reinterpret_cast<const f32x4*>(Sk(bi) + 32 * g + 4 * i);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int j = kb * F8_KB + 32 * g + 4 * i + e;
        const float x = fa_logit(mk, sc[i][e] * sq * skv[e], tq, j);
        sc[i][e] = x;
        mx = fmaxf(mx, x);
      }
    }
    mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float mn = fmaxf(m, mx);
    const float alpha = mn == -INFINITY ? 1.f : __expf(m - mn);
    float sum = 0.f;
    unsigned pw[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float pv[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        pv[e] = mn == -INFINITY ? 0.f : __expf(sc[i][e] - mn);
        sum += pv[e];
      }
      pw[i] = f8_enc4(pv[0] * 256.f, pv[1] * 256.f, pv[2] * 256.f, pv[3] * 256.f);
    }
    sum += __shfl_xor(sum, 16, 64);
    sum += __shfl_xor(sum, 32, 64);
    l = l * alpha + sum;
    m = mn;
#pragma unroll
    for (int db = 0; db < 16; ++db) o[db] *= alpha;
    const i32x8 pf = i32x8{(int)pw[0], (int)pw[1], (int)pw[2], (int)pw[3], (int)pw[4], (int)pw[5], (int)pw[6], (int)pw[7]};
    // O^T[d][q] += V^T[d][keys 32 g ..] P^T[..][q]
    const char* V = Vt(bi);
#pragma unroll
    for (int db = 0; db < 16; ++db) {
      const int d = 16 * db + l15, sw = f8_vswz(d);
      const u32x4 lo = *reinterpret_cast<const u32x4*>(V + d * 128 + (((2 * g) ^ sw) << 4));
      const u32x4 hi = *reinterpret_cast<const u32x4*>(V + d * 128 + (((2 * g + 1) ^ sw) << 4));
      o[db] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(f8_cat(lo, hi), pf, o[db], 0, 0, 0, 0, 0, 0);
    }
    __syncthreads();  // every wave done with this block's buffers
    if (more) store(bi ^ 1);
    __syncthreads();
  }
  if (r >= a.nq) return;
  // O^T rows d = 16 db + 4 g + e: the V column scales and the 1/256 of the P codes
  const float* svb = vs + b * 256;
  if (gridDim.z > 1) {
    float* pO = (float*)a.ws;
    float* pml = pO + (int64_t)gridDim.z * gridDim.y * a.nq * 256;
    const int64_t row = ((int64_t)blockIdx.z * gridDim.y + b) * a.nq + r;
#pragma unroll
    for (int db = 0; db < 16; ++db) {
      const int d = 16 * db + 4 * g;
      const f32x4 sv4 = *reinterpret_cast<const f32x4*>(svb + d);
      *reinterpret_cast<f32x4*>(pO + row * 256 + d) = o[db] * sv4 * (1.f / 256.f);
    }
    if (g == 0) {
      pml[2 * row] = m;
      pml[2 * row + 1] = l;
    }
    return;
  }
  const float inv = l > 0.f ? 1.f / (256.f * l) : 0.f;
  const FaRow fr{&a};
  const int gi = fr.grp(r);
  bf16_t* O = (bf16_t*)a.g_o[gi] + fr.off(b, 0, r, gi);
#pragma unroll
  for (int db = 0; db < 16; ++db) {
    const int d = 16 * db + 4 * g;
    const f32x4 sv4 = *reinterpret_cast<const f32x4*>(svb + d);
    const f32x4 v = o[db] * sv4 * inv;
    *reinterpret_cast<u32x2*>(O + d) = u32x2{pack2bf(v[0], v[1]), pack2bf(v[2], v[3])};
  }
  if (g == 0 && a.lse) a.lse[b * a.nq + r] = m + __logf(l);
}

}  // namespace

// head dims with instantiated kernels: the Pi0 shapes (SigLIP 72, Gemma 256) and the tiny test config (16, 32)
#define FA_DISPATCH(HDV_, KERNEL, GRID, ...)                                                        \
  switch (HDV_) {                                                                                   \
    case 256: hipLaunchKernelGGL(KERNEL<256>, GRID, __VA_ARGS__); break;                            \
    case 72: hipLaunchKernelGGL(KERNEL<72>, GRID, __VA_ARGS__); break;                              \
    case 32: hipLaunchKernelGGL(KERNEL<32>, GRID, __VA_ARGS__); break;                              \
    default: hipLaunchKernelGGL(KERNEL<16>, GRID, __VA_ARGS__); break;                              \
  }
// FA_DISPATCH over a kernel with a second template argument: FA_T2(k, X)<HD> = k<HD, X>
#define FA_T2(K, X) FaT2<X>::template K##_t
template <auto X>
struct FaT2 {
  template <int HD> static constexpr auto flash_bwd_q2_kernel_t = flash_bwd_q2_kernel<HD, (bool)X>;
  template <int HD> static constexpr auto flash_bwd_kv_kernel_t = flash_bwd_kv_kernel<HD, (int)X>;
};
// joint backward element-wise path: 1 fast, 2 fast + soft-cap
static int fa_fast_bwd(const pz_flash_args* a) { return a->cap > 0.f ? 2 : 1; }
static bool fa_hd_ok(int64_t hd) { return hd == 256 || hd == 72 || hd == 32 || hd == 16; }

// SigLIP shape: the whole key / query side of a unit fits the resident kernels' LDS images
static bool fa_resident(const pz_flash_args* a) {
  const char* e = getenv("PZ_FLASH_RESIDENT");  // "0": step-staged kernels (A/B runs; read per call)
  if (e && e[0] == '0') return false;
  return a->head_dim == 72 && a->nq <= FR_MAX && a->nk <= FR_MAX;
}

// one workgroup per unit for the resident shape when there are enough units to fill the chip (the
// training micro-batch: 1024); few units (B = 1 inference: 16) keep the 2- / 4-workgroup resident
// kernels' parallelism.  PZ_FLASH_UNIT "0" / "1" forces either (tests, A/B runs)
static bool fa_unit(const pz_flash_args* a) {
  const char* e = getenv("PZ_FLASH_UNIT");
  if (e && e[0] == '0') return false;
  if (e && e[0] == '1') return true;
  return a->Z * a->H >= 128;
}

// no mask, no soft-cap (SigLIP): the unit kernels' log2-domain element-wise fast path
static bool fa_plain(const pz_flash_args* a) { return a->mask_mode == 0 && a->cap == 0.f; }

// compute units of the current device (the persistent SigLIP grid: one workgroup per CU)
static int fa_device_cus() {
  static int cache[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (!cache[dev]) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cache[dev] = n;
  }
  return cache[dev];
}

// workgroups of the persistent SigLIP kernels: one per CU (units are taken from per-XCD ticket counters, FsTickets)
static int fa_sig_grid(const pz_flash_args* a) { return (int)std::min<int64_t>(a->Z * a->H, fa_device_cus()); }

// the SigLIP training shape (256 x 256 keys, head 72, plain, one output group): the persistent pipelined
// kernels; PZ_FLASH_SIG "0" keeps the one-workgroup-per-unit kernels (tests, A/B runs)
static bool fa_sig(const pz_flash_args* a) {
  const char* e = getenv("PZ_FLASH_SIG");
  if (e && e[0] == '0') return false;
  return fa_plain(a) && a->head_dim == 72 && a->nq == FS_N && a->nk == FS_N && a->n_groups == 1 &&
         a->o_hstride % 8 == 0 && a->g_ld[0] % 8 == 0 && a->g_bstride[0] % 8 == 0 &&
         a->ldq * FS_N < (1 << 30) && a->ldk * FS_N < (1 << 30) && a->ldv * FS_N < (1 << 30) &&
         a->g_ld[0] * FS_N < (1 << 30);
}

// Raise the kernel's dynamic-LDS limit once; a refusal is cleared here (the launch is checked on
// its own) so it cannot surface as a later launch's error
template <class Kern>
static void fa_smem_attr(Kern k, int bytes, bool& done) {
  if (!done) {
    if (hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, bytes) != hipSuccess)
      (void)hipGetLastError();
    done = true;
  }
}

extern "C" int pz_flash_fwd(const pz_flash_args* a, void* stream) {
  PZ_CHECK_ARG(a && a->q && a->k && a->v && a->Z > 0 && a->H > 0 && a->nq > 0 && a->nk > 0,
               "flash_fwd: bad args");
  PZ_CHECK_ARG(fa_hd_ok(a->head_dim), "flash_fwd: head_dim %lld unsupported (16, 32, 72, 256)",
               (long long)a->head_dim);
  PZ_CHECK_ARG(a->n_groups >= 1 && a->n_groups <= 3 && a->g_row0[0] == 0, "flash_fwd: output groups");
  for (int i = 0; i < a->n_groups; ++i) PZ_CHECK_ARG(a->g_o[i] && a->g_ld[i] % 4 == 0, "flash_fwd: group %d", i);
  PZ_CHECK_ARG(PZ_ALIGNED(a->q, 16) && PZ_ALIGNED(a->k, 16) && PZ_ALIGNED(a->v, 16) && a->ldq % 8 == 0 &&
                   a->ldk % 8 == 0 && a->ldv % 8 == 0 && a->q_hstride % 8 == 0 && a->k_hstride % 8 == 0 &&
                   a->v_hstride % 8 == 0 && a->q_bstride % 8 == 0 && a->k_bstride % 8 == 0 &&
                   a->v_bstride % 8 == 0 && a->o_hstride % 4 == 0,
               "flash_fwd: operands need 16-byte aligned rows");
  if (a->mask_mode == 1) PZ_CHECK_ARG(a->cnt && a->rows_per_token > 0, "flash_fwd: block mask needs cnt");
  PZ_CHECK_ARG(a->nq + a->mask_row0 < (1 << 22) && a->nk < (1 << 22) && a->mask_row0 >= 0, "flash_fwd: nq/nk too large");
  PZ_CHECK_ARG(a->Z * a->H < 65536, "flash_fwd: too many units");
  const int64_t qblk = (a->nq + 127) / 128, units = qblk * a->Z * a->H;  // 128 query rows per workgroup
  // few workgroups (inference: one action chunk, one prefix): split the keys over up to 16
  // workgroups per unit when the caller gave a workspace for the partials
  const int64_t nkb = (a->nk + FA_KB - 1) / FA_KB;
  int64_t sp = 1;
  if (a->ws && units < 128 && nkb > 1 && a->head_dim % 4 == 0) {
    sp = (256 + units - 1) / units;
    sp = sp < nkb ? sp : nkb;
    sp = sp < 16 ? sp : 16;
    while (sp > 1 && sp * a->Z * a->H * a->nq * (a->head_dim + 2) * 4 > a->ws_bytes) --sp;
    const int64_t per = (nkb + sp - 1) / sp;
    sp = (nkb + per - 1) / per;  // no empty split
  }
  dim3 grid((unsigned)qblk, (unsigned)(a->Z * a->H), (unsigned)sp);
  hipStream_t st = (hipStream_t)stream;
  if (sp == 1 && fa_resident(a) && fa_unit(a)) {
    static bool attr = false;
    static bool attr2 = false;
    static bool attr3 = false;
    const dim3 gu((unsigned)(a->Z * a->H));
    if (fa_sig(a)) {
      const int G = fa_sig_grid(a);
      (void)attr3;
      {
        static bool attr4 = false;
        fa_smem_attr(flash_fwd_sig_kernel<1>, FS_SMEM, attr4);
        hipLaunchKernelGGL(flash_fwd_sig_kernel<1>, dim3((unsigned)G), dim3(16 * 64), FS_SMEM, st, *a, G);
      }
    } else if (fa_plain(a)) {
      fa_smem_attr(flash_fwd_unit_kernel<72, true>, FR_SMEM_KQ, attr);
      hipLaunchKernelGGL((flash_fwd_unit_kernel<72, true>), gu, dim3(FU_NW * 64), FR_SMEM_KQ, st, *a);
    } else {
      fa_smem_attr(flash_fwd_unit_kernel<72, false>, FR_SMEM_KQ, attr2);
      hipLaunchKernelGGL((flash_fwd_unit_kernel<72, false>), gu, dim3(FU_NW * 64), FR_SMEM_KQ, st, *a);
    }
    PZ_CHECK_LAUNCH();
    return PZ_OK;
  }
  if (sp == 1 && fa_resident(a)) {
    static bool attr = false;
    fa_smem_attr(flash_fwd_res_kernel<72>, FR_SMEM_KQ, attr);
    hipLaunchKernelGGL(flash_fwd_res_kernel<72>, dim3((unsigned)((a->nq + FR_NW * 16 - 1) / (FR_NW * 16) * a->Z * a->H)),
                       dim3(FR_NW * 64), FR_SMEM_KQ, st, *a);
    PZ_CHECK_LAUNCH();
    return PZ_OK;
  }
  FA_DISPATCH(a->head_dim, flash_fwd_kernel, grid, dim3((a->head_dim == 256 ? 8 : 4) * 64), 0, st, *a);
  PZ_CHECK_LAUNCH();
  if (sp > 1) {
    const int64_t n = a->Z * a->H * a->nq * (a->head_dim / 4);
    FA_DISPATCH(a->head_dim, flash_fwd_combine_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, *a,
                (int)sp);
    PZ_CHECK_LAUNCH();
  }
  return PZ_OK;
}


extern "C" int pz_flash_fwd_probs(const pz_flash_args* a, void* P, void* tcap, int64_t ldp, void* stream) {
  PZ_CHECK_ARG(a && a->q && a->k && a->v && P && a->Z > 0 && a->H > 0 && a->nq > 0 && a->nk > 0,
               "flash_fwd_probs: bad args");
  PZ_CHECK_ARG(a->head_dim == 256, "flash_fwd_probs: head_dim %lld (256 only)", (long long)a->head_dim);
  PZ_CHECK_ARG(a->nk <= JP_MAXKB * FA_KB && ldp >= a->nk && ldp % 4 == 0, "flash_fwd_probs: nk %lld / ldp %lld",
               (long long)a->nk, (long long)ldp);
  PZ_CHECK_ARG(a->mask_mode == 0 || (a->mask_mode == 1 && a->cnt && a->rows_per_token > 0),
               "flash_fwd_probs: mask mode %d", a->mask_mode);
  PZ_CHECK_ARG(a->n_groups >= 1 && a->n_groups <= 3 && a->g_row0[0] == 0, "flash_fwd_probs: output groups");
  for (int i = 0; i < a->n_groups; ++i) PZ_CHECK_ARG(a->g_o[i] && a->g_ld[i] % 4 == 0, "flash_fwd_probs: group %d", i);
  PZ_CHECK_ARG(PZ_ALIGNED(a->q, 16) && PZ_ALIGNED(a->k, 16) && PZ_ALIGNED(a->v, 16) && PZ_ALIGNED(P, 8) &&
                   (!tcap || PZ_ALIGNED(tcap, 8)) && a->ldq % 8 == 0 && a->ldk % 8 == 0 && a->ldv % 8 == 0 &&
                   a->q_bstride % 8 == 0 && a->k_bstride % 8 == 0 && a->v_bstride % 8 == 0,
               "flash_fwd_probs: operands need 16-byte aligned rows");
  PZ_CHECK_ARG(a->nq + a->mask_row0 < (1 << 22) && a->Z * a->H < 65536, "flash_fwd_probs: nq / units too large");
  const int64_t units = a->Z * a->H, nqb = (a->nq + JP_NW * 16 - 1) / (JP_NW * 16);
  {
    static bool attr0 = false, attr1 = false;
    if (a->cap > 0.f) {
      fa_smem_attr(flash_fwd_probs_dma_kernel<true>, JD_SMEM, attr1);
      hipLaunchKernelGGL(flash_fwd_probs_dma_kernel<true>, dim3((unsigned)(nqb * units)), dim3(JP_NW * 64), JD_SMEM,
                         (hipStream_t)stream, *a, (bf16_t*)P, (bf16_t*)tcap, ldp);
    } else {
      fa_smem_attr(flash_fwd_probs_dma_kernel<false>, JD_SMEM, attr0);
      hipLaunchKernelGGL(flash_fwd_probs_dma_kernel<false>, dim3((unsigned)(nqb * units)), dim3(JP_NW * 64), JD_SMEM,
                         (hipStream_t)stream, *a, (bf16_t*)P, (bf16_t*)tcap, ldp);
    }
    PZ_CHECK_LAUNCH();
    return PZ_OK;
  }
}

extern "C" int pz_flash_bwd_ds(const pz_flash_args* a, const void* P, const void* tcap, void* dS, int64_t ldp,
                               void* stream) {
  PZ_CHECK_ARG(a && a->v && P && dS && a->Z > 0 && a->H > 0 && a->nq > 0 && a->nk > 0, "flash_bwd_ds: bad args");
  PZ_CHECK_ARG(a->head_dim == 256, "flash_bwd_ds: head_dim %lld (256 only)", (long long)a->head_dim);
  PZ_CHECK_ARG(a->nk <= JP_MAXKB * FA_KB && ldp >= a->nk && ldp % 4 == 0, "flash_bwd_ds: nk %lld / ldp %lld",
               (long long)a->nk, (long long)ldp);
  PZ_CHECK_ARG(a->cap <= 0.f || tcap, "flash_bwd_ds: soft-cap needs tcap");
  PZ_CHECK_ARG(a->n_groups >= 1 && a->n_groups <= 3 && a->g_row0[0] == 0, "flash_bwd_ds: output groups");
  for (int i = 0; i < a->n_groups; ++i) PZ_CHECK_ARG(!a->g_do[i] || a->g_ld[i] % 8 == 0, "flash_bwd_ds: dO group %d", i);
  PZ_CHECK_ARG(PZ_ALIGNED(a->v, 16) && a->ldv % 8 == 0 && a->v_bstride % 8 == 0 && PZ_ALIGNED(P, 8) &&
                   PZ_ALIGNED(dS, 8) && (!tcap || PZ_ALIGNED(tcap, 8)),
               "flash_bwd_ds: alignment");
  if (a->dq)
    PZ_CHECK_ARG(a->k && PZ_ALIGNED(a->k, 16) && a->ldk % 8 == 0 && a->k_bstride % 8 == 0 && PZ_ALIGNED(a->dq, 8) &&
                     a->ldq % 4 == 0 && a->q_bstride % 4 == 0,
                 "flash_bwd_ds: dQ needs K (16-byte rows) and an 8-byte aligned dQ");
  PZ_CHECK_ARG(a->Z * a->H < 65536, "flash_bwd_ds: too many units");
  const int64_t units = a->Z * a->H, nqb = (a->nq + JP_NW * 16 - 1) / (JP_NW * 16);
  static bool attr = false;
  fa_smem_attr(flash_bwd_ds_dma_kernel, JD_SMEM, attr);
  hipLaunchKernelGGL(flash_bwd_ds_dma_kernel, dim3((unsigned)(nqb * units)), dim3(JP_NW * 64), JD_SMEM,
                     (hipStream_t)stream, *a, (const bf16_t*)P, (const bf16_t*)tcap, (bf16_t*)dS, ldp);
  PZ_CHECK_LAUNCH();
  return PZ_OK;
}

extern "C" int pz_flash_bwd_prep(const pz_flash_args* a, void* stream) {
  PZ_CHECK_ARG(a && a->delta && a->n_groups >= 1 && a->n_groups <= 3, "flash_bwd_prep: bad args");
  for (int i = 0; i < a->n_groups; ++i) PZ_CHECK_ARG(a->g_o[i] && a->g_do[i], "flash_bwd_prep: group %d", i);
  const int64_t rows = a->Z * a->H * a->nq;
  PZ_CHECK_ARG(fa_hd_ok(a->head_dim), "flash_bwd_prep: head_dim");
  FA_DISPATCH(a->head_dim, flash_bwd_prep_kernel, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, (hipStream_t)stream,
              *a);
  PZ_CHECK_LAUNCH();
  return PZ_OK;
}

extern "C" int pz_flash_bwd(const pz_flash_args* a, void* stream) {
  PZ_CHECK_ARG(a && a->lse && a->delta && a->dq && a->dk && a->dv, "flash_bwd: bad args");
  PZ_CHECK_ARG(fa_hd_ok(a->head_dim), "flash_bwd: head_dim");
  PZ_CHECK_ARG(PZ_ALIGNED(a->dq, 16) && PZ_ALIGNED(a->dk, 16) && PZ_ALIGNED(a->dv, 16), "flash_bwd: alignment");
  for (int i = 0; i < a->n_groups; ++i) PZ_CHECK_ARG(a->g_do[i] && a->g_ld[i] % 8 == 0, "flash_bwd: dO group %d", i);
  hipStream_t st = (hipStream_t)stream;
  // query split of the dK/dV pass when it has too few workgroups to fill the chip (joint MQA: 5 key
  // blocks per sample); fp32 partials in the caller's workspace, summed by a second pass
  const int64_t nkb = (a->nk + FA_KB - 1) / FA_KB;
  int64_t splits = 1;
  if (a->ws && a->head_dim % 4 == 0) {
    splits = (1024 + nkb * a->Z * a->H - 1) / (nkb * a->Z * a->H);
    splits = splits < 8 ? splits : 8;
    while (splits > 1 && splits * 2 * a->Z * a->H * a->nk * a->head_dim * 4 > a->ws_bytes) --splits;
  }
  // dQ pass first: it also writes delta, which the dK/dV pass reads
  if (fa_resident(a) && fa_unit(a)) {
    static bool aq = false, akv = false, aq2 = false, akv2 = false, aq3 = false, akv3 = false;
    const dim3 gu((unsigned)(a->Z * a->H));
    if (fa_sig(a)) {  // delta pass, then the persistent dQ and dK / dV kernels
      const int G = fa_sig_grid(a);
      fa_smem_attr(flash_bwd_kv_sig_kernel, FS_SMEM, akv3);
      (void)aq3;
      {
        static bool aq4 = false;
        fa_smem_attr(flash_bwd_q_sig_kernel<true>, FS_SMEM, aq4);
        hipLaunchKernelGGL(flash_bwd_q_sig_kernel<true>, dim3((unsigned)G), dim3(FS_NW * 64), FS_SMEM, st, *a, G);
      }
      PZ_CHECK_LAUNCH();
      hipLaunchKernelGGL(flash_bwd_kv_sig_kernel, dim3((unsigned)G), dim3(FS_NW * 64), FS_SMEM, st, *a, G);
    } else if (fa_plain(a)) {
      fa_smem_attr(flash_bwd_q_unit_kernel<72, true>, FR_SMEM_KQ, aq);
      fa_smem_attr(flash_bwd_kv_unit_kernel<72, true>, FU_SMEM_KV, akv);
      hipLaunchKernelGGL((flash_bwd_q_unit_kernel<72, true>), gu, dim3(FU_NW * 64), FR_SMEM_KQ, st, *a);
      PZ_CHECK_LAUNCH();
      hipLaunchKernelGGL((flash_bwd_kv_unit_kernel<72, true>), gu, dim3(FU_NW * 64), FU_SMEM_KV, st, *a);
    } else {
      fa_smem_attr(flash_bwd_q_unit_kernel<72, false>, FR_SMEM_KQ, aq2);
      fa_smem_attr(flash_bwd_kv_unit_kernel<72, false>, FU_SMEM_KV, akv2);
      hipLaunchKernelGGL((flash_bwd_q_unit_kernel<72, false>), gu, dim3(FU_NW * 64), FR_SMEM_KQ, st, *a);
      PZ_CHECK_LAUNCH();
      hipLaunchKernelGGL((flash_bwd_kv_unit_kernel<72, false>), gu, dim3(FU_NW * 64), FU_SMEM_KV, st, *a);
    }
    PZ_CHECK_LAUNCH();
    return PZ_OK;
  }
  if (fa_resident(a)) {
    static bool aq = false, akv = false;
    fa_smem_attr(flash_bwd_q_res_kernel<72>, FR_SMEM_KQ, aq);
    fa_smem_attr(flash_bwd_kv_res_kernel<72>, FR_SMEM_KV, akv);
    hipLaunchKernelGGL(flash_bwd_q_res_kernel<72>, dim3((unsigned)((a->nq + FR_NW * 16 - 1) / (FR_NW * 16) * a->Z * a->H)),
                       dim3(FR_NW * 64), FR_SMEM_KQ, st, *a);
    PZ_CHECK_LAUNCH();
    hipLaunchKernelGGL(flash_bwd_kv_res_kernel<72>, dim3((unsigned)(nkb * a->Z * a->H)), dim3(FR_NW * 64),
                       FR_SMEM_KV, st, *a);
    PZ_CHECK_LAUNCH();
    return PZ_OK;
  }
  const int fm = fa_fast_bwd(a);
  {
    const int64_t units = a->Z * a->H, nqb = (a->nq + JQ_NW * 32 - 1) / (JQ_NW * 32);
    const dim3 gq2((unsigned)(nqb * units));
    if (fm == 2) {
      FA_DISPATCH(a->head_dim, FA_T2(flash_bwd_q2_kernel, true), gq2, dim3(JQ_NW * 64), 0, st, *a);
    } else {
      FA_DISPATCH(a->head_dim, FA_T2(flash_bwd_q2_kernel, false), gq2, dim3(JQ_NW * 64), 0, st, *a);
    }
  }
  PZ_CHECK_LAUNCH();
  const dim3 gkv1((unsigned)(nkb * a->Z * a->H * splits));
  if (fm == 2) {
    FA_DISPATCH(a->head_dim, FA_T2(flash_bwd_kv_kernel, 2), gkv1, dim3(FA_NW * 64), 0, st, *a, (int)splits);
  } else {
    FA_DISPATCH(a->head_dim, FA_T2(flash_bwd_kv_kernel, 1), gkv1, dim3(FA_NW * 64), 0, st, *a, (int)splits);
  }
  if (splits > 1) {
    PZ_CHECK_LAUNCH();
    const int64_t n4 = 2 * a->Z * a->H * a->nk * (a->head_dim / 4);
    FA_DISPATCH(a->head_dim, flash_bwd_kv_reduce_kernel, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, st, *a,
                (int)splits);
  }
  PZ_CHECK_LAUNCH();
  return PZ_OK;
}

extern "C" int pz_flash_fwd_f8(const pz_flash_args* a, const void* qc, const float* qs, const void* kc, const float* ks,
                               int64_t krows, const void* vtc, const float* vs, int64_t ldvt, void* stream) {
  PZ_CHECK_ARG(a && qc && qs && kc && ks && vtc && vs && a->Z > 0 && a->nq > 0 && a->nk > 0 && a->H == 1,
               "flash_fwd_f8: bad args (one K / V head: H == 1)");
  PZ_CHECK_ARG(a->head_dim == 256, "flash_fwd_f8: head_dim %lld (256 only)", (long long)a->head_dim);
  PZ_CHECK_ARG(krows >= a->nk && ldvt >= (a->nk + F8_KB - 1) / F8_KB * F8_KB && ldvt % 16 == 0,
               "flash_fwd_f8: krows %lld / ldvt %lld (ldvt >= nk rounded up to 128)", (long long)krows,
               (long long)ldvt);
  PZ_CHECK_ARG(PZ_ALIGNED(qc, 16) && PZ_ALIGNED(kc, 16) && PZ_ALIGNED(vtc, 16) && PZ_ALIGNED(vs, 16),
               "flash_fwd_f8: 16-byte aligned codes / scales");
  PZ_CHECK_ARG(a->n_groups >= 1 && a->n_groups <= 3 && a->g_row0[0] == 0 && a->o_hstride == 0, "flash_fwd_f8: groups");
  for (int i = 0; i < a->n_groups; ++i) PZ_CHECK_ARG(a->g_o[i] && a->g_ld[i] % 4 == 0, "flash_fwd_f8: group %d", i);
  PZ_CHECK_ARG(a->mask_mode == 0 || (a->mask_mode == 1 && a->cnt && a->rows_per_token > 0), "flash_fwd_f8: mask");
  PZ_CHECK_ARG(a->nq + a->mask_row0 < (1 << 22) && a->Z < 65536, "flash_fwd_f8: nq / Z too large");
  const int64_t qblk = (a->nq + 127) / 128, nkb = (a->nk + F8_KB - 1) / F8_KB;
  // key split (few query blocks: the B = 1 prefill) into the caller's workspace; PZ_F8_SPLIT "0": never (A/B), "1":
  // whenever fewer than 128 workgroups (read per call)
  const char* esp = getenv("PZ_F8_SPLIT");
  const bool split_ok = !(esp && esp[0] == '0');
  int64_t sp = 1;
  if (split_ok && a->ws && qblk * a->Z < 128 && nkb > 1) {
    sp = (256 + qblk * a->Z - 1) / (qblk * a->Z);
    sp = sp < nkb ? sp : nkb;
    sp = sp < 16 ? sp : 16;
    while (sp > 1 && sp * a->Z * a->nq * (256 + 2) * 4 > a->ws_bytes) --sp;
    const int64_t per = (nkb + sp - 1) / sp;
    sp = (nkb + per - 1) / per;
  }
  static bool attr = false;
  fa_smem_attr(flash_fwd_f8_kernel, F8_SMEM, attr);
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(flash_fwd_f8_kernel, dim3((unsigned)qblk, (unsigned)a->Z, (unsigned)sp), dim3(512), F8_SMEM, st, *a,
                     (const uint8_t*)qc, qs, (const uint8_t*)kc, ks, krows, (const uint8_t*)vtc, vs, ldvt);
  PZ_CHECK_LAUNCH();
  if (sp > 1) {
    const int64_t n = a->Z * a->nq * 64;
    hipLaunchKernelGGL(flash_fwd_combine_kernel<256>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, *a, (int)sp);
    PZ_CHECK_LAUNCH();
  }
  return PZ_OK;
}
