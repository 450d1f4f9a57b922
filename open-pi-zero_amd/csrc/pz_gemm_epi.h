// GEMM argument block and the shared epilogue helpers (pz_gemm.hip, pz_gemm_rows.hip).
// GemmP is a plain struct with ONE definition (both translation units include this header);
// the device helpers live in an anonymous namespace (each TU inlines its own copies).
#pragma once

#include <type_traits>

#include "pz_common.h"

struct GemmP {
  const bf16_t* A;
  const bf16_t* B;
  void* C;
  const bf16_t* bias;
  const bf16_t* resid;
  bf16_t* aux;
  int64_t M, N, K, lda, ldb, ldc, ld_resid, ld_aux, geglu_I;
  int64_t batch_inner, sAo, sAi, sBo, sBi, sCo, sCi, sRo, sRi;
  int tiles_m, tiles_n, epi, c_fp32, beta;
  float alpha;
  // split-K (batch-1 only): blockIdx.y = split index; raw fp32 partials -> ws[z][M][ldw]
  float* ws;
  int64_t ksplit, ldw;
  // skinny-64 split-K combined inside the launch (gemm_skinny64_kernel): first arrival counter of this launch's
  // tiles in g_sk_ctr; -1 = partials summed by a separate splitk_epilogue_kernel launch
  int sk_tk;
  // batched 128-tile launches (gemm_kernel, batch % 8 == 0, no split-K): 1-D grid, the tiles of one batch
  // entry on one XCD so its operand panels are shared in that XCD's L2 (batch_xcd = number of batch entries)
  int batch_xcd;
  // 8-phase split tail (batch-1 only, tail_s > 0): work units [0, dp_tiles) are whole tiles; unit
  // dp_tiles + u is K-piece (u % tail_s) (tail_kt K-tiles) of tile dp_tiles + u / tail_s, whose raw
  // accumulators go to ws[u] (256 KiB, thread-major) for gemm8p_tail_epilogue.
  int dp_tiles, tail_s, tail_kt;
  // fused Gemma RMSNorm of the A rows (skinny path only): bf16 (1 + w) weights [K] or NULL
  const bf16_t* nw;
  float neps;
  // fp8 W8A8 (gemm8p_f8_kernel): per-row activation scales [M] or NULL
  const float* rs;
  // measurement knob (PZ_GEMM_DBG, read per call): 1 = the 8-phase kernels skip their epilogue stores
  // (tools/epi_probe.py: main-loop time alone); 0 in every product run
  int dbg;
  // fused q|k|v RoPE epilogue (pz_gemm_qkv_rope; 8-phase kernel, head_dim 256 = one column tile per head):
  // the bf16-rounded projection of head n0/256 is rotated at rpos[m] (table rcs) and scattered into the
  // joint Q / K / V buffers like pz_qkv_rope_split; C is not written.  rcs == NULL: off.
  const int64_t* rpos;
  const float* rcs;
  bf16_t *rq, *rk, *rv;
  int64_t rT, rnh, rLq, rqoff, rLk, rkoff;
  // 8-phase LDS-staged epilogues: non-temporal (streaming) 16-B output stores (PZ_GEMM_NT, read per call)
  int nt_store;
  // ... and for the saved activations only (aux: GeGLU g|u, GELU / SiLU pre-activation -- read again only by the
  // backward, long after; PZ_GEMM_NT_AUX, read per call)
  int nt_aux;
  // super-row height of the 8-phase kernels' tile order (tile_coords; PZ_GEMM_GROUP, read per call; default 8)
  int group;
};

namespace {

// bijective XCD-aware remap + grouped (super-row) tile order
__device__ __forceinline__ void tile_coords(int bid, int nwg, int tiles_m, int tiles_n, int& tm, int& tn,
                                            int GROUP = 8) {
  const int xcd = bid & 7, local = bid >> 3;
  const int q = nwg >> 3, r = nwg & 7;
  const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + local;
  GROUP = GROUP >= 1 ? GROUP : 8;
  const int per_group = GROUP * tiles_n;
  const int g = wg / per_group;
  const int first_m = g * GROUP;
  const int gsize = min(tiles_m - first_m, GROUP);
  const int in = wg - g * per_group;
  tm = first_m + in % gsize;
  tn = in / gsize;
}

// ---- epilogue: one lane owns C[m][n..n+3] (swapped-operand MFMA layout) -------
// Side inputs of the epilogue (residual, saved activations, old C for beta accumulation, bias) are
// loaded by epi_load4 into raw registers and consumed by epi_store4.  Kernels that own many output
// groups per lane issue the loads of the next groups before the stores of the current ones: the
// pointers may alias C (resid == C, DGEGLU in place), so the compiler cannot hoist a load above an
// earlier store by itself and would otherwise pay one memory round trip per 4-column group.
struct Side {
  u32x4 w;  // .xy: aux (DGELU/DSILU pre-activation, DGEGLU g) or old bf16 C (beta); .zw: resid or DGEGLU u
            // (fp32 C with beta: all four lanes hold the old fp32 values)
};

__device__ __forceinline__ u32x2 ld4bf(const bf16_t* X, bool full, int64_t n, int64_t N) {
  if (full) return *reinterpret_cast<const u32x2*>(X);
  unsigned h[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) h[r] = n + r < N ? (unsigned)X[r] : 0u;
  return u32x2{h[0] | (h[1] << 16), h[2] | (h[3] << 16)};
}
__device__ __forceinline__ void unpack4(u32x2 w, float (&o)[4]) {
  o[0] = __uint_as_float(w[0] << 16); o[1] = __uint_as_float(w[0] & 0xffff0000u);
  o[2] = __uint_as_float(w[1] << 16); o[3] = __uint_as_float(w[1] & 0xffff0000u);
}
__device__ __forceinline__ void store4(bf16_t* X, bool full, int64_t n, int64_t N, const float (&v)[4]) {
  if (full) {
    *reinterpret_cast<u32x2*>(X) = u32x2{pack2bf(v[0], v[1]), pack2bf(v[2], v[3])};
  } else {
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (n + r < N) X[r] = f2bf(v[r]);
  }
}

__device__ __forceinline__ u32x2 epi_load_bias(const GemmP& p, int64_t n) {
  if (!p.bias || n >= p.N) return u32x2{0u, 0u};
  return ld4bf(p.bias + n, n + 4 <= p.N, n, p.N);
}

// epilogue classes (compile-time, so each fully unrolled 8-phase epilogue carries one class's code)
enum EpiMode { EM_BF16 = 0, EM_F32 = 1, EM_DACT = 2, EM_DGEGLU = 3 };

template <int EM>
__device__ __forceinline__ void epi_load4(const GemmP& p, int64_t cofs, int64_t rofs, int64_t m, int64_t n,
                                          Side& s) {
  s.w = u32x4{0u, 0u, 0u, 0u};
  if (m >= p.M || n >= p.N) return;
  const bool full = n + 4 <= p.N;
  if constexpr (EM == EM_DGEGLU) {
    const bf16_t* X = p.aux + m * p.ld_aux + n;
    const u32x2 g = ld4bf(X, full, n, p.N), u = ld4bf(X + p.geglu_I, full, n, p.N);
    s.w = u32x4{g[0], g[1], u[0], u[1]};
  } else if constexpr (EM == EM_DACT) {
    const u32x2 x = ld4bf(p.aux + m * p.ld_aux + n, full, n, p.N);
    s.w = u32x4{x[0], x[1], 0u, 0u};
  } else if constexpr (EM == EM_F32) {
    if (p.beta) {
      const float* Cp = reinterpret_cast<const float*>(p.C) + cofs + m * p.ldc + n;
      if (full) {
        s.w = *reinterpret_cast<const u32x4*>(Cp);
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) s.w[r] = n + r < p.N ? __float_as_uint(Cp[r]) : 0u;
      }
    } else if (p.resid) {
      const u32x2 x = ld4bf(p.resid + rofs + m * p.ld_resid + n, full, n, p.N);
      s.w = u32x4{0u, 0u, x[0], x[1]};
    }
  } else {
    u32x2 x0{0u, 0u}, x1{0u, 0u};
    if (p.resid) x1 = ld4bf(p.resid + rofs + m * p.ld_resid + n, full, n, p.N);
    if (p.beta) x0 = ld4bf(reinterpret_cast<const bf16_t*>(p.C) + cofs + m * p.ldc + n, full, n, p.N);
    s.w = u32x4{x0[0], x0[1], x1[0], x1[1]};
  }
}

template <int EM>
__device__ __forceinline__ void epi_store4(const GemmP& p, int64_t cofs, int64_t rofs, int64_t m, int64_t n,
                                           const f32x4& acc, const Side& s, u32x2 bias) {
  if (m >= p.M || n >= p.N) return;
  const bool full = n + 4 <= p.N;
  float v[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) v[r] = acc[r] * p.alpha;
  float x0[4], x1[4];
  unpack4(u32x2{s.w[0], s.w[1]}, x0);
  unpack4(u32x2{s.w[2], s.w[3]}, x1);
  bf16_t* Cb = reinterpret_cast<bf16_t*>(p.C) + cofs + m * p.ldc + n;
  if constexpr (EM == EM_DGEGLU) {  // GeGLU backward from saved [g | u]: two outputs, nothing else applies
    float dg[4], du[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float gl_, gr_;
      gelu_tanh_both(x0[r], gl_, gr_);
      dg[r] = v[r] * x1[r] * gr_;
      du[r] = v[r] * gl_;
    }
    store4(Cb, full, n, p.N, dg);
    store4(Cb + p.geglu_I, full, n, p.N, du);
  } else if constexpr (EM == EM_DACT) {  // activation backward from the saved pre-activation
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] *= p.epi == PZ_EPI_DGELU ? gelu_tanh_grad(x0[r]) : silu_grad(x0[r]);
    store4(Cb, full, n, p.N, v);
  } else {
    if (p.bias) {
      float b[4];
      unpack4(bias, b);
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] += b[r];
    }
    if (p.epi == PZ_EPI_GELU || p.epi == PZ_EPI_SILU) {
      if (p.aux) store4(p.aux + m * p.ld_aux + n, full, n, p.N, v);
      if (p.epi == PZ_EPI_GELU) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = gelu_tanh(v[r]);
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = silu(v[r]);
      }
    }
    if constexpr (EM == EM_F32) {
      if (p.beta) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] += __uint_as_float(s.w[r]);
      } else if (p.resid) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] += x1[r];
      }
      float* Cp = reinterpret_cast<float*>(p.C) + cofs + m * p.ldc + n;
      if (full) {
        *reinterpret_cast<f32x4*>(Cp) = f32x4{v[0], v[1], v[2], v[3]};
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (n + r < p.N) Cp[r] = v[r];
      }
    } else {
      if (p.resid) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] += x1[r];
      }
      if (p.beta) {
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] += x0[r];
      }
      store4(Cb, full, n, p.N, v);
    }
  }
}

__device__ __forceinline__ int epi_mode(const GemmP& p) {
  if (p.epi == PZ_EPI_DGEGLU) return EM_DGEGLU;
  if (p.epi == PZ_EPI_DGELU || p.epi == PZ_EPI_DSILU) return EM_DACT;
  return p.c_fp32 ? EM_F32 : EM_BF16;
}

template <int EM>
__device__ __forceinline__ void store_out4_m(const GemmP& p, int64_t cofs, int64_t rofs, int64_t m, int64_t n,
                                             const f32x4& acc) {
  Side s;
  epi_load4<EM>(p, cofs, rofs, m, n, s);
  epi_store4<EM>(p, cofs, rofs, m, n, acc, s, epi_load_bias(p, n));
}

// one group, runtime-general (edge tiles of the 8-phase kernel: one compact copy per group)
__device__ __forceinline__ void store_out4_rt(const GemmP& p, int64_t cofs, int64_t rofs, int64_t m, int64_t n,
                                              const f32x4& acc) {
  if (m >= p.M || n >= p.N) return;
  const bool full = n + 4 <= p.N;
  float v[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) v[r] = acc[r] * p.alpha;
  if (p.epi == PZ_EPI_DGEGLU) {
    float g[4], u[4], dg[4], du[4];
    const bf16_t* X = p.aux + m * p.ld_aux + n;
    unpack4(ld4bf(X, full, n, p.N), g);
    unpack4(ld4bf(X + p.geglu_I, full, n, p.N), u);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float gl_, gr_;
      gelu_tanh_both(g[r], gl_, gr_);
      dg[r] = v[r] * u[r] * gr_;
      du[r] = v[r] * gl_;
    }
    bf16_t* Cp = reinterpret_cast<bf16_t*>(p.C) + cofs + m * p.ldc + n;
    store4(Cp, full, n, p.N, dg);
    store4(Cp + p.geglu_I, full, n, p.N, du);
    return;
  }
  if (p.epi == PZ_EPI_DGELU || p.epi == PZ_EPI_DSILU) {
    float x[4];
    unpack4(ld4bf(p.aux + m * p.ld_aux + n, full, n, p.N), x);
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] *= p.epi == PZ_EPI_DGELU ? gelu_tanh_grad(x[r]) : silu_grad(x[r]);
  }
  if (p.bias) {
    float b[4];
    unpack4(ld4bf(p.bias + n, full, n, p.N), b);
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] += b[r];
  }
  if (p.epi == PZ_EPI_GELU || p.epi == PZ_EPI_SILU) {
    if (p.aux) store4(p.aux + m * p.ld_aux + n, full, n, p.N, v);
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = p.epi == PZ_EPI_GELU ? gelu_tanh(v[r]) : silu(v[r]);
  }
  if (p.resid) {
    float x[4];
    unpack4(ld4bf(p.resid + rofs + m * p.ld_resid + n, full, n, p.N), x);
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] += x[r];
  }
  if (p.c_fp32) {
    float* Cp = reinterpret_cast<float*>(p.C) + cofs + m * p.ldc + n;
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (full || n + r < p.N) Cp[r] = p.beta ? Cp[r] + v[r] : v[r];
  } else {
    bf16_t* Cp = reinterpret_cast<bf16_t*>(p.C) + cofs + m * p.ldc + n;
    if (p.beta) {
      float o[4];
      unpack4(ld4bf(Cp, full, n, p.N), o);
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] += o[r];
    }
    store4(Cp, full, n, p.N, v);
  }
}

// run f(std::integral_constant<int, EM>) for the epilogue class of p (one branch per launch, outside
// the unrolled per-group loops)
template <class F>
__device__ __forceinline__ void epi_dispatch(const GemmP& p, F&& f) {
  switch (epi_mode(p)) {
    case EM_DGEGLU: f(std::integral_constant<int, EM_DGEGLU>{}); break;
    case EM_DACT: f(std::integral_constant<int, EM_DACT>{}); break;
    case EM_F32: f(std::integral_constant<int, EM_F32>{}); break;
    default: f(std::integral_constant<int, EM_BF16>{}); break;
  }
}

// one group, loads then stores (kernels with few groups per lane)
__device__ __forceinline__ void store_out4(const GemmP& p, int64_t cofs, int64_t rofs, int64_t m, int64_t n,
                                           const f32x4& acc) {
  switch (epi_mode(p)) {
    case EM_DGEGLU: store_out4_m<EM_DGEGLU>(p, cofs, rofs, m, n, acc); break;
    case EM_DACT: store_out4_m<EM_DACT>(p, cofs, rofs, m, n, acc); break;
    case EM_F32: store_out4_m<EM_F32>(p, cofs, rofs, m, n, acc); break;
    default: store_out4_m<EM_BF16>(p, cofs, rofs, m, n, acc); break;
  }
}

// GeGLU: gate and up accumulators of the same (m, n..n+3) -> h = gelu_tanh(g) * u (+ saved g|u)
__device__ __forceinline__ void store_geglu4(const GemmP& p, int64_t cofs, int64_t m, int64_t n, const f32x4& ga,
                                             const f32x4& ua) {
  if (m >= p.M || n >= p.geglu_I) return;
  float h[4], g[4], u[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    g[r] = ga[r] * p.alpha;
    u[r] = ua[r] * p.alpha;
    h[r] = gelu_tanh(g[r]) * u[r];
  }
  bf16_t* Cp = reinterpret_cast<bf16_t*>(p.C) + cofs + m * p.ldc + n;
  *reinterpret_cast<u32x2*>(Cp) = u32x2{pack2bf(h[0], h[1]), pack2bf(h[2], h[3])};
  if (p.aux) {
    bf16_t* X = p.aux + m * p.ld_aux + n;
    *reinterpret_cast<u32x2*>(X) = u32x2{pack2bf(g[0], g[1]), pack2bf(g[2], g[3])};
    *reinterpret_cast<u32x2*>(X + p.geglu_I) = u32x2{pack2bf(u[0], u[1]), pack2bf(u[2], u[3])};
  }
}
}  // namespace
// row-slab GEMM launcher (pz_gemm_rows.hip): w waves, tnb 16-column blocks per 64-row tile
int pz_rows_launch(const GemmP& p, int w, int tnb, bool geglu, int f8w, hipStream_t st);
// skinny-64 GEMM launcher (pz_gemm_rows.hip): 16 < M <= 64 rows (and fp8-weight W8A16), w waves, nc columns
// per block, mb 16-row blocks
int pz_sk64_launch(const GemmP& p, int w, int nc, int mb, bool f8w, int64_t tiles_n, hipStream_t st);
// tall-tile GEMM launcher (pz_gemm_tall.hip): 64 * mi rows per tile, k-contiguous A, B k-contiguous or (plain
// epilogues) k-strided, split-K over blockIdx.y when splits > 1
int pz_tall_launch(const GemmP& p, int mi, bool geglu, bool bkc, int splits, hipStream_t st);
// split-K second pass (pz_gemm.hip): C = epilogue(sum of the S fp32 partial slabs in p.ws)
int pz_splitk_epi_launch(const GemmP& p, int S, hipStream_t st);
