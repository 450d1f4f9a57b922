// Few-row (skinny-64) and row-slab GEMM kernels (own translation unit: pz_gemm.hip takes minutes to compile).
#include <atomic>

#include "pz_gemm_epi.h"

namespace {

__device__ __forceinline__ void fp8x16_to_bf16(const u32x4 q, bf16x8& lo, bf16x8& hi) {
  typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
  bf16x2 h[8];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    h[2 * e] = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8((int)q[e], 1.f, false);
    h[2 * e + 1] = __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8((int)q[e], 1.f, true);
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    lo[2 * e] = h[e][0];
    lo[2 * e + 1] = h[e][1];
    hi[2 * e] = h[4 + e][0];
    hi[2 * e + 1] = h[4 + e][1];
  }
}

// -------------------------------------------------------------------------
// Row-slab GEMM for 64 < M <= 512 rows with k-contiguous A [M][K] and B [N][K]: the forward (NT) GEMMs
// of the B = 1 SigLIP / Gemma prefill (256 / 276 rows) and of the action expert's training rows
// (64 samples x 5 = 320).  One workgroup owns a (16 TMB) x (16 TNB) output tile over the WHOLE K: no
// split-K partials and no second launch (the 128-tile + split-K pair it replaces spent ~20 us per GEMM
// on one K-tile in flight and a partial-sum round trip).  The W waves split K into contiguous ranges
// of 64-chunks and stream their MFMA fragments straight from global into VGPRs, two register buffers
// (chunk c + 1's loads issued before chunk c's MFMAs):
// lane group g takes k = 64c + 32h + 8g + [0, 8) of a row, so a row's 64-B half-line is read by 4
// adjacent lanes per instruction.  The W partial tiles are summed through LDS in fixed wave order
// (deterministic) and each wave finishes a share of the 16 x 16 blocks through the shared forward
// epilogues (bias, GELU / SiLU (+ aux), GeGLU (+ g|u), residual, beta, fp32 C).  K % 8 == 0: a last
// partial 64-chunk zeroes its 8-element pieces past K.  Tiles of one column slab are consecutive in
// tile_coords' order, i.e. on one XCD (their weight slice is read from HBM once per L2).
// -------------------------------------------------------------------------
// F8W: B holds OCP e4m3 codes [N][K] (ldb in codes; W8A16, the C5 prefill's fp8 weights at 768-789 rows): lane
// group g takes k = 64c + 16g + [0, 16) -- the A row's two bf16x8 and ONE 16-B load of 16 codes expanded exactly
// to bf16 (skinny-64's mapping); the weight scale is alpha.  K % 64 == 0.
template <int W, int TMB, int TNB, bool GEGLU, bool F8W = false>
__global__ void __launch_bounds__(W * 64, W == 4 ? 2 : 1) gemm_rows_kernel(GemmP p) {
  constexpr int NB = TMB * TNB, NS = GEGLU ? 2 : 1;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  f32x4* red = reinterpret_cast<f32x4*>(smem);  // [W][NS][NB][64]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, rl = lane & 15;
  const int64_t ncols = GEGLU ? p.geglu_I : p.N;
  int tm, tn;
  tile_coords(blockIdx.x, gridDim.x, p.tiles_m, p.tiles_n, tm, tn);
  const int64_t m0 = (int64_t)tm * (16 * TMB), n0 = (int64_t)tn * (16 * TNB);
  // rows / columns past the edge are clamped onto the last one (finite data, never stored)
  constexpr int AG = F8W ? 16 : 8;  // k offset of lane group g within a 64-chunk half
  const bf16_t* Ar[TMB];
  const bf16_t* Br[NS][TNB];
  const unsigned char* Bq[NS][TNB];  // F8W: code rows
#pragma unroll
  for (int mb = 0; mb < TMB; ++mb) Ar[mb] = p.A + min(m0 + 16 * mb + rl, p.M - 1) * p.lda + AG * g;
#pragma unroll
  for (int nb = 0; nb < TNB; ++nb) {
    const int64_t col = min(n0 + 16 * nb + rl, ncols - 1);
    Br[0][nb] = p.B + col * p.ldb + 8 * g;
    Bq[0][nb] = reinterpret_cast<const unsigned char*>(p.B) + col * p.ldb + 16 * g;
    if (GEGLU) {
      Br[NS - 1][nb] = p.B + (p.geglu_I + col) * p.ldb + 8 * g;
      Bq[NS - 1][nb] = reinterpret_cast<const unsigned char*>(p.B) + (p.geglu_I + col) * p.ldb + 16 * g;
    }
  }
  const int nfull = (int)(p.K / 64), nch = (int)((p.K + 63) / 64);  // nch > nfull: a last partial chunk
  const int per = (nch + W - 1) / W;
  const int kb = min(nch, wave * per), ke = min(nch, kb + per), kf = min(ke, nfull);
  f32x4 acc[NS][TMB][TNB];
#pragma unroll
  for (int s = 0; s < NS; ++s)
#pragma unroll
    for (int mb = 0; mb < TMB; ++mb)
#pragma unroll
      for (int nb = 0; nb < TNB; ++nb) acc[s][mb][nb] = f32x4{0.f, 0.f, 0.f, 0.f};
  // two register buffers: chunk c + 1's loads are issued before chunk c's MFMAs (software pipeline)
  bf16x8 fa[2][TMB][2], fb[2][NS][TNB][2];
  auto load = [&](auto B_, int c, bool partial) {
    constexpr int bi = decltype(B_)::value;
    if constexpr (F8W) {  // (host: K % 64 == 0, no partial chunk)
#pragma unroll
      for (int mb = 0; mb < TMB; ++mb) {
        fa[bi][mb][0] = *reinterpret_cast<const bf16x8*>(Ar[mb] + (int64_t)c * 64);
        fa[bi][mb][1] = *reinterpret_cast<const bf16x8*>(Ar[mb] + (int64_t)c * 64 + 8);
      }
#pragma unroll
      for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int nb = 0; nb < TNB; ++nb)
          fp8x16_to_bf16(*reinterpret_cast<const u32x4*>(Bq[s][nb] + (int64_t)c * 64), fb[bi][s][nb][0],
                         fb[bi][s][nb][1]);
      return;
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int64_t ko = (int64_t)c * 64 + 32 * h;
      // last partial chunk: 8-element pieces past K read a clamped in-bounds piece and are zeroed
      const bool ok = !partial || ko + 8 * g < p.K;
      const int64_t kl = ok ? ko : 0;
#pragma unroll
      for (int mb = 0; mb < TMB; ++mb) fa[bi][mb][h] = *reinterpret_cast<const bf16x8*>(Ar[mb] + kl);
#pragma unroll
      for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int nb = 0; nb < TNB; ++nb) fb[bi][s][nb][h] = *reinterpret_cast<const bf16x8*>(Br[s][nb] + kl);
      if (partial && !ok) {
#pragma unroll
        for (int mb = 0; mb < TMB; ++mb) fa[bi][mb][h] = bf16x8{};
      }
    }
  };
  auto mma = [&](auto B_) {
    constexpr int bi = decltype(B_)::value;
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int mb = 0; mb < TMB; ++mb)
#pragma unroll
          for (int nb = 0; nb < TNB; ++nb)
            acc[s][mb][nb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[bi][s][nb][h], fa[bi][mb][h], acc[s][mb][nb], 0, 0, 0);
  };
  const std::integral_constant<int, 0> B0;
  const std::integral_constant<int, 1> B1;
  int c = kb;
  if (c < kf) load(B0, c, false);
  while (c < kf) {
    if (c + 1 < kf) load(B1, c + 1, false);
    mma(B0);
    if (++c >= kf) break;
    if (c + 1 < kf) load(B0, c + 1, false);
    mma(B1);
    ++c;
  }
  if (nfull < nch && kb <= nfull && nfull < ke) {  // this wave owns the partial chunk
    load(B0, nfull, true);
    mma(B0);
  }
#pragma unroll
  for (int s = 0; s < NS; ++s)
#pragma unroll
    for (int mb = 0; mb < TMB; ++mb)
#pragma unroll
      for (int nb = 0; nb < TNB; ++nb) red[((wave * NS + s) * NB + mb * TNB + nb) * 64 + lane] = acc[s][mb][nb];
  __syncthreads();
  for (int blk = wave; blk < NB; blk += W) {
    f32x4 o[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) o[s] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int w = 0; w < W; ++w)
#pragma unroll
      for (int s = 0; s < NS; ++s) o[s] += red[((w * NS + s) * NB + blk) * 64 + lane];
    const int mb = blk / TNB, nb = blk % TNB;
    const int64_t m = m0 + 16 * mb + rl, n = n0 + 16 * nb + 4 * g;
    if (GEGLU) store_geglu4(p, 0, m, n, o[0], o[NS - 1]);
    else store_out4(p, 0, 0, m, n, o[0]);
  }
}

// -------------------------------------------------------------------------
// W8A8 row slab (C5's fp8 prefill q|k|v / o at 768-789 rows): the row-slab scheme with BOTH
// operands OCP e4m3 codes, on the fp8 MFMA.  p.K / p.lda / p.ldb arrive in code PAIRS (pz_gemm's W8A8 convention), so
// chunk c covers 128 codes (64 pairs) of a row; lane group g takes codes 128c + 32g + [0, 32) of the A row and of the
// B row (two 16-B loads each) and ONE v_mfma_f32_16x16x128_f8f6f4 sums them -- the same k set on both operands, so
// the plain dot product.  After the fixed-order LDS reduction each row's sum is scaled by its activation scale
// (p.rs[m]) and the weight scale (alpha, in the shared epilogue).  K % 128 codes == 0 (host-checked), no GeGLU.
template <int W, int TMB, int TNB>
__global__ void __launch_bounds__(W * 64, W == 4 ? 2 : 1) gemm_rows_f8a_kernel(GemmP p) {
  constexpr int NB = TMB * TNB;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  f32x4* red = reinterpret_cast<f32x4*>(smem);  // [W][NB][64]
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4, rl = lane & 15;
  int tm, tn;
  tile_coords(blockIdx.x, gridDim.x, p.tiles_m, p.tiles_n, tm, tn);
  const int64_t m0 = (int64_t)tm * (16 * TMB), n0 = (int64_t)tn * (16 * TNB);
  const unsigned char* Ar[TMB];
  const unsigned char* Br[TNB];
#pragma unroll
  for (int mb = 0; mb < TMB; ++mb)
    Ar[mb] = reinterpret_cast<const unsigned char*>(p.A) + min(m0 + 16 * mb + rl, p.M - 1) * (2 * p.lda) + 32 * g;
#pragma unroll
  for (int nb = 0; nb < TNB; ++nb)
    Br[nb] = reinterpret_cast<const unsigned char*>(p.B) + min(n0 + 16 * nb + rl, p.N - 1) * (2 * p.ldb) + 32 * g;
  const int nch = (int)(p.K / 64);  // 128-code chunks
  const int per = (nch + W - 1) / W;
  const int kb = min(nch, wave * per), ke = min(nch, kb + per);
  f32x4 acc[TMB][TNB];
#pragma unroll
  for (int mb = 0; mb < TMB; ++mb)
#pragma unroll
    for (int nb = 0; nb < TNB; ++nb) acc[mb][nb] = f32x4{0.f, 0.f, 0.f, 0.f};
  i32x8 fa[2][TMB], fb[2][TNB];
  auto ld32 = [](const unsigned char* q) {
    const u32x4 lo = *reinterpret_cast<const u32x4*>(q), hi = *reinterpret_cast<const u32x4*>(q + 16);
    return i32x8{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2], (int)hi[3]};
  };
  auto load = [&](auto B_, int c) {
    constexpr int bi = decltype(B_)::value;
#pragma unroll
    for (int mb = 0; mb < TMB; ++mb) fa[bi][mb] = ld32(Ar[mb] + (int64_t)c * 128);
#pragma unroll
    for (int nb = 0; nb < TNB; ++nb) fb[bi][nb] = ld32(Br[nb] + (int64_t)c * 128);
  };
  auto mma = [&](auto B_) {
    constexpr int bi = decltype(B_)::value;
#pragma unroll
    for (int mb = 0; mb < TMB; ++mb)
#pragma unroll
      for (int nb = 0; nb < TNB; ++nb)
        acc[mb][nb] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(fb[bi][nb], fa[bi][mb], acc[mb][nb], 0, 0, 0, 0,
                                                                        0, 0);
  };
  const std::integral_constant<int, 0> B0;
  const std::integral_constant<int, 1> B1;
  int c = kb;
  if (c < ke) load(B0, c);
  while (c < ke) {
    if (c + 1 < ke) load(B1, c + 1);
    mma(B0);
    if (++c >= ke) break;
    if (c + 1 < ke) load(B0, c + 1);
    mma(B1);
    ++c;
  }
#pragma unroll
  for (int mb = 0; mb < TMB; ++mb)
#pragma unroll
    for (int nb = 0; nb < TNB; ++nb) red[(wave * NB + mb * TNB + nb) * 64 + lane] = acc[mb][nb];
  __syncthreads();
  for (int blk = wave; blk < NB; blk += W) {
    f32x4 o = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int w = 0; w < W; ++w) o += red[(w * NB + blk) * 64 + lane];
    const int mb = blk / TNB, nb = blk % TNB;
    const int64_t m = m0 + 16 * mb + rl, n = n0 + 16 * nb + 4 * g;
    o *= p.rs[min(m, p.M - 1)];
    store_out4(p, 0, 0, m, n, o);
  }
}

// -------------------------------------------------------------------------
// Skinny GEMM for 16 < M <= 64 rows, and for fp8 (OCP e4m3) weights at M <= 64 (W8A16): the C5
// denoise steps (an action chunk of 50 rows per sample).  The scheme of gemm_skinny_kernel -- W waves
// per NC output columns, K split into W contiguous ranges, weights streamed once into VGPRs, LDS
// reduction -- with MB 16-row blocks sharing every weight fragment (MB MFMAs per fragment; the
// activation rows are re-read from L2 by every block).  K is walked in 64-k chunks: lane group g
// takes k = 64c + 16g + [0, 16) of A (two bf16x8) and of B (two bf16x8, or ONE 16-byte load of fp8
// codes expanded in registers by v_cvt_scalef32_pk_bf16_fp8 -- exact, every e4m3 value is a bf16);
// the chunk's two MFMAs sum over k = 64c + 16g + [0, 8) and [8, 16), g = 0..3: the same k set on
// both operands, so the sum is the plain dot product.  The weight scale of fp8 codes is alpha.
// Requires K % 64 == 0, k-contiguous A and B, batch 1.
// -------------------------------------------------------------------------

// Split-K combined inside the launch (the C5 denoise o / down projections: 64 tiles x 4 K-slices): every slice
// writes its fp32 partial tile write-through (sc1, 16 B per lane) into a slab private to the tile
// (ws[z][tile][64][NC]: no 128-B line is shared by two tiles), drains its stores and joins a barrier; one lane adds to
// the tile's arrival counter (relaxed, agent scope); the slice that arrives last resets the counter and sums the S
// slabs in slice order with sc1 loads (L1 bypassed: cdna_hip_programming.md Guideline 16's counter hand-off, every
// store and load of the slabs sc1, so no release or acquire fence) and runs the epilogue, whose residual / bias
// loads every slice issued before the hand-off.  Same partials, same order: the bits of the two-launch form
// (splitk_epilogue_kernel), one kernel boundary less per projection.  Counters live in g_sk_ctr (zero at load,
// reset by each tile's reducer); the host hands every launch its own range (launch_sk64), so launches on concurrent
// streams never share one.
constexpr int SK_CTRS = 1 << 16;
__device__ unsigned g_sk_ctr[SK_CTRS];

template <int NC>
__device__ __forceinline__ void sk64_combine(const GemmP& p, const f32x4& o, bool mine, int64_t row0, int64_t Mc,
                                             int64_t n0, int64_t ncols, int g, f32x4* lds) {
  constexpr int Q = NC / 4;
  const int S = (int)gridDim.z, T = (int)(gridDim.x * gridDim.y), tile = (int)(blockIdx.y * gridDim.x + blockIdx.x);
  const int t = (int)threadIdx.x;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(p.ws, (short)0, 0x7fffffff, 0x00020000);
  if (mine && 4 * g < NC) {
    const int rl = (t >> 6) * 16 + (t & 15);
    const int off = (((int)blockIdx.z * T + tile) * 64 + rl) * NC + 4 * g;
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, o), rs, off * 4, 0, 16);  // aux 16: sc1
  }
  // the reducer's epilogue side inputs (residual, bias), loaded by every slice before the hand-off
  const bool red_ok = t < Mc * Q && n0 + 4 * (t % Q) < ncols;
  const int64_t m = row0 + t / Q, n = n0 + 4 * (t % Q);
  Side sd;
  u32x2 bias = {0u, 0u};
  if (red_ok) {
    epi_load4<EM_BF16>(p, 0, 0, m, n, sd);
    bias = epi_load_bias(p, n);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains before the arrival
  __syncthreads();
  unsigned* flag = reinterpret_cast<unsigned*>(lds);  // (the reduction array: every wave has read it)
  if (t == 0) {
    unsigned* ctr = g_sk_ctr + p.sk_tk + tile;
    const unsigned old = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const bool last = old == (unsigned)(S - 1);
    if (last) __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *flag = last ? 1u : 0u;
  }
  __syncthreads();
  if (*flag == 0u || !red_ok) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // (no instruction: keeps the loads below the hand-off)
  // reducer: one thread per (row, 4 columns) = 16 contiguous bytes of each slab; all S loads in flight (clamped
  // slice index, no branch around a load), summed from +0 in slice order
  u32x4 v[8];
#pragma unroll
  for (int z = 0; z < 8; ++z)
    v[z] = __builtin_amdgcn_raw_buffer_load_b128(rs, ((min(z, S - 1) * T + tile) * 64 * NC + 4 * t) * 4, 0, 16);
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int z = 0; z < 8; ++z)
    if (z < S) acc += __builtin_bit_cast(f32x4, v[z]);
  epi_store4<EM_BF16>(p, 0, 0, m, n, acc, sd, bias);
}

template <int W, int NC, int MB, bool F8W>
__global__ void __launch_bounds__(W * 64) gemm_skinny64_kernel(GemmP p) {
  static_assert(W >= MB, "one wave per row block in the epilogue");
  constexpr int U = MB >= 3 ? 2 : 4;  // 64-k chunks per load batch (register budget: A is MB x 8 VGPRs)
  __shared__ f32x4 red[W][MB][64];
  __shared__ float redn[W][MB][16];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, g = lane >> 4;
  const bool geglu = p.epi == PZ_EPI_GEGLU;
  const bool nrm = p.nw != nullptr;
  const int64_t ncols = geglu ? p.geglu_I : p.N;
  const int64_t n0 = (int64_t)blockIdx.x * NC;
  // fused RoPE + Q / K / V scatter (pz_gemm_qkv_rope few-row path, NC == 16, head_dim 256): block = 8 rotation
  // pairs of one head -- columns i..i+7 and their partners i+128..i+135 -- so the epilogue holds both halves
  const bool rope = p.rcs != nullptr;
  const int64_t nr = rope ? (int64_t)(blockIdx.x >> 4) * 256 + (blockIdx.x & 15) * 8 + (lane & 7) + ((lane & 8) << 4)
                          : n0 + (lane & 15) % NC;
  const bool nok = nr < ncols;
  // row chunks of 64 (blockIdx.y): M > 64 runs as independent 64-row problems sharing the weights in L2
  const int64_t row0 = (int64_t)blockIdx.y * 64;
  const int64_t Mc = min((int64_t)64, p.M - row0);
  constexpr int ES = F8W ? 1 : 2;  // weight element bytes
  const char* Bc = reinterpret_cast<const char*>(p.B);
  const char* Brow = Bc + (nr * p.ldb + 16 * g) * ES;
  const char* Brow2 = Bc + ((p.geglu_I + nr) * p.ldb + 16 * g) * ES;
  const bf16_t* Arow[MB];
  bool mok[MB];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) {
    const int64_t m = mb * 16 + (lane & 15);
    mok[mb] = m < Mc;
    Arow[mb] = p.A + (row0 + m) * p.lda + 16 * g;
  }
  const bf16_t* Wn = p.nw + 16 * g;
  f32x4 acc[MB], acc2[MB];
  float ss[MB];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) {
    acc[mb] = acc2[mb] = f32x4{0.f, 0.f, 0.f, 0.f};
    ss[mb] = 0.f;
  }
  // split-K over blockIdx.z (p.ksplit > 0: raw fp32 partials -> ws, summed by splitk_epilogue_kernel)
  const bool split = p.ksplit > 0;
  const int64_t kchunks_all = p.K / 64;
  const int64_t kz0 = split ? (int64_t)blockIdx.z * (p.ksplit / 64) : 0;
  const int64_t kchunks = split ? min(kchunks_all - kz0, p.ksplit / 64) : kchunks_all;
  const int64_t per = (kchunks + W - 1) / W;
  const int64_t kb = kz0 + wave * per, ke = kz0 + min(kchunks, (int64_t)(wave + 1) * per);
  auto load_b = [&](const char* row, int64_t c, bf16x8& lo, bf16x8& hi) {
    if (!nok) {
      lo = hi = bf16x8{};
    } else if (F8W) {
      fp8x16_to_bf16(*reinterpret_cast<const u32x4*>(row + c * 64), lo, hi);
    } else {
      lo = *reinterpret_cast<const bf16x8*>(row + c * 128);
      hi = *reinterpret_cast<const bf16x8*>(row + c * 128 + 16);
    }
  };
  int64_t kc = kb;
  auto run = [&](auto U_) {
    constexpr int UU = decltype(U_)::value;
    for (; kc + UU <= ke; kc += UU) {
      bf16x8 a[UU][MB][2], b[UU][2], b2[UU][2], wv[UU][2];
      u32x4 braw[UU], braw2[UU];
#pragma unroll
      for (int u = 0; u < UU; ++u) {
        if (F8W) {  // raw codes first (all loads in flight), expanded after the A loads are issued
          braw[u] = nok ? *reinterpret_cast<const u32x4*>(Brow + (kc + u) * 64) : u32x4{0u, 0u, 0u, 0u};
          if (geglu) braw2[u] = nok ? *reinterpret_cast<const u32x4*>(Brow2 + (kc + u) * 64) : u32x4{0u, 0u, 0u, 0u};
        } else {
          load_b(Brow, kc + u, b[u][0], b[u][1]);
          if (geglu) load_b(Brow2, kc + u, b2[u][0], b2[u][1]);
        }
#pragma unroll
        for (int mb = 0; mb < MB; ++mb)
#pragma unroll
          for (int h = 0; h < 2; ++h)
            a[u][mb][h] = mok[mb] ? *reinterpret_cast<const bf16x8*>(Arow[mb] + (kc + u) * 64 + 8 * h) : bf16x8{};
        if (nrm)
#pragma unroll
          for (int h = 0; h < 2; ++h) wv[u][h] = *reinterpret_cast<const bf16x8*>(Wn + (kc + u) * 64 + 8 * h);
      }
#pragma unroll
      for (int u = 0; u < UU; ++u) {
        if (F8W) {
          fp8x16_to_bf16(braw[u], b[u][0], b[u][1]);
          if (geglu) fp8x16_to_bf16(braw2[u], b2[u][0], b2[u][1]);
        }
#pragma unroll
        for (int h = 0; h < 2; ++h) {
#pragma unroll
          for (int mb = 0; mb < MB; ++mb) {
            if (nrm) {  // sum of squares of the raw row; the product takes x * (1 + w), rsqrt applied after
              const u32x4 xa = __builtin_bit_cast(u32x4, a[u][mb][h]), xw = __builtin_bit_cast(u32x4, wv[u][h]);
              u32x4 o;
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                const float x0 = __uint_as_float(xa[e] << 16), x1 = __uint_as_float(xa[e] & 0xffff0000u);
                const float w0 = __uint_as_float(xw[e] << 16), w1 = __uint_as_float(xw[e] & 0xffff0000u);
                ss[mb] += x0 * x0 + x1 * x1;
                o[e] = pack2bf(x0 * (1.f + w0), x1 * (1.f + w1));
              }
              a[u][mb][h] = __builtin_bit_cast(bf16x8, o);
            }
            acc[mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[u][h], a[u][mb][h], acc[mb], 0, 0, 0);
            if (geglu) acc2[mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b2[u][h], a[u][mb][h], acc2[mb], 0, 0, 0);
          }
        }
      }
    }
  };
  run(std::integral_constant<int, U>{});
  run(std::integral_constant<int, 1>{});
  // D[n_local = 4g + r][m = mb*16 + (lane & 15)]; wave w < MB finishes row block w
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) {
    red[wave][mb][lane] = acc[mb];
    if (nrm) {
      float t = ss[mb];
      t += __shfl_xor(t, 16, 64);
      t += __shfl_xor(t, 32, 64);
      if (lane < 16) redn[wave][mb][lane] = t;
    }
  }
  __syncthreads();
  const int mb = wave;
  f32x4 o = {0.f, 0.f, 0.f, 0.f}, o2 = {0.f, 0.f, 0.f, 0.f};
  if (mb < MB)
    for (int w = 0; w < W; ++w) o += red[w][mb][lane];
  if (geglu) {
    __syncthreads();
#pragma unroll
    for (int b = 0; b < MB; ++b) red[wave][b][lane] = acc2[b];
    __syncthreads();
    if (mb < MB)
      for (int w = 0; w < W; ++w) o2 += red[w][mb][lane];
  }
  if (split && p.sk_tk >= 0) {  // every wave joins the combine's barriers (host: no norm / GeGLU / RoPE with split)
    sk64_combine<NC>(p, o, mb < MB && mb * 16 + (lane & 15) < Mc, row0, Mc, n0, ncols, g, &red[0][0][0]);
    return;
  }
  if (mb >= MB) return;
  const int64_t ml = mb * 16 + (lane & 15);
  if (rope) {  // (host: no split, no GeGLU / bias / residual)
    float scale = p.alpha;
    if (nrm) {
      float t = 0.f;
      for (int w = 0; w < W; ++w) t += redn[w][mb][lane & 15];
      scale *= rsqrtf(t / (float)p.K + p.neps);
    }
    // the bf16 projection (what pz_qkv_rope_split reads), then the partner half of each rotation pair from lane
    // ^ 32 (lane group g ^ 2: local columns 4g.. are pairs 4(g & 1).. of the low half for g < 2, the high half
    // for g >= 2); both lanes of a pair hold the same row, so they are active together
    float x[4], y[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) x[r] = bf2f(f2bf(o[r] * scale));
#pragma unroll
    for (int r = 0; r < 4; ++r) y[r] = __shfl_xor(x[r], 32, 64);
    if (ml >= Mc) return;
    const int64_t mm = row0 + ml;
    const int64_t head = blockIdx.x >> 4, b = mm / p.rT, t = mm - b * p.rT;
    const int i = (blockIdx.x & 15) * 8 + 4 * (g & 1);  // pair index of x[0]
    const bool hi = g >= 2;
    float v[4];
    bf16_t* dst;
    if (head == p.rnh + 1) {  // value head: copied
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = x[r];
      dst = p.rv + (b * p.rLk + p.rkoff + t) * 256;
    } else {
      const float* cs = p.rcs + p.rpos[mm] * 256 + 2 * i;  // (cos, sin) of pairs i..i+3
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float o1, o2;
        if (hi) rope_pair(y[r], x[r], cs[2 * r], cs[2 * r + 1], o1, o2);
        else rope_pair(x[r], y[r], cs[2 * r], cs[2 * r + 1], o1, o2);
        v[r] = hi ? o2 : o1;
      }
      dst = head < p.rnh ? p.rq + (b * p.rLq + p.rqoff + t) * (p.rnh * 256) + head * 256
                         : p.rk + (b * p.rLk + p.rkoff + t) * 256;
    }
    *reinterpret_cast<u32x2*>(dst + i + (hi ? 128 : 0)) = u32x2{pack2bf(v[0], v[1]), pack2bf(v[2], v[3])};
    return;
  }
  if (ml >= Mc) return;
  const int64_t mm = row0 + ml;
  if (split) {  // two-launch form: partials for splitk_epilogue_kernel
    float* wz = p.ws + (int64_t)blockIdx.z * p.M * p.ldw + mm * p.ldw;
    for (int r = 0; r < 4; ++r) {
      const int64_t nn = n0 + 4 * g + r;
      if (4 * g + r < NC && nn < ncols) wz[nn] = o[r];
    }
    return;
  }
  float scale = p.alpha;
  if (nrm) {
    float t = 0.f;
    for (int w = 0; w < W; ++w) t += redn[w][mb][lane & 15];
    scale *= rsqrtf(t / (float)p.K + p.neps);
  }
  const int64_t n = n0 + 4 * g;
  for (int r = 0; r < 4; ++r) {
    const int64_t nn = n + r;
    if (4 * g + r >= NC || nn >= ncols) continue;
    float x = o[r] * scale;
    if (geglu) {
      const float gg = x, u = o2[r] * scale;
      if (p.aux) {
        p.aux[mm * p.ld_aux + nn] = f2bf(gg);
        p.aux[mm * p.ld_aux + p.geglu_I + nn] = f2bf(u);
      }
      x = gelu_tanh(gg) * u;
    } else {
      if (p.bias) x += bf2f(p.bias[nn]);
      if (p.epi == PZ_EPI_GELU || p.epi == PZ_EPI_SILU) {
        if (p.aux) p.aux[mm * p.ld_aux + nn] = f2bf(x);
        x = p.epi == PZ_EPI_GELU ? gelu_tanh(x) : silu(x);
      }
      if (p.resid) x += bf2f(p.resid[mm * p.ld_resid + nn]);
    }
    if (p.c_fp32) {
      float* Cp = reinterpret_cast<float*>(p.C) + mm * p.ldc + nn;
      *Cp = p.beta ? *Cp + x : x;
    } else {
      bf16_t* Cp = reinterpret_cast<bf16_t*>(p.C) + mm * p.ldc + nn;
      *Cp = f2bf(p.beta ? bf2f(*Cp) + x : x);
    }
  }
}

}  // namespace

template <int W, int TMB, int TNB, bool GEGLU, bool F8W = false>
static int launch_rows_k(const GemmP& p, hipStream_t st) {
  constexpr int smem = W * (GEGLU ? 2 : 1) * TMB * TNB * 1024;
  auto kern = gemm_rows_kernel<W, TMB, TNB, GEGLU, F8W>;
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, smem);
    attr_set = true;
  }
  hipLaunchKernelGGL(kern, dim3((unsigned)(p.tiles_m * p.tiles_n)), dim3(W * 64), smem, st, p);
  PZ_CHECK_LAUNCH();
  return PZ_OK;
}

template <int W>
static int launch_rows_w(const GemmP& p, int tnb, bool geglu, hipStream_t st) {
  if (geglu) return tnb == 2 ? launch_rows_k<W, 4, 2, true>(p, st) : launch_rows_k<W, 4, 1, true>(p, st);
  if (tnb == 4) return launch_rows_k<W, 4, 4, false>(p, st);
  if (tnb == 2) return launch_rows_k<W, 4, 2, false>(p, st);
  return launch_rows_k<W, 4, 1, false>(p, st);
}

template <int W>
static int launch_rows_f8(const GemmP& p, int tnb, bool geglu, hipStream_t st) {
  if (geglu) return tnb == 2 ? launch_rows_k<W, 4, 2, true, true>(p, st) : launch_rows_k<W, 4, 1, true, true>(p, st);
  if (tnb == 4) return launch_rows_k<W, 4, 4, false, true>(p, st);
  if (tnb == 2) return launch_rows_k<W, 4, 2, false, true>(p, st);
  return launch_rows_k<W, 4, 1, false, true>(p, st);
}

template <int W, int TNB>
static int launch_rows_f8a_k(const GemmP& p, hipStream_t st) {
  constexpr int smem = W * 4 * TNB * 1024;
  auto kern = gemm_rows_f8a_kernel<W, 4, TNB>;
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, smem);
    attr_set = true;
  }
  hipLaunchKernelGGL(kern, dim3((unsigned)(p.tiles_m * p.tiles_n)), dim3(W * 64), smem, st, p);
  PZ_CHECK_LAUNCH();
  return PZ_OK;
}

template <int W>
static int launch_rows_f8a(const GemmP& p, int tnb, hipStream_t st) {
  if (tnb == 4) return launch_rows_f8a_k<W, 4>(p, st);
  if (tnb == 2) return launch_rows_f8a_k<W, 2>(p, st);
  return launch_rows_f8a_k<W, 1>(p, st);
}

// f8w: 1 = W8A16 (bf16 rows, e4m3 weights), 2 = W8A8 (both e4m3, per-row activation scales)
int pz_rows_launch(const GemmP& p, int w, int tnb, bool geglu, int f8w, hipStream_t st) {
  if (f8w == 2) return w == 8 ? launch_rows_f8a<8>(p, tnb, st) : launch_rows_f8a<4>(p, tnb, st);
  if (f8w) return w == 8 ? launch_rows_f8<8>(p, tnb, geglu, st) : launch_rows_f8<4>(p, tnb, geglu, st);
  return w == 8 ? launch_rows_w<8>(p, tnb, geglu, st) : launch_rows_w<4>(p, tnb, geglu, st);
}

template <int W, int NC, int MB, bool F8W>
static int launch_sk64(const GemmP& p0, int64_t tiles_n, hipStream_t st) {
  GemmP p = p0;
  const int S = p.ksplit > 0 ? (int)((p.K / 64 + p.ksplit / 64 - 1) / (p.ksplit / 64)) : 1;
  const int64_t tiles = tiles_n * ((p.M + 63) / 64);
  // in-launch combine (PZ_SK64_FUSED=0: the two-launch form, A/B; read per call): each launch gets its own range
  // of arrival counters, dealt round-robin in 256-counter steps (256 launches in flight before a range is reused)
  const char* e = getenv("PZ_SK64_FUSED");
  const bool fits = p.sk_tk >= 0;  // (pz_gemm: the tile-private slabs fit the workspace, forward bf16 epilogue)
  p.sk_tk = -1;
  if (S > 1 && S <= 8 && tiles <= 256 && fits && !(e && e[0] == '0')) {
    static std::atomic<unsigned> next{0};
    p.sk_tk = (int)((next.fetch_add(1) % (SK_CTRS / 256)) * 256);
  }
  hipLaunchKernelGGL((gemm_skinny64_kernel<W, NC, MB, F8W>), dim3((unsigned)tiles_n, (unsigned)((p.M + 63) / 64), S),
                     dim3(W * 64), 0, st, p);
  PZ_CHECK_LAUNCH();
  if (S > 1 && p.sk_tk < 0) return pz_splitk_epi_launch(p, S, st);
  return PZ_OK;
}

template <int W, int MB, bool F8W>
static int launch_sk64_nc(const GemmP& p, int nc, int64_t tiles_n, hipStream_t st) {
  if (nc == 4) return launch_sk64<W, 4, MB, F8W>(p, tiles_n, st);
  if (nc == 8) return launch_sk64<W, 8, MB, F8W>(p, tiles_n, st);
  return launch_sk64<W, 16, MB, F8W>(p, tiles_n, st);
}

template <bool F8W>
static int launch_sk64_any(const GemmP& p, int w, int nc, int mb, int64_t tn, hipStream_t st) {
  if (w == 8) {
    if (mb == 1) return launch_sk64_nc<8, 1, F8W>(p, nc, tn, st);
    if (mb == 2) return launch_sk64_nc<8, 2, F8W>(p, nc, tn, st);
    return launch_sk64_nc<8, 4, F8W>(p, nc, tn, st);
  }
  if (mb == 1) return launch_sk64_nc<4, 1, F8W>(p, nc, tn, st);
  if (mb == 2) return launch_sk64_nc<4, 2, F8W>(p, nc, tn, st);
  return launch_sk64_nc<4, 4, F8W>(p, nc, tn, st);
}

int pz_sk64_launch(const GemmP& p, int w, int nc, int mb, bool f8w, int64_t tiles_n, hipStream_t st) {
  return f8w ? launch_sk64_any<true>(p, w, nc, mb, tiles_n, st) : launch_sk64_any<false>(p, w, nc, mb, tiles_n, st);
}
