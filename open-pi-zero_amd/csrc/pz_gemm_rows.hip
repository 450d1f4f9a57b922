// Row-slab GEMM kernel (own translation unit: pz_gemm.hip takes minutes to compile).
#include "pz_gemm_epi.h"

namespace {

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
template <int W, int TMB, int TNB, bool GEGLU>
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
  const bf16_t* Ar[TMB];
  const bf16_t* Br[NS][TNB];
#pragma unroll
  for (int mb = 0; mb < TMB; ++mb) Ar[mb] = p.A + min(m0 + 16 * mb + rl, p.M - 1) * p.lda + 8 * g;
#pragma unroll
  for (int nb = 0; nb < TNB; ++nb) {
    const int64_t col = min(n0 + 16 * nb + rl, ncols - 1);
    Br[0][nb] = p.B + col * p.ldb + 8 * g;
    if (GEGLU) Br[NS - 1][nb] = p.B + (p.geglu_I + col) * p.ldb + 8 * g;
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

}  // namespace

template <int W, int TNB, bool GEGLU>
static int launch_rows_k(const GemmP& p, hipStream_t st) {
  constexpr int smem = W * (GEGLU ? 2 : 1) * 4 * TNB * 1024;
  auto kern = gemm_rows_kernel<W, 4, TNB, GEGLU>;
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
  if (geglu) return tnb == 2 ? launch_rows_k<W, 2, true>(p, st) : launch_rows_k<W, 1, true>(p, st);
  if (tnb == 4) return launch_rows_k<W, 4, false>(p, st);
  if (tnb == 2) return launch_rows_k<W, 2, false>(p, st);
  return launch_rows_k<W, 1, false>(p, st);
}

int pz_rows_launch(const GemmP& p, int w, int tnb, bool geglu, hipStream_t st) {
  return w == 8 ? launch_rows_w<8>(p, tnb, geglu, st) : launch_rows_w<4>(p, tnb, geglu, st);
}
