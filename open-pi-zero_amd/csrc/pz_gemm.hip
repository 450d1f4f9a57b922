// bf16 MFMA GEMM for gfx950 with fused epilogues (the Pi0 hot-path workhorse).
//
//   C[z](m,n) = epilogue( alpha * sum_k A[z](m,k) * B[z](k,n) )
//
// Operands are bf16 and each may be "k-contiguous" (A stored [M][K], B stored
// [N][K]: nn.Linear weights) or "k-strided" (A stored [K][M], B stored [K][N]).
// That covers forward (NT), dgrad (NN) and wgrad (TN) of every nn.Linear in
// SigLIP / Gemma / the action expert, and the attention products
// S = Q K^T, O = P V, dP = dO V^T, dQ = dS K, dK = dS^T Q, dV = P^T dO
//  without any transpose kernels: k-strided tiles are staged in LDS
// [k][row] and read with ds_read_b64_tr_b16 (gfx950 hardware transpose read).
//
// Tile 128x128x64, 256 threads = 4 waves, mfma_f32_16x16x32_bf16, register
// staged double-buffered LDS (issue-early / write-late, one barrier per K
// step), XOR-swizzled LDS images (conflict-free ds_read_b128 and tr reads),
// XCD-aware tile order.  MFMA operands are swapped (B-frag first) so each lane
// owns 4 consecutive output columns -> vectorised epilogue stores.
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <type_traits>

#include "pz_gemm_epi.h"

namespace {

constexpr int BM = 128, BN = 128, BK = 64, NT = 256;
constexpr int TILE_BYTES = 128 * 64 * 2;  // one operand tile image in LDS


// two bf16-shaped fragments (8 x 16 bit each = 16 fp8 codes) -> one 32-code f8f6f4 operand
__device__ __forceinline__ i32x8 cat_f8(const bf16x8& lo, const bf16x8& hi) {
  const u32x4 a = __builtin_bit_cast(u32x4, lo), b = __builtin_bit_cast(u32x4, hi);
  return i32x8{(int)a[0], (int)a[1], (int)a[2], (int)a[3], (int)b[0], (int)b[1], (int)b[2], (int)b[3]};
}

__device__ __forceinline__ int sw_tr(int k) { return ((k & 3) | (((k >> 3) & 1) << 2)) << 2; }

// ---- global -> registers (4 x 16 B per thread per operand tile) -------------
template <bool KC>
__device__ __forceinline__ void g2r(u32x4 (&r)[4], const bf16_t* __restrict__ base, int64_t ld,
                                    int64_t row0, int64_t R, int64_t k0, int64_t K,
                                    bool geglu, int64_t gI) {
  const int t = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = t + NT * i;
    u32x4 v = {0u, 0u, 0u, 0u};
    if (KC) {
      const int rr = c >> 3, kc = c & 7;
      int64_t grow;
      bool ok;
      if (geglu) {
        const int64_t lr = row0 + (rr & 63);
        ok = lr < gI;
        grow = (rr < 64) ? lr : gI + lr;
      } else {
        grow = row0 + rr;
        ok = grow < R;
      }
      const int64_t kk = k0 + 8 * kc;
      if (ok && kk < K) v = *reinterpret_cast<const u32x4*>(base + grow * ld + kk);
    } else {
      const int kr = c >> 4, rc = c & 15;
      const int64_t kk = k0 + kr, rr = row0 + 8 * rc;
      if (kk < K && rr < R) v = *reinterpret_cast<const u32x4*>(base + kk * ld + rr);
    }
    r[i] = v;
  }
}

template <bool KC>
__device__ __forceinline__ void r2s(const u32x4 (&r)[4], char* lds) {
  const int t = threadIdx.x;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = t + NT * i;
    int off;
    if (KC) {
      const int rr = c >> 3, kc = c & 7;
      off = rr * 128 + ((kc ^ ((rr >> 1) & 7)) << 4);
    } else {
      const int kr = c >> 4, rc = c & 15;
      off = kr * 256 + (((2 * rc) ^ sw_tr(kr)) << 3);
    }
    *reinterpret_cast<u32x4*>(lds + off) = r[i];
  }
}

// fragment for rows rb*16.., k = kk*32 + 8*(lane>>4) + j
template <bool KC, int TRROW = 256>
__device__ __forceinline__ bf16x8 frag(const char* lds, int rb, int kk, int lane) {
  if (KC) {
    const int r = rb * 16 + (lane & 15);
    const int ch = kk * 4 + (lane >> 4);
    return *reinterpret_cast<const bf16x8*>(lds + r * 128 + ((ch ^ ((r >> 1) & 7)) << 4));
  } else {
    const int q = (lane & 15) >> 2, p = lane & 3;
    s16x8 out;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int k = kk * 32 + 8 * (lane >> 4) + 4 * t + q;
      const int off = k * TRROW + (((4 * rb + p) ^ sw_tr(k)) << 3);
      s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
          (__attribute__((address_space(3))) s16x4*)(lds + off));
      out[4 * t + 0] = v[0];
      out[4 * t + 1] = v[1];
      out[4 * t + 2] = v[2];
      out[4 * t + 3] = v[3];
    }
    return __builtin_bit_cast(bf16x8, out);
  }
}


// TAG only separates kernel symbols (profiling): 1 = the Gemma-2B MLP gate|up GeGLU GEMM (M >= 2048 rows)
template <bool AKC, bool BKC, int WM, int TAG>
__global__ void __launch_bounds__(NT, 2) gemm_kernel(GemmP p) {
  constexpr int WN = 4 / WM;
  constexpr int MI = (BM / WM) / 16;  // m blocks per wave
  constexpr int NI = (BN / WN) / 16;  // n blocks per wave
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* sA = smem;                    // [2][TILE_BYTES]
  char* sB = smem + 2 * TILE_BYTES;   // [2][TILE_BYTES]

  const bool geglu = p.epi == PZ_EPI_GEGLU;
  int tm, tn;
  int64_t z = blockIdx.y;
  if (p.batch_xcd) {
    // workgroups are dealt round-robin over the 8 XCDs: XCD x takes batch entries x, x + 8, ..., each
    // entry's tiles consecutive in its local order (all resident together, sharing the entry's panels)
    const int ntile = p.tiles_m * p.tiles_n, xcd = blockIdx.x & 7, local = blockIdx.x >> 3;
    const int bi = local / ntile, tile = local - bi * ntile;
    z = (int64_t)bi * 8 + xcd;
    tm = tile % p.tiles_m;
    tn = tile / p.tiles_m;
  } else {
    tile_coords(blockIdx.x, gridDim.x, p.tiles_m, p.tiles_n, tm, tn);
  }
  const bool split = p.ksplit > 0;
  const int64_t zo = split ? 0 : z / p.batch_inner, zi = split ? 0 : z % p.batch_inner;
  const bf16_t* A = p.A + zo * p.sAo + zi * p.sAi;
  const bf16_t* B = p.B + zo * p.sBo + zi * p.sBi;
  const int64_t m0 = (int64_t)tm * BM;
  const int64_t n0 = geglu ? (int64_t)tn * (BN / 2) : (int64_t)tn * BN;
  const int64_t kbeg = split ? z * p.ksplit : 0;
  const int64_t kend = split ? min(p.K, kbeg + p.ksplit) : p.K;

  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave / WN, wn = wave % WN;

  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (int)((kend - kbeg + BK - 1) / BK);
  u32x4 ra[4], rb[4];
  g2r<AKC>(ra, A, p.lda, m0, p.M, kbeg, kend, false, 0);
  g2r<BKC>(rb, B, p.ldb, n0, p.N, kbeg, kend, geglu, p.geglu_I);
  r2s<AKC>(ra, sA);
  r2s<BKC>(rb, sB);
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const bool more = kt + 1 < nk;
    if (more) {
      g2r<AKC>(ra, A, p.lda, m0, p.M, kbeg + (int64_t)(kt + 1) * BK, kend, false, 0);
      g2r<BKC>(rb, B, p.ldb, n0, p.N, kbeg + (int64_t)(kt + 1) * BK, kend, geglu, p.geglu_I);
    }
    const char* a_img = sA + cur * TILE_BYTES;
    const char* b_img = sB + cur * TILE_BYTES;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 af[MI], bfr[NI];
#pragma unroll
      for (int i = 0; i < MI; ++i) af[i] = frag<AKC>(a_img, wm * MI + i, kk, lane);
#pragma unroll
      for (int j = 0; j < NI; ++j) bfr[j] = frag<BKC>(b_img, wn * NI + j, kk, lane);
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
    }
    if (more) {
      r2s<AKC>(ra, sA + (cur ^ 1) * TILE_BYTES);
      r2s<BKC>(rb, sB + (cur ^ 1) * TILE_BYTES);
    }
    __syncthreads();
  }

  // ---------------------------------------------------------------- epilogue
  if (split) {
    // raw partial sums; GEGLU keeps the [gate | up] column layout of B (cols n, I + n)
    float* W = p.ws + z * p.M * p.ldw;
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int64_t m = m0 + wm * (BM / WM) + i * 16 + (lane & 15);
      if (m >= p.M) continue;
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        int64_t n;
        if (geglu) {
          const int64_t nl = n0 + (j % (NI / 2)) * 16 + 4 * (lane >> 4);
          if (nl >= p.geglu_I) continue;
          n = j < NI / 2 ? nl : p.geglu_I + nl;
        } else {
          n = n0 + wn * (BN / WN) + j * 16 + 4 * (lane >> 4);
          if (n >= p.N) continue;
        }
        *reinterpret_cast<f32x4*>(W + m * p.ldw + n) = acc[i][j];
      }
    }
    return;
  }
  const int64_t cofs = zo * p.sCo + zi * p.sCi;
  const int64_t rofs = zo * p.sRo + zi * p.sRi;
  if (geglu) {
    // wave tile = 32 rows x 128 cols: cols [0,64) gate, [64,128) up
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int64_t m = m0 + wm * (BM / WM) + i * 16 + (lane & 15);
#pragma unroll
      for (int j = 0; j < NI / 2; ++j)
        store_geglu4(p, cofs, m, n0 + j * 16 + 4 * (lane >> 4), acc[i][j], acc[i][j + NI / 2]);
    }
    return;
  }
  epi_dispatch(p, [&](auto em) {
    constexpr int EM = decltype(em)::value;
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int64_t m = m0 + wm * (BM / WM) + i * 16 + (lane & 15);
#pragma unroll
      for (int j = 0; j < NI; ++j)
        store_out4_m<EM>(p, cofs, rofs, m, n0 + wn * (BN / WN) + j * 16 + 4 * (lane >> 4), acc[i][j]);
    }
  });
}

// split-K second pass: C = epilogue(sum_z ws[z]) -- one thread per (row, 4 columns)
__global__ void __launch_bounds__(256) splitk_epilogue_kernel(GemmP p, int S) {
  const bool geglu = p.epi == PZ_EPI_GEGLU;
  const int64_t ncols = geglu ? p.geglu_I : p.N;
  const int64_t groups = (ncols + 3) / 4;
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= p.M * groups) return;
  const int64_t m = idx / groups, n = (idx - m * groups) * 4;
  const float* W = p.ws + m * p.ldw + n;
  const int64_t slab = p.M * p.ldw;
  // slabs loaded 4 at a time (all in flight together), summed in slab order (deterministic)
  auto sum_slabs = [&](const float* src) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int z = 0; z < S; z += 4) {
      f32x4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        v[u] = z + u < S ? *reinterpret_cast<const f32x4*>(src + (z + u) * slab) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int u = 0; u < 4; ++u) acc += v[u];
    }
    return acc;
  };
  if (geglu) {
    const f32x4 s = sum_slabs(W);
    const f32x4 u = sum_slabs(W + p.geglu_I);
    store_geglu4(p, 0, m, n, s, u);
    return;
  }
  // the epilogue's side inputs (residual, saved activation, bias) issued with the first slabs, not after their sum
  epi_dispatch(p, [&](auto em) {
    constexpr int EM = decltype(em)::value;
    Side sd;
    epi_load4<EM>(p, 0, 0, m, n, sd);
    const u32x2 bias = epi_load_bias(p, n);
    const f32x4 s = sum_slabs(W);
    epi_store4<EM>(p, 0, 0, m, n, s, sd, bias);
  });
}

// -------------------------------------------------------------------------
// 256x256 tile, 512 threads = 8 waves (4 along M x 2 along N, 64x128 per wave),
// operands streamed global -> LDS by LDS-DMA (global_load_lds_dwordx4, 1 KiB per
// wave-instruction, no VGPR staging).  Two pipelines are built from one body:
//   BK2 = 64, 2 stages (2 x 64 KiB): the next K-tile's DMA is issued before the
//     current tile's 64 MFMAs per wave; one vmcnt(0) + barrier per K step;
//   BK2 = 32, 4-slot ring (4 x 32 KiB): three K-tiles in flight, counted
//     vmcnt (never 0 in steady state) + raw s_barrier per K step.
// Measured on MI355X (tools/gemm_bench.py, random bf16): the 64/2-stage form
// is faster on every Pi0 shape (fewer barriers outweigh the deeper prefetch),
// so it is the one dispatched; the ring is kept for A/B experiments.
// LDS images are XOR-swizzled for conflict-free ds_read_b128 (k-contiguous
// operands) and ds_read_b64_tr_b16 (k-strided operands, [k][row] 512-B rows);
// the swizzle is applied to each lane's GLOBAL source address because an
// LDS-DMA write is lane-linear.  Requires K % BK2 == 0; M/N tails clamp the
// source rows (clamped rows are never stored).  GEGLU: B rows interleave
// gate/up in 64-row blocks so each wave's 128 virtual columns are 64 gate +
// the matching 64 up columns.
// -------------------------------------------------------------------------
constexpr int BT = 256, NT2 = 512;

__device__ __forceinline__ void glds16(const bf16_t* src, char* lds_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds_base, 16, 0, 0);
}

// k-contiguous image [256 rows][BKT k]: 16-B chunk ch of row r lives at chunk ch ^ swz(r)
template <int BKT>
__device__ __forceinline__ int swz_kc(int r) {
  return BKT == 64 ? ((r >> 1) & 7) : 3 * ((r >> 3) & 1);
}

// global source of lane `lane` for DMA instruction j of an operand tile (BKT*256*2/1024 instructions)
template <bool KC, int BKT>
__device__ __forceinline__ const bf16_t* dma_src(const bf16_t* base, int64_t ld, int j, int lane, int64_t row0,
                                                 int64_t R, bool geglu, int64_t gI) {
  if (KC) {
    constexpr int CPR = BKT / 8;          // 16-B chunks per row
    constexpr int RPI = 64 / CPR;         // rows per 1 KiB instruction
    const int r = RPI * j + lane / CPR;
    const int kc = (lane % CPR) ^ swz_kc<BKT>(r);
    int64_t grow;
    if (geglu) {
      const int blk = r >> 6;
      int64_t idx = row0 + (blk >> 1) * 64 + (r & 63);
      idx = idx < gI ? idx : gI - 1;
      grow = (blk & 1) ? gI + idx : idx;
    } else {
      grow = row0 + r;
      grow = grow < R ? grow : R - 1;
    }
    return base + grow * ld + 8 * kc;
  } else {
    const int k = 2 * j + (lane >> 5);
    const int c = (2 * (lane & 31)) ^ sw_tr(k);
    int64_t r = row0 + 4 * c;
    r = r <= R - 8 ? r : R - 8;
    return base + (int64_t)k * ld + r;
  }
}

template <bool KC, int BKT>
__device__ __forceinline__ bf16x8 frag256(const char* lds, int rb, int kk, int lane) {
  if (KC) {
    const int r = rb * 16 + (lane & 15);
    const int ch = kk * 4 + (lane >> 4);
    return *reinterpret_cast<const bf16x8*>(lds + r * (BKT * 2) + ((ch ^ swz_kc<BKT>(r)) << 4));
  } else {
    return frag<false, 512>(lds, rb, kk, lane);
  }
}

#define PZ_WAIT_VM(n) asm volatile("s_waitcnt vmcnt(" #n ")" ::: "memory")
#define PZ_BARRIER()                                   \
  do {                                                 \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); \
    __builtin_amdgcn_s_barrier();                      \
    asm volatile("" ::: "memory");                     \
  } while (0)

template <bool AKC, bool BKC, bool GEGLU, int BKT>
__global__ void __launch_bounds__(NT2, 1) gemm256_kernel(GemmP p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int MI = 4, NI = 8;
  constexpr int NSTAGE = BKT == 64 ? 2 : 4;
  constexpr int IMG = 256 * BKT * 2;
  constexpr int STAGE = 2 * IMG;
  constexpr int NI_DMA = IMG / 1024 / 8;  // DMA instructions per wave per operand per K-tile
  int tm, tn;
  tile_coords(blockIdx.x, gridDim.x, p.tiles_m, p.tiles_n, tm, tn);
  const int64_t m0 = (int64_t)tm * BT;
  const int64_t n0 = GEGLU ? (int64_t)tn * (BT / 2) : (int64_t)tn * BT;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int64_t z = blockIdx.y;
  const int64_t zo = z / p.batch_inner, zi = z % p.batch_inner;
  const bf16_t* Ab = p.A + zo * p.sAo + zi * p.sAi;
  const bf16_t* Bb = p.B + zo * p.sBo + zi * p.sBi;
  const int64_t cofs = zo * p.sCo + zi * p.sCi;
  const int64_t rofs = zo * p.sRo + zi * p.sRi;

  const bf16_t* sa[NI_DMA];
  const bf16_t* sb[NI_DMA];
#pragma unroll
  for (int i = 0; i < NI_DMA; ++i) {
    sa[i] = dma_src<AKC, BKT>(Ab, p.lda, wave * NI_DMA + i, lane, m0, p.M, false, 0);
    sb[i] = dma_src<BKC, BKT>(Bb, p.ldb, wave * NI_DMA + i, lane, n0, p.N, GEGLU, p.geglu_I);
  }
  const int64_t stepA = AKC ? BKT : BKT * p.lda;
  const int64_t stepB = BKC ? BKT : BKT * p.ldb;

  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (int)(p.K / BKT);
  auto issue = [&](int kt) {
    char* ia = smem + (kt % NSTAGE) * STAGE;
    char* ib = ia + IMG;
#pragma unroll
    for (int i = 0; i < NI_DMA; ++i) {
      glds16(sa[i] + kt * stepA, ia + (wave * NI_DMA + i) * 1024);
      glds16(sb[i] + kt * stepB, ib + (wave * NI_DMA + i) * 1024);
    }
  };
  auto compute = [&](int kt) {
    const char* a_img = smem + (kt % NSTAGE) * STAGE;
    const char* b_img = a_img + IMG;
#pragma unroll
    for (int kk = 0; kk < BKT / 32; ++kk) {
      bf16x8 bfr[NI];
#pragma unroll
      for (int j = 0; j < NI; ++j) bfr[j] = frag256<BKC, BKT>(b_img, wn * NI + j, kk, lane);
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const bf16x8 af = frag256<AKC, BKT>(a_img, wm * MI + i, kk, lane);
#pragma unroll
        for (int j = 0; j < NI; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af, acc[i][j], 0, 0, 0);
      }
    }
  };
  if constexpr (BKT == 64) {
    issue(0);
    PZ_WAIT_VM(0);
    PZ_BARRIER();
    for (int kt = 0; kt < nk; ++kt) {
      if (kt + 1 < nk) issue(kt + 1);
      compute(kt);
      PZ_WAIT_VM(0);
      PZ_BARRIER();
    }
  } else {
    issue(0);
    if (nk > 1) issue(1);
    if (nk > 2) issue(2);
    if (nk > 2) PZ_WAIT_VM(8);
    else if (nk > 1) PZ_WAIT_VM(4);
    else PZ_WAIT_VM(0);
    PZ_BARRIER();
    for (int kt = 0; kt < nk; ++kt) {
      if (kt + 3 < nk) issue(kt + 3);
      compute(kt);
      if (kt + 3 < nk) PZ_WAIT_VM(8);  // retire tile kt+1, keep kt+2, kt+3 in flight
      else if (kt + 2 < nk) PZ_WAIT_VM(4);
      else PZ_WAIT_VM(0);
      PZ_BARRIER();
    }
  }
  if (GEGLU) {
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int64_t m = m0 + wm * 64 + i * 16 + (lane & 15);
#pragma unroll
      for (int j = 0; j < NI / 2; ++j)
        store_geglu4(p, cofs, m, n0 + wn * 64 + j * 16 + 4 * (lane >> 4), acc[i][j], acc[i][j + NI / 2]);
    }
  } else {
    epi_dispatch(p, [&](auto em) {
      constexpr int EM = decltype(em)::value;
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int64_t m = m0 + wm * 64 + i * 16 + (lane & 15);
#pragma unroll
        for (int j = 0; j < NI; ++j)
          store_out4_m<EM>(p, cofs, rofs, m, n0 + wn * 128 + j * 16 + 4 * (lane >> 4), acc[i][j]);
      }
    });
  }
}

constexpr int BK256 = 64;  // dispatched K-tile of the 256 kernel (see above)

// -------------------------------------------------------------------------
// 256x256x64 "8-phase" ping-pong GEMM (the dispatched large-GEMM kernel).
//
// 8 waves as 2 (M) x 4 (N), 128 x 64 outputs per wave (acc[8][4], 128 AGPR/VGPR).
// With A k-contiguous (every forward GEMM and the large NN dgrads) each 64-deep K-tile
// is consumed in 2 sections of 32 MFMAs: section 0 reads A-lo + all of B and runs
// output quadrants (0,0) (0,1), section 1 reads A-hi and runs (1,1) (1,0).  Every
// section = [issue LDS-DMA pieces, ds_reads, counted vmcnt, lgkmcnt(0)] barrier
// [32 MFMA at setprio 1] barrier.  (A k-strided, PZ_GEMM_MAIN=quad only: the older
// 4 phases of 16 MFMAs, order (0,0) (0,1) (1,1) (1,0), reads A-lo + B-lo / B-hi /
// A-hi / nothing.)  The M-row-1 wave group runs one barrier behind the row-0 group,
// so on every SIMD (waves w and w+4) one wave's MFMAs overlap the other's LDS reads
// / DMA issue.
//
// LDS: two K-tile buffers of 64 KiB, each = 4 regions of 16 KiB:
//   A region 0 (rows with (r % 128) < 64), A region 1 (the other 128 rows),
//   B region 0 (virtual cols 0..127), B region 1 (cols 128..255).
// A region is free as soon as the section (phase) that last reads it has ended,
// so the next-but-one K-tile streams in piece by piece (two sections: A1(kt+1) in
// section 0, A0/B0/B1(kt+2) in section 1); 4 pieces (64 KiB) stay in flight and
// the counted waits (vmcnt 8) never drain the DMA queue in steady state.  Hazards
// (one barrier per section boundary, stagger included): a piece is waited for
// (vmcnt, issuing waves) in a section strictly before the one that reads it; a
// region is restaged >= 1 section after its last read, whose lgkmcnt(0) precedes
// that section's first barrier.
// -------------------------------------------------------------------------
constexpr int P8_BUF = 65536, P8_REG = 16384;

// global row of region-row rr (0..127) of an operand region; B may be the GeGLU [gate; up] stack
template <bool ISA, bool GEGLU>
__device__ __forceinline__ int64_t p8_row(int region, int rr, int64_t row0, int64_t R, int64_t gI) {
  if (ISA) {
    const int64_t g = row0 + (rr >> 6) * 128 + region * 64 + (rr & 63);
    return g < R ? g : R - 1;
  } else if (GEGLU) {
    const int v = region * 128 + rr;  // virtual column: wave (v >> 6), gate/up (v >> 5 & 1)
    int64_t g = row0 + (v >> 6) * 32 + (v & 31);
    g = g < gI ? g : gI - 1;
    return ((v >> 5) & 1) ? gI + g : g;
  } else {
    const int64_t g = row0 + region * 128 + rr;
    return g < R ? g : R - 1;
  }
}

// per-thread global source of DMA instruction i (0/1) of a region image
template <bool KC, bool ISA, bool GEGLU>
__device__ __forceinline__ const bf16_t* p8_src(const bf16_t* base, int64_t ld, int region, int i, int t,
                                                int64_t row0, int64_t R, int64_t gI) {
  if (KC) {  // image [128 rows][64 k], 128-B rows, chunk ch of row r at ch ^ ((r >> 1) & 7)
    const int r = i * 64 + (t >> 3);
    const int ch = (t & 7) ^ ((r >> 1) & 7);
    return base + p8_row<ISA, GEGLU>(region, r, row0, R, gI) * ld + 8 * ch;
  } else {  // whole-operand image [64 k][256 rows], 512-B rows; "region" r = k-rows 32r..32r+31;
            // 16-B chunk c of k-row k at c ^ (sw_tr(k) >> 1) (as the 2-stage kernel's image)
    const int k = region * 32 + i * 16 + (t >> 5);
    const int c = (t & 31) ^ (sw_tr(k) >> 1);
    int64_t g = row0 + 8 * c;  // first of 8 consecutive tile rows
    g = g <= R - 8 ? g : R - 8;
    return base + (int64_t)k * ld + g;
  }
}

// k-strided fragment through inline-asm ds_read_b64_tr_b16.  With the builtin, hipcc cannot
// tell the read from the in-flight LDS-DMA writes and drains the DMA queue (s_waitcnt vmcnt(0))
// before every transposed read, which serialises the 8-phase pipeline.  The asm result is NOT
// tracked by the compiler's lgkmcnt: callers wait lgkmcnt(0) (PZ_WAIT_LGKM0) before any use,
// and a sched_barrier keeps the consuming MFMAs behind that wait.
__device__ __forceinline__ s16x4 ds_tr_asm(const char* p) {
  s16x4 v;
  const unsigned a = (unsigned)(size_t)(const __attribute__((address_space(3))) char*)p;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"(a));
  return v;
}

template <int TRROW>
__device__ __forceinline__ bf16x8 frag_tr_asm(const char* lds, int rb, int kk, int lane) {
  const int q = (lane & 15) >> 2, p = lane & 3;
  s16x8 out;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int k = kk * 32 + 8 * (lane >> 4) + 4 * t + q;
    const s16x4 v = ds_tr_asm(lds + k * TRROW + (((4 * rb + p) ^ sw_tr(k)) << 3));
    out[4 * t + 0] = v[0];
    out[4 * t + 1] = v[1];
    out[4 * t + 2] = v[2];
    out[4 * t + 3] = v[3];
  }
  return __builtin_bit_cast(bf16x8, out);
}

#define PZ_SCHED() __builtin_amdgcn_sched_barrier(0)
#define PZ_RAW_BARRIER()           \
  do {                             \
    PZ_SCHED();                    \
    __builtin_amdgcn_s_barrier();  \
    PZ_SCHED();                    \
  } while (0)
#define PZ_WAIT_LGKM0() asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory")

// 8-phase epilogue: wave (wr, wc) owns rows wr*128 + 16*rb + (lane & 15) and columns
// wc*64 + 16*cb + 4*(lane >> 4) .. +3 (GeGLU: gate cb = 0,1 with up cb + 2 of the same column)
// ---- 8-phase epilogue -------------------------------------------------------
// Wave (wr, wc) owns rows wr*128 + 16*rb + (lane & 15) and columns wc*64 + 16*cb + 4*(lane >> 4) .. +3
// (GeGLU: gate cb = 0,1 with up cb + 2 of the same column).  Interior tiles (the vast majority)
// take a lean path per epilogue class: no bounds checks, row pointers stepped by 16 rows, and the
// side inputs (residual / old C / saved activations) of row block rb + 1 loaded before the stores
// of row block rb, so their latency overlaps the stores (vmcnt retires the older loads first).
// Edge tiles use the general per-group store_out4_rt.
enum FastMode { FM_STORE = 0, FM_BF16 = 1, FM_F32 = 2, FM_DACT = 3, FM_DGEGLU = 4 };

__host__ __device__ __forceinline__ int fast_mode(const GemmP& p) {
  if (p.epi == PZ_EPI_DGEGLU) return FM_DGEGLU;
  if (p.epi == PZ_EPI_DGELU || p.epi == PZ_EPI_DSILU) return FM_DACT;
  if (p.c_fp32) return FM_F32;
  if (!p.resid && !p.beta && p.epi == PZ_EPI_NONE) return FM_STORE;
  return FM_BF16;
}

__device__ __forceinline__ u32x2 pk4(const float (&v)[4]) {
  return u32x2{pack2bf(v[0], v[1]), pack2bf(v[2], v[3])};
}

template <int FM>
__device__ __forceinline__ void epi8p_fast(const GemmP& p, int64_t cofs, int64_t rofs, int64_t m, int64_t nb,
                                           const f32x4 (&acc)[8][4]) {
  const float alpha = p.alpha;
  const int64_t crow = 16 * p.ldc;
  float bias[4][4];
#pragma unroll
  for (int cb = 0; cb < 4; ++cb) {
    if (FM <= FM_F32 && p.bias) {
      unpack4(*reinterpret_cast<const u32x2*>(p.bias + nb + cb * 16), bias[cb]);
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r) bias[cb][r] = 0.f;
    }
  }
  if constexpr (FM == FM_STORE) {
    bf16_t* C = reinterpret_cast<bf16_t*>(p.C) + cofs + m * p.ldc + nb;
#pragma unroll
    for (int rb = 0; rb < 8; ++rb) {
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) {
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = acc[rb][cb][r] * alpha + bias[cb][r];
        *reinterpret_cast<u32x2*>(C + rb * crow + cb * 16) = pk4(v);
      }
    }
  } else if constexpr (FM == FM_F32) {
    float* C = reinterpret_cast<float*>(p.C) + cofs + m * p.ldc + nb;
    const bf16_t* R = p.resid ? p.resid + rofs + m * p.ld_resid + nb : nullptr;
    const int64_t rrow = 16 * p.ld_resid;
    const bool ld = p.beta || R;
    f32x4 side[2][4];
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
      side[0][cb] = f32x4{0.f, 0.f, 0.f, 0.f};
      side[1][cb] = f32x4{0.f, 0.f, 0.f, 0.f};
    }
    auto load = [&](int rb, f32x4 (&d)[4]) {
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) {
        if (p.beta) {
          d[cb] = *reinterpret_cast<const f32x4*>(C + rb * crow + cb * 16);
        } else {
          float x[4];
          unpack4(*reinterpret_cast<const u32x2*>(R + rb * rrow + cb * 16), x);
          d[cb] = f32x4{x[0], x[1], x[2], x[3]};
        }
      }
    };
    if (ld) load(0, side[0]);
#pragma unroll
    for (int rb = 0; rb < 8; ++rb) {
      if (ld && rb + 1 < 8) load(rb + 1, side[(rb + 1) & 1]);
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) {
        f32x4 v;
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = acc[rb][cb][r] * alpha + bias[cb][r] + side[rb & 1][cb][r];
        *reinterpret_cast<f32x4*>(C + rb * crow + cb * 16) = v;
      }
    }
  } else {
    // bf16 output with side inputs: FM_BF16 (resid and/or old C, optional GELU/SILU with saved
    // pre-activation), FM_DACT (aux = pre-activation), FM_DGEGLU (aux = [g | u], two outputs)
    bf16_t* C = reinterpret_cast<bf16_t*>(p.C) + cofs + m * p.ldc + nb;
    const bool aux_in = FM == FM_DACT || FM == FM_DGEGLU;
    const bf16_t* X0 = aux_in ? p.aux + m * p.ld_aux + nb : (p.beta ? C : nullptr);
    const int64_t x0row = aux_in ? 16 * p.ld_aux : crow;
    const bf16_t* X1 = FM == FM_DGEGLU ? X0 + p.geglu_I : (FM == FM_BF16 && p.resid ? p.resid + rofs + m * p.ld_resid + nb : nullptr);
    const int64_t x1row = FM == FM_DGEGLU ? x0row : 16 * p.ld_resid;
    u32x2 s0[2][4], s1[2][4];
    auto load = [&](int rb, u32x2 (&d0)[4], u32x2 (&d1)[4]) {
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) {
        d0[cb] = X0 ? *reinterpret_cast<const u32x2*>(X0 + rb * x0row + cb * 16) : u32x2{0u, 0u};
        d1[cb] = X1 ? *reinterpret_cast<const u32x2*>(X1 + rb * x1row + cb * 16) : u32x2{0u, 0u};
      }
    };
    load(0, s0[0], s1[0]);
    const bool act = FM == FM_BF16 && (p.epi == PZ_EPI_GELU || p.epi == PZ_EPI_SILU);
    const bool gelu = p.epi == PZ_EPI_GELU || p.epi == PZ_EPI_DGELU;
    bf16_t* Aux = act && p.aux ? p.aux + m * p.ld_aux + nb : nullptr;
    const int64_t arow = 16 * p.ld_aux;
#pragma unroll
    for (int rb = 0; rb < 8; ++rb) {
      if (rb + 1 < 8) load(rb + 1, s0[(rb + 1) & 1], s1[(rb + 1) & 1]);
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) {
        float v[4], x0[4], x1[4];
        unpack4(s0[rb & 1][cb], x0);
        unpack4(s1[rb & 1][cb], x1);
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = acc[rb][cb][r] * alpha;
        bf16_t* Cp = C + rb * crow + cb * 16;
        if constexpr (FM == FM_DGEGLU) {
          float dg[4], du[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float gl_, gr_;
            gelu_tanh_both(x0[r], gl_, gr_);
            dg[r] = v[r] * x1[r] * gr_;
            du[r] = v[r] * gl_;
          }
          *reinterpret_cast<u32x2*>(Cp) = pk4(dg);
          *reinterpret_cast<u32x2*>(Cp + p.geglu_I) = pk4(du);
        } else if constexpr (FM == FM_DACT) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] *= gelu ? gelu_tanh_grad(x0[r]) : silu_grad(x0[r]);
          *reinterpret_cast<u32x2*>(Cp) = pk4(v);
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] += bias[cb][r];
          if (act) {
            if (Aux) *reinterpret_cast<u32x2*>(Aux + rb * arow + cb * 16) = pk4(v);
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = gelu ? gelu_tanh(v[r]) : silu(v[r]);
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] += x1[r] + x0[r];  // resid, old C (zeros when absent)
          *reinterpret_cast<u32x2*>(Cp) = pk4(v);
        }
      }
    }
  }
}

// ---- LDS-staged output images (interior tiles) ------------------------------------------------
// A swapped-operand MFMA accumulator gives each lane 4 consecutive columns of one row, so direct
// stores are 8 B per lane spread over 16 rows (32-B pieces of many cache lines per instruction).
// Plain and GeGLU interior tiles instead write bf16 256 x 128 images into the idle LDS (16-B chunk
// index XOR-swizzled by row: conflict-free 8-B writes and 16-B reads) and copy them out row-
// contiguously, 16 B per lane (each wave instruction = 4 full 256-B row segments).
__device__ __forceinline__ void img_put(char* img, int row, int col, u32x2 v) {
  const int ch = col >> 3;
  *reinterpret_cast<u32x2*>(img + row * 256 + ((ch ^ (row & 15)) << 4) + ((col >> 2) & 1) * 8) = v;
}
// 16-B output store; nt: non-temporal (streaming) cache policy (PZ_GEMM_NT=1, A/B)
__device__ __forceinline__ void st16(bf16_t* dst, const u32x4& v, bool nt) {
  if (nt) __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(dst));
  else *reinterpret_cast<u32x4*>(dst) = v;
}
__device__ __forceinline__ void img_flush(const char* img, bf16_t* dst, int64_t ld, bool nt = false) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int c = threadIdx.x + i * NT2, row = c >> 4, ch = c & 15;
    const u32x4 v = *reinterpret_cast<const u32x4*>(img + row * 256 + ((ch ^ (row & 15)) << 4));
    st16(dst + row * ld + ch * 8, v, nt);
  }
}
__device__ __forceinline__ void lds_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// staged epilogue with side inputs (interior tiles): alpha*acc (+bias) -> two bf16 256 x 128 LDS images,
// then each thread finishes 16-B row chunks: residual / old C / saved activations are read as 16-B
// row-contiguous loads (a batch of 8 chunks in flight), outputs written as 16-B stores.
//   FM_BF16: [aux = pre; act(pre)] (+ resid) (+ old C);  FM_DACT: * act'(aux);  FM_DGEGLU: d(gate|up)
__device__ __forceinline__ void unpack8(const u32x4& w, float (&o)[8]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    o[2 * i] = __uint_as_float(w[i] << 16);
    o[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}
__device__ __forceinline__ u32x4 pack8v(const float (&v)[8]) {
  return u32x4{pack2bf(v[0], v[1]), pack2bf(v[2], v[3]), pack2bf(v[4], v[5]), pack2bf(v[6], v[7])};
}

template <int FM>
__device__ __forceinline__ void epi8p_staged(const GemmP& p, int64_t cofs, int64_t rofs, int64_t m0, int64_t n0,
                                             int wr, int wc, int lane, const f32x4 (&acc)[8][4], char* smem) {
  const int g4 = 4 * (lane >> 4), rl = lane & 15;
  const int64_t nb = n0 + wc * 64 + g4;
  char* img = smem + (wc >> 1) * 65536;
#pragma unroll
  for (int cb = 0; cb < 4; ++cb) {
    float bias[4] = {0.f, 0.f, 0.f, 0.f};
    if (FM == FM_BF16 && p.bias) unpack4(*reinterpret_cast<const u32x2*>(p.bias + nb + cb * 16), bias);
#pragma unroll
    for (int rb = 0; rb < 8; ++rb) {
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = acc[rb][cb][r] * p.alpha + bias[r];
      img_put(img, wr * 128 + rb * 16 + rl, (wc & 1) * 64 + cb * 16 + g4, u32x2{pack2bf(v[0], v[1]), pack2bf(v[2], v[3])});
    }
  }
  lds_sync();
  bf16_t* C = reinterpret_cast<bf16_t*>(p.C) + cofs + m0 * p.ldc + n0;
  const bf16_t* X0 = nullptr;  // side input 0: aux (DACT: pre-activation, DGEGLU: g) or old C
  const bf16_t* X1 = nullptr;  // side input 1: resid or DGEGLU u
  int64_t ld0 = 0, ld1 = 0;
  if (FM == FM_DACT || FM == FM_DGEGLU) {
    X0 = p.aux + m0 * p.ld_aux + n0;
    ld0 = p.ld_aux;
    if (FM == FM_DGEGLU) {
      X1 = X0 + p.geglu_I;
      ld1 = p.ld_aux;
    }
  } else {
    if (p.beta) {
      X0 = C;
      ld0 = p.ldc;
    }
    if (p.resid) {
      X1 = p.resid + rofs + m0 * p.ld_resid + n0;
      ld1 = p.ld_resid;
    }
  }
  const bool act = FM == FM_BF16 && (p.epi == PZ_EPI_GELU || p.epi == PZ_EPI_SILU);
  const bool gelu = p.epi == PZ_EPI_GELU || p.epi == PZ_EPI_DGELU;
  // side inputs in 4 batches of 4 chunks (8 x 16 B per thread in flight); batches of 8 chunks (128 KiB per CU in
  // flight) make hipcc spill 136-172 B in every non-GeGLU 8-phase kernel, so they were not measured
  constexpr int CPB = 4;
#pragma unroll
  for (int half = 0; half < 16 / CPB; ++half) {  // a batch's loads issued together
    u32x4 a0[CPB], a1[CPB], iv[CPB];
#pragma unroll
    for (int i = 0; i < CPB; ++i) {
      const int c = threadIdx.x + (half * CPB + i) * NT2;  // 0 .. 8191 over the two images
      const int im = c >> 12, row = (c >> 4) & 255, ch = c & 15;
      const int col = im * 128 + ch * 8;
      iv[i] = *reinterpret_cast<const u32x4*>(smem + im * 65536 + row * 256 + ((ch ^ (row & 15)) << 4));
      a0[i] = X0 ? *reinterpret_cast<const u32x4*>(X0 + row * ld0 + col) : u32x4{0u, 0u, 0u, 0u};
      a1[i] = X1 ? *reinterpret_cast<const u32x4*>(X1 + row * ld1 + col) : u32x4{0u, 0u, 0u, 0u};
    }
#pragma unroll
    for (int i = 0; i < CPB; ++i) {
      const int c = threadIdx.x + (half * CPB + i) * NT2;
      const int im = c >> 12, row = (c >> 4) & 255, ch = c & 15;
      const int col = im * 128 + ch * 8;
      float v[8], x0[8], x1[8];
      unpack8(iv[i], v);
      unpack8(a0[i], x0);
      unpack8(a1[i], x1);
      bf16_t* Cp = C + row * p.ldc + col;
      if (FM == FM_DGEGLU) {
        float dg[8], du[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          float gl_, gr_;
          gelu_tanh_both(x0[e], gl_, gr_);
          dg[e] = v[e] * x1[e] * gr_;
          du[e] = v[e] * gl_;
        }
        st16(Cp, pack8v(dg), p.nt_store);
        st16(Cp + p.geglu_I, pack8v(du), p.nt_store);
      } else if (FM == FM_DACT) {
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] *= gelu ? gelu_tanh_grad(x0[e]) : silu_grad(x0[e]);
        st16(Cp, pack8v(v), p.nt_store);
      } else {
        if (act) {
          if (p.aux) st16(p.aux + (m0 + row) * p.ld_aux + n0 + col, iv[i], p.nt_aux);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = gelu ? gelu_tanh(v[e]) : silu(v[e]);
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += x1[e] + x0[e];  // resid, old C (zeros when absent)
        st16(Cp, pack8v(v), p.nt_store);
      }
    }
  }
}

// fused RoPE + Q / K / V scatter (pz_gemm_qkv_rope): the tile (256 rows x one head of 256 columns) is
// rounded to bf16 into two LDS images (columns 0..127 | 128..255 = the two halves of every rotation pair,
// utils.py:4-16 rotate_half), then each thread rotates 16-B chunk pairs (i..i+7 with i+128..i+135) and
// writes them to the joint buffers -- the arithmetic of qkv_rope_split_kernel on the same bf16 inputs.
__device__ __forceinline__ void epi8p_rope(const GemmP& p, int64_t m0, int64_t n0, int wr, int wc, int lane,
                                           const f32x4 (&acc)[8][4], char* smem) {
  const int g4 = 4 * (lane >> 4), rl = lane & 15;
  char* img = smem + (wc >> 1) * 65536;
#pragma unroll
  for (int rb = 0; rb < 8; ++rb)
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = acc[rb][cb][r] * p.alpha;
      img_put(img, wr * 128 + rb * 16 + rl, (wc & 1) * 64 + cb * 16 + g4, u32x2{pack2bf(v[0], v[1]), pack2bf(v[2], v[3])});
    }
  lds_sync();
  const int64_t h = n0 >> 8;  // head: 0..nh-1 query, nh key, nh+1 value
#pragma unroll 2
  for (int it = 0; it < 8; ++it) {
    const int c = threadIdx.x + it * NT2, row = c >> 4, ch = c & 15;
    const int64_t m = m0 + row;
    if (m >= p.M) continue;
    const int off = (ch ^ (row & 15)) << 4;
    const u32x4 w1 = *reinterpret_cast<const u32x4*>(smem + row * 256 + off);
    const u32x4 w2 = *reinterpret_cast<const u32x4*>(smem + 65536 + row * 256 + off);
    const int64_t b = m / p.rT, t = m - b * p.rT;
    if (h == p.rnh + 1) {  // value head: copied
      bf16_t* dv = p.rv + (b * p.rLk + p.rkoff + t) * 256 + ch * 8;
      *reinterpret_cast<u32x4*>(dv) = w1;
      *reinterpret_cast<u32x4*>(dv + 128) = w2;
      continue;
    }
    float x1[8], x2[8], o1[8], o2[8];
    unpack8(w1, x1);
    unpack8(w2, x2);
    const float4* cs = reinterpret_cast<const float4*>(p.rcs + p.rpos[m] * 256 + 16 * ch);  // (cos, sin) x 8
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4 c2 = cs[q];
      const float co0 = c2.x, si0 = c2.y, co1 = c2.z, si1 = c2.w;
      rope_pair(x1[2 * q], x2[2 * q], co0, si0, o1[2 * q], o2[2 * q]);
      rope_pair(x1[2 * q + 1], x2[2 * q + 1], co1, si1, o1[2 * q + 1], o2[2 * q + 1]);
    }
    bf16_t* d = h < p.rnh ? p.rq + (b * p.rLq + p.rqoff + t) * (p.rnh * 256) + h * 256 + ch * 8
                          : p.rk + (b * p.rLk + p.rkoff + t) * 256 + ch * 8;
    *reinterpret_cast<u32x4*>(d) = pack8v(o1);
    *reinterpret_cast<u32x4*>(d + 128) = pack8v(o2);
  }
}

template <bool GEGLU>
__device__ __forceinline__ void epilogue8p(const GemmP& p, int64_t cofs, int64_t rofs, int64_t m0, int64_t n0,
                                           int wr, int wc, int lane, const f32x4 (&acc)[8][4], char* smem) {
  if (!GEGLU && p.rcs) {
    epi8p_rope(p, m0, n0, wr, wc, lane, acc, smem);
    return;
  }
  const int g4 = 4 * (lane >> 4), rl = lane & 15;
  if (GEGLU) {
    if (m0 + BT <= p.M && n0 + BT / 2 <= p.geglu_I && p.aux) {
      // h and g staged through the two 64 KiB LDS images (16-B row stores), u stored straight from the
      // accumulators (8 B per lane) in the same pass: one image round instead of two (u needs no LDS round
      // trip of its own; 4.03 vs 4.08-4.24 ms at 35328 x 32768 x 2048, bitwise equal,
      // profiles/r04/geglu_epi_ab.log; all three through direct 8-B stores measured 4.64 ms)
#pragma unroll
      for (int rb = 0; rb < 8; ++rb) {
        const int64_t m = m0 + wr * 128 + rb * 16 + rl;
        bf16_t* Ur = p.aux + m * p.ld_aux + p.geglu_I + n0 + wc * 32 + g4;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          float gg[4], hh[4], uu[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            gg[r] = acc[rb][j][r] * p.alpha;
            uu[r] = acc[rb][2 + j][r] * p.alpha;
            hh[r] = gelu_tanh(gg[r]) * uu[r];
          }
          const int row = wr * 128 + rb * 16 + rl, col = wc * 32 + j * 16 + g4;
          img_put(smem, row, col, u32x2{pack2bf(hh[0], hh[1]), pack2bf(hh[2], hh[3])});
          img_put(smem + 65536, row, col, u32x2{pack2bf(gg[0], gg[1]), pack2bf(gg[2], gg[3])});
          if (p.nt_aux) __builtin_nontemporal_store(pk4(uu), reinterpret_cast<u32x2*>(Ur + j * 16));
          else *reinterpret_cast<u32x2*>(Ur + j * 16) = pk4(uu);
        }
      }
      lds_sync();
      img_flush(smem, reinterpret_cast<bf16_t*>(p.C) + cofs + m0 * p.ldc + n0, p.ldc, p.nt_store);
      img_flush(smem + 65536, p.aux + m0 * p.ld_aux + n0, p.ld_aux, p.nt_aux);
      return;
    }
#pragma unroll
    for (int rb = 0; rb < 8; ++rb) {
      const int64_t m = m0 + wr * 128 + rb * 16 + rl;
#pragma unroll
      for (int j = 0; j < 2; ++j) store_geglu4(p, cofs, m, n0 + wc * 32 + j * 16 + g4, acc[rb][j], acc[rb][2 + j]);
    }
    return;
  }
  const int64_t m = m0 + wr * 128 + (lane & 15), nb = n0 + wc * 64 + 4 * (lane >> 4);
  if (m0 + BT <= p.M && n0 + BT <= p.N) {
    switch (fast_mode(p)) {
      case FM_STORE: {  // two 256 x 128 images (columns 0..127 | 128..255), one pass
        float bias[4][4];
#pragma unroll
        for (int cb = 0; cb < 4; ++cb) {
          if (p.bias) {
            unpack4(*reinterpret_cast<const u32x2*>(p.bias + nb + cb * 16), bias[cb]);
          } else {
#pragma unroll
            for (int r = 0; r < 4; ++r) bias[cb][r] = 0.f;
          }
        }
        char* img = smem + (wc >> 1) * 65536;
#pragma unroll
        for (int rb = 0; rb < 8; ++rb)
#pragma unroll
          for (int cb = 0; cb < 4; ++cb) {
            float v[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = acc[rb][cb][r] * p.alpha + bias[cb][r];
            img_put(img, wr * 128 + rb * 16 + rl, (wc & 1) * 64 + cb * 16 + g4, u32x2{pack2bf(v[0], v[1]), pack2bf(v[2], v[3])});
          }
        lds_sync();
        bf16_t* C = reinterpret_cast<bf16_t*>(p.C) + cofs + m0 * p.ldc + n0;
        img_flush(smem, C, p.ldc, p.nt_store);
        img_flush(smem + 65536, C + 128, p.ldc, p.nt_store);
        break;
      }
      case FM_F32: epi8p_fast<FM_F32>(p, cofs, rofs, m, nb, acc); break;
      case FM_DACT: epi8p_staged<FM_DACT>(p, cofs, rofs, m0, n0, wr, wc, lane, acc, smem); break;
      case FM_DGEGLU: epi8p_staged<FM_DGEGLU>(p, cofs, rofs, m0, n0, wr, wc, lane, acc, smem); break;
      default: epi8p_staged<FM_BF16>(p, cofs, rofs, m0, n0, wr, wc, lane, acc, smem); break;
    }
    return;
  }
  // edge tile: park each half of the wave's accumulators in its own 16 KiB of the (now idle) LDS
  // and run ONE runtime-general group store in a rolled loop (lane-private slots: no barrier)
  f32x4* park = reinterpret_cast<f32x4*>(smem) + (wr * 4 + wc) * 1024 + lane;
#pragma unroll
  for (int half = 0; half < 2; ++half) {
#pragma unroll
    for (int g = 0; g < 16; ++g) park[g * 64] = acc[half * 4 + (g >> 2)][g & 3];
#pragma unroll 1
    for (int g = 0; g < 16; ++g)
      store_out4_rt(p, cofs, rofs, m + (half * 4 + (g >> 2)) * 16, nb + (g & 3) * 16, park[g * 64]);
  }
}

// F8: fp8 (OCP e4m3) A and B, both k-contiguous, staged by the same byte-identical pipeline: the
// caller passes K, lda, ldb in units of 2 codes ("bf16-sized" elements), so a 64-unit K-tile is 128
// codes, and each (row block, column block) of a K-tile is ONE v_mfma_f32_16x16x128_f8f6f4 on the two
// bf16-shaped fragments of that tile concatenated (lane group g: codes 16g..16g+15 and 64+16g..
// 64+16g+15 of the tile on BOTH operands -- the same k set, so the sum is the plain dot product) at
// twice the bf16 MFMA rate.  The per-row activation scale (p.rs) multiplies the accumulators after
// the main loop (before the split-tail partials are written, so the tail sum stays linear); the
// weight scale is alpha.
template <bool AKC, bool BKC, bool GEGLU, bool KTAIL, bool F8>
__device__ __forceinline__ void gemm8p_body(const GemmP& p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int nk_all = (int)((p.K + 63) / 64);
  int lid = blockIdx.x, piece = -1, kt0 = 0, nk = nk_all;
  if (p.tail_s && lid >= p.dp_tiles) {  // split tail: one K-piece of a leftover tile
    const int u = lid - p.dp_tiles;
    piece = u;
    lid = p.dp_tiles + u / p.tail_s;
    kt0 = (u % p.tail_s) * p.tail_kt;
    nk = min(nk_all - kt0, p.tail_kt);
  }
  int tm, tn;
  tile_coords(lid, p.tiles_m * p.tiles_n, p.tiles_m, p.tiles_n, tm, tn, p.group);
  const int64_t m0 = (int64_t)tm * BT;
  const int64_t n0 = GEGLU ? (int64_t)tn * (BT / 2) : (int64_t)tn * BT;
  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int64_t z = blockIdx.y;
  const int64_t zo = z / p.batch_inner, zi = z % p.batch_inner;
  const bf16_t* Ab = p.A + zo * p.sAo + zi * p.sAi;
  const bf16_t* Bb = p.B + zo * p.sBo + zi * p.sBi;

  // pieces: 0 = A region 0, 1 = B region 0, 2 = B region 1, 3 = A region 1
  const bf16_t* src[4][2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    src[0][i] = p8_src<AKC, true, false>(Ab, p.lda, 0, i, t, m0, p.M, 0);
    src[3][i] = p8_src<AKC, true, false>(Ab, p.lda, 1, i, t, m0, p.M, 0);
    src[1][i] = p8_src<BKC, false, GEGLU>(Bb, p.ldb, 0, i, t, n0, p.N, p.geglu_I);
    src[2][i] = p8_src<BKC, false, GEGLU>(Bb, p.ldb, 1, i, t, n0, p.N, p.geglu_I);
  }
  const int64_t stepA = AKC ? 64 : 64 * p.lda;
  const int64_t stepB = BKC ? 64 : 64 * p.ldb;
  if (kt0) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      src[0][i] += kt0 * stepA;
      src[3][i] += kt0 * stepA;
      src[1][i] += kt0 * stepB;
      src[2][i] += kt0 * stepB;
    }
  }
  constexpr int lds_off[4] = {0, 2 * P8_REG, 3 * P8_REG, P8_REG};
  // K % 64 != 0: the last K-tile has krem valid k; every lane's source is clamped into the
  // tensor (finite data) and the A fragments of k >= krem are zeroed before the MFMAs.
  // (KTAIL = false instantiations assume K % 64 == 0 and carry none of this code; a K-piece
  // that does not end the reduction has no tail)
  const int krem = (KTAIL && kt0 + nk == nk_all) ? (int)(p.K - (int64_t)(nk_all - 1) * 64) : 64;  // 1..64
  auto issue = [&](int piece, int kt) {
    char* dst = smem + (kt & 1) * P8_BUF + lds_off[piece] + wave * 1024;
    const bool isA = piece == 0 || piece == 3;
    const int64_t step = isA ? stepA : stepB;
    const bool kc = isA ? AKC : BKC;
    const int region = (piece == 3 || piece == 2) ? 1 : 0;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const bf16_t* g = src[piece][i] + kt * step;
      if (KTAIL && krem < 64 && kt == nk - 1) {
        if (kc) {  // this lane's 8 k: 8 * chunk within the tile
          const int r = i * 64 + (t >> 3);
          const int kl = 8 * ((t & 7) ^ ((r >> 1) & 7));
          if (kl >= krem) g -= kl - (krem - 8);
        } else {   // this lane's k-row within the tile
          const int kl = region * 32 + i * 16 + (t >> 5);
          if (kl >= krem) g -= (int64_t)(kl - (krem - 1)) * (isA ? p.lda : p.ldb);
        }
      }
      glds16(g, dst + i * 8192);
    }
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 af[4][2], bf[2][2][2];  // A quadrant rows (4 x 16) x kk;  B [bh][2 x 16 cols][kk]
  auto mask_tail_a = [&](int kt) {
    if (KTAIL && krem < 64 && kt == nk - 1) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
          if (kk * 32 + 8 * (lane >> 4) >= krem) af[i][kk] = bf16x8{};
    }
  };

  auto read_a = [&](const char* buf, int ah) {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
        af[i][kk] = AKC ? frag<true>(buf + ah * P8_REG, wr * 4 + i, kk, lane)
                        : frag_tr_asm<512>(buf, wr * 8 + ah * 4 + i, kk, lane);
  };
  auto read_b = [&](const char* buf, int bh) {
    const char* reg = buf + 2 * P8_REG + (wc >> 1) * P8_REG;
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
        bf[bh][j][kk] = BKC ? frag<true>(reg, (wc & 1) * 4 + bh * 2 + j, kk, lane)
                            : frag_tr_asm<512>(buf + 2 * P8_REG, wc * 4 + bh * 2 + j, kk, lane);
  };
  auto mfma_quad = [&](int ah, int bh) {
    __builtin_amdgcn_s_setprio(1);
    if (F8) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[ah * 4 + i][bh * 2 + j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(
              cat_f8(bf[bh][j][0], bf[bh][j][1]), cat_f8(af[i][0], af[i][1]), acc[ah * 4 + i][bh * 2 + j], 0, 0, 0, 0,
              0, 0);
    } else {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            acc[ah * 4 + i][bh * 2 + j] =
                __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[bh][j][kk], af[i][kk], acc[ah * 4 + i][bh * 2 + j], 0, 0, 0);
    }
    __builtin_amdgcn_s_setprio(0);
  };

  // Per-operand schedule.  k-contiguous operands stream region by region as soon as each is
  // free (A: A1(kt+1) in phase 0, A0(kt+2) in phase 1; B: B0 in 2, B1 in 3); k-strided ones
  // load both regions together (B in phase 2, A in phase 3) so every k-row's 512-B span is
  // fetched by back-to-back instructions.  vmcnt counts (pieces of 2 DMA instructions issued
  // after the one a wait retires) are the same for all four combinations: 5 / 4 at phase 1
  // (A split only), 4 at phase 3; tails retire everything.
  constexpr bool AS = AKC, BS = BKC;
#ifndef PZ_GEMM_QUAD4
  if constexpr (AS) {
    // Two sections per K-tile (A k-contiguous; B either way -- a k-strided B is read whole in section 0 through
    // transposed loads): section 0 reads A region 0 and all of B (16 fragment loads) and runs quadrants
    // (0,0), (0,1); section 1 reads A region 1 (8) and runs (1,1), (1,0).  32 MFMAs per section against the other row group's reads; the four-phase
    // schedule below front-loads 12 of its 24 loads into one 16-MFMA phase, and its loads, not its DMA, set
    // that phase's length (profiles/r05/feed_ab_*.log).  DMA: A1(kt+1) in section 0 (its region was last read
    // in section 1 of kt-1), A0 | B0 | B1 (kt+2) in section 1 (last read in section 0 of kt).  Waits (2 DMA
    // instructions per piece): section 0 retires A1(kt) (4 newer pieces), section 1 retires tile kt+1's
    // section-0 pieces (4 newer, or only A1(kt+1) on the next-to-last tile); each is followed by the
    // barrier the next reader of those regions passes.
    issue(0, 0);
    issue(1, 0);
    issue(2, 0);
    issue(3, 0);
    if (nk > 1) {
      issue(0, 1);
      issue(1, 1);
      issue(2, 1);
      PZ_WAIT_VM(8);
    } else {
      PZ_WAIT_VM(2);
    }
    PZ_RAW_BARRIER();
    if (wr == 1) PZ_RAW_BARRIER();  // stagger: row-1 waves run one barrier behind
    for (int kt = 0; kt < nk; ++kt) {
      const char* buf = smem + (kt & 1) * P8_BUF;
      const bool n1 = kt + 1 < nk, n2 = kt + 2 < nk;
      // section 0: quadrants (0,0), (0,1)
      if (n1) issue(3, kt + 1);
      read_a(buf, 0);
      read_b(buf, 0);
      read_b(buf, 1);
      if (n1) PZ_WAIT_VM(8);
      else PZ_WAIT_VM(0);
      PZ_WAIT_LGKM0();
      PZ_RAW_BARRIER();
      mask_tail_a(kt);
      mfma_quad(0, 0);
      mfma_quad(0, 1);
      PZ_RAW_BARRIER();
      // section 1: quadrants (1,1), (1,0)
      if (n2) {
        issue(0, kt + 2);
        issue(1, kt + 2);
        issue(2, kt + 2);
      }
      read_a(buf, 1);
      if (n2) PZ_WAIT_VM(8);
      else if (n1) PZ_WAIT_VM(2);
      PZ_WAIT_LGKM0();
      PZ_RAW_BARRIER();
      mask_tail_a(kt);
      mfma_quad(1, 1);
      mfma_quad(1, 0);
      PZ_RAW_BARRIER();
    }
  } else
#endif
  {
  if (AS) {
    issue(0, 0);
    issue(1, 0);
    issue(2, 0);
    issue(3, 0);
    if (nk > 1) {
      issue(0, 1);
      issue(1, 1);
      issue(2, 1);
      PZ_WAIT_VM(8);
    } else {
      PZ_WAIT_VM(2);
    }
  } else {
    issue(1, 0);
    issue(2, 0);
    issue(0, 0);
    issue(3, 0);
    if (nk > 1) {
      issue(1, 1);
      issue(2, 1);
      issue(0, 1);
      issue(3, 1);
      PZ_WAIT_VM(8);
    } else {
      PZ_WAIT_VM(0);
    }
  }
  PZ_RAW_BARRIER();
  if (wr == 1) PZ_RAW_BARRIER();  // stagger: row-1 waves run one barrier behind

  for (int kt = 0; kt < nk; ++kt) {
    const char* buf = smem + (kt & 1) * P8_BUF;
    const bool n1 = kt + 1 < nk, n2 = kt + 2 < nk;
    // phase 0: quadrant (0,0)
    if (AS && n1) issue(3, kt + 1);
    read_a(buf, 0);
    read_b(buf, 0);
    PZ_WAIT_LGKM0();
    PZ_RAW_BARRIER();
    mask_tail_a(kt);
    mfma_quad(0, 0);
    PZ_RAW_BARRIER();
    // phase 1: quadrant (0,1); (A split) retire A region 1 of this tile for phase 2
    if (AS && n2) issue(0, kt + 2);
    read_b(buf, 1);
    if (AS) {
      if (n2) PZ_WAIT_VM(10);
      else if (n1) PZ_WAIT_VM(8);
      else PZ_WAIT_VM(0);
    }
    PZ_WAIT_LGKM0();
    PZ_RAW_BARRIER();
    mfma_quad(0, 1);
    PZ_RAW_BARRIER();
    // phase 2: quadrant (1,1)
    if (n2) {
      issue(1, kt + 2);
      if (!BS) issue(2, kt + 2);
    }
    read_a(buf, 1);
    PZ_WAIT_LGKM0();
    PZ_RAW_BARRIER();
    mask_tail_a(kt);
    mfma_quad(1, 1);
    PZ_RAW_BARRIER();
    // phase 3: quadrant (1,0); retire tile kt+1's phase-0 operands (all of A when merged)
    if (n2) {
      if (BS) issue(2, kt + 2);
      if (!AS) {
        issue(0, kt + 2);
        issue(3, kt + 2);
      }
    }
    if (n2) PZ_WAIT_VM(8);
    else if (n1) {
      if (AS) PZ_WAIT_VM(2);
      else PZ_WAIT_VM(0);
    }
    PZ_RAW_BARRIER();
    mfma_quad(1, 0);
    PZ_RAW_BARRIER();
  }
  }
  if (wr == 0) PZ_RAW_BARRIER();
  if (F8 && p.rs) {  // per-row activation scale: lane rows m0 + wr*128 + 16 rb + (lane & 15)
#pragma unroll
    for (int rb = 0; rb < 8; ++rb) {
      const int64_t row = min(m0 + wr * 128 + 16 * rb + (lane & 15), p.M - 1);
      const float sr = p.rs[row];
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) acc[rb][cb] *= sr;
    }
  }

  if (p.dbg == 1) return;
  if (piece >= 0) {  // split tail: raw partial sums, summed + epilogued by gemm8p_tail_epilogue
    f32x4* W = reinterpret_cast<f32x4*>(p.ws) + (int64_t)piece * (32 * NT2);
#pragma unroll
    for (int rb = 0; rb < 8; ++rb)
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) W[(rb * 4 + cb) * NT2 + t] = acc[rb][cb];
    return;
  }
  epilogue8p<GEGLU>(p, zo * p.sCo + zi * p.sCi, zo * p.sRo + zi * p.sRi, m0, n0, wr, wc, lane, acc, smem);
}

template <bool AKC, bool BKC, bool GEGLU, bool KTAIL>
__global__ void __launch_bounds__(NT2, 1) gemm8p_kernel(GemmP p) {
  gemm8p_body<AKC, BKC, GEGLU, KTAIL, false>(p);
}

// fp8 e4m3 x e4m3 (W8A8) instantiation of the 8-phase kernel (C5 prefill MLP GEMMs)
template <bool GEGLU, bool KTAIL>
__global__ void __launch_bounds__(NT2, 1) gemm8p_f8_kernel(GemmP p) {
  gemm8p_body<true, true, GEGLU, KTAIL, true>(p);
}

// ---- k-half variant of the ping-pong kernel -----------------------------------
// Same tile (256 x 256 x 64, 8 waves of 128 x 64), same accumulator layout, epilogue and split
// tail as gemm8p_kernel, but each K-tile is consumed in TWO segments per wave -- k 0..31 then
// k 32..63, each 32 MFMAs over the whole 128 x 64 wave tile -- instead of four 16-MFMA quadrant
// segments: half the barriers per K-tile and twice the matrix work beside each partner's
// LDS-read segment.  LDS regions are k-halves (per buffer: A h0 | A h1 | B h0 | B h1, 16 KiB
// each): k-contiguous images are [256 rows][32 k] (64-B rows, 16-B chunk c of row r at
// c ^ 3*((r >> 3) & 1): conflict-free ds_read_b128), k-strided ones the [32 k][256 rows] images of
// gemm8p_kernel.  Region (kt, h) is refilled with tile kt + 2 as soon as both wave groups have read
// it (h0 in segment 2 of kt, h1 in segment 0 of kt + 1): ~1.5 K-tiles of loads stay in flight.
constexpr int KH_REG = 16384;

template <bool GEGLU>
__device__ __forceinline__ int64_t kh_rowB(int v, int64_t row0, int64_t R, int64_t gI) {
  if (GEGLU) {  // virtual column v: wave (v >> 6), gate/up (v >> 5 & 1)
    int64_t g = row0 + (v >> 6) * 32 + (v & 31);
    g = g < gI ? g : gI - 1;
    return ((v >> 5) & 1) ? gI + g : g;
  }
  const int64_t g = row0 + v;
  return g < R ? g : R - 1;
}

// per-thread global source of DMA instruction i (0/1) of the k-half-0 region image of an operand
template <bool KC, bool GEGLU>
__device__ __forceinline__ const bf16_t* kh_src(const bf16_t* base, int64_t ld, int i, int t, int64_t row0,
                                                int64_t R, int64_t gI) {
  if (KC) {
    const int r = i * 128 + (t >> 2);
    const int ch = (t & 3) ^ (3 * ((r >> 3) & 1));
    return base + kh_rowB<GEGLU>(r, row0, R, gI) * ld + 8 * ch;
  } else {
    const int k = i * 16 + (t >> 5);
    const int c = (t & 31) ^ (sw_tr(k) >> 1);
    int64_t g = row0 + 8 * c;
    g = g <= R - 8 ? g : R - 8;
    return base + (int64_t)k * ld + g;
  }
}

template <bool KC>
__device__ __forceinline__ bf16x8 kh_frag(const char* opbase, int h, int rb, int lane) {
  if (KC) {
    const char* reg = opbase + h * KH_REG;
    const int r = rb * 16 + (lane & 15);
    const int ch = lane >> 4;
    return *reinterpret_cast<const bf16x8*>(reg + r * 64 + ((ch ^ (3 * ((r >> 3) & 1))) << 4));
  } else {
    return frag_tr_asm<512>(opbase, rb, h, lane);  // k-half h = k-rows 32h.. at 16 KiB * h
  }
}

template <bool AKC, bool BKC, bool GEGLU, bool KTAIL>
__global__ void __launch_bounds__(NT2, 1) gemm8k_kernel(GemmP p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int nk_all = (int)((p.K + 63) / 64);
  int lid = blockIdx.x, piece = -1, kt0 = 0, nk = nk_all;
  if (p.tail_s && lid >= p.dp_tiles) {
    const int u = lid - p.dp_tiles;
    piece = u;
    lid = p.dp_tiles + u / p.tail_s;
    kt0 = (u % p.tail_s) * p.tail_kt;
    nk = min(nk_all - kt0, p.tail_kt);
  }
  int tm, tn;
  tile_coords(lid, p.tiles_m * p.tiles_n, p.tiles_m, p.tiles_n, tm, tn, p.group);
  const int64_t m0 = (int64_t)tm * BT;
  const int64_t n0 = GEGLU ? (int64_t)tn * (BT / 2) : (int64_t)tn * BT;
  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int64_t z = blockIdx.y;
  const int64_t zo = z / p.batch_inner, zi = z % p.batch_inner;
  const bf16_t* Ab = p.A + zo * p.sAo + zi * p.sAi;
  const bf16_t* Bb = p.B + zo * p.sBo + zi * p.sBi;

  const int64_t stepA = AKC ? 64 : 64 * p.lda;
  const int64_t stepB = BKC ? 64 : 64 * p.ldb;
  const int64_t halfA = AKC ? 32 : 32 * p.lda;
  const int64_t halfB = BKC ? 32 : 32 * p.ldb;
  const bf16_t* srcA[2];
  const bf16_t* srcB[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    srcA[i] = kh_src<AKC, false>(Ab, p.lda, i, t, m0, p.M, 0) + kt0 * stepA;
    srcB[i] = kh_src<BKC, GEGLU>(Bb, p.ldb, i, t, n0, p.N, p.geglu_I) + kt0 * stepB;
  }
  const int krem = (KTAIL && kt0 + nk == nk_all) ? (int)(p.K - (int64_t)(nk_all - 1) * 64) : 64;
  // K % 64 != 0: every lane's source of the last K-tile is clamped into the tensor (finite data)
  // and the A fragments of k >= krem are zeroed before the MFMAs
  auto clamp_tail = [&](const bf16_t* g, bool kc, int h, int i, int64_t ld, int kt) {
    if (KTAIL && krem < 64 && kt == nk - 1) {
      if (kc) {
        const int r = i * 128 + (t >> 2);
        const int kl = 32 * h + 8 * ((t & 3) ^ (3 * ((r >> 3) & 1)));
        if (kl >= krem) g -= kl - (krem - 8);
      } else {
        const int kl = 32 * h + i * 16 + (t >> 5);
        if (kl >= krem) g -= (int64_t)(kl - (krem - 1)) * ld;
      }
    }
    return g;
  };
  // k-half h of K-tile kt (both operands): 2 + 2 DMA instructions per wave
  auto issue = [&](int kt, int h) {
    char* dst = smem + (kt & 1) * P8_BUF + h * KH_REG + wave * 1024;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      glds16(clamp_tail(srcA[i] + kt * stepA + h * halfA, AKC, h, i, p.lda, kt), dst + i * 8192);
      glds16(clamp_tail(srcB[i] + kt * stepB + h * halfB, BKC, h, i, p.ldb, kt), dst + 2 * KH_REG + i * 8192);
    }
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 af[8], bfr[4];
  auto read_frags = [&](const char* buf, int h) {
#pragma unroll
    for (int i = 0; i < 8; ++i) af[i] = kh_frag<AKC>(buf, h, wr * 8 + i, lane);
#pragma unroll
    for (int j = 0; j < 4; ++j) bfr[j] = kh_frag<BKC>(buf + 2 * KH_REG, h, wc * 4 + j, lane);
  };
  auto mask_tail_a = [&](int kt, int h) {
    if (KTAIL && krem < 64 && kt == nk - 1) {
      if (32 * h + 8 * (lane >> 4) >= krem) {
#pragma unroll
        for (int i = 0; i < 8; ++i) af[i] = bf16x8{};
      }
    }
  };
  auto mfma_half = [&]() {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  // issue order: (0,0) (0,1) (1,0) | per tile kt: (kt+1,1) in segment 0, (kt+2,0) in segment 2.
  // Waits (4 DMA instructions per wave per k-half): segment 0 retires (kt,1), segment 2 retires
  // (kt+1,0); each is followed by the barrier the next reader of that region passes.
  issue(0, 0);
  issue(0, 1);
  if (nk > 1) {
    issue(1, 0);
    PZ_WAIT_VM(8);
  } else {
    PZ_WAIT_VM(4);
  }
  PZ_RAW_BARRIER();
  if (wr == 1) PZ_RAW_BARRIER();  // stagger: waves 4..7 run one barrier behind

  for (int kt = 0; kt < nk; ++kt) {
    const char* buf = smem + (kt & 1) * P8_BUF;
    const bool n1 = kt + 1 < nk, n2 = kt + 2 < nk;
    // segment 0: read k-half 0
    if (n1) issue(kt + 1, 1);
    read_frags(buf, 0);
    if (n1) PZ_WAIT_VM(8);
    else PZ_WAIT_VM(0);
    PZ_WAIT_LGKM0();
    PZ_RAW_BARRIER();
    // segment 1: MFMAs of k-half 0
    mask_tail_a(kt, 0);
    mfma_half();
    PZ_RAW_BARRIER();
    // segment 2: read k-half 1
    if (n2) issue(kt + 2, 0);
    read_frags(buf, 1);
    if (n2) PZ_WAIT_VM(8);
    else if (n1) PZ_WAIT_VM(4);
    PZ_WAIT_LGKM0();
    PZ_RAW_BARRIER();
    // segment 3: MFMAs of k-half 1
    mask_tail_a(kt, 1);
    mfma_half();
    PZ_RAW_BARRIER();
  }
  if (wr == 0) PZ_RAW_BARRIER();

  if (piece >= 0) {
    f32x4* W = reinterpret_cast<f32x4*>(p.ws) + (int64_t)piece * (32 * NT2);
#pragma unroll
    for (int rb = 0; rb < 8; ++rb)
#pragma unroll
      for (int cb = 0; cb < 4; ++cb) W[(rb * 4 + cb) * NT2 + t] = acc[rb][cb];
    return;
  }
  epilogue8p<GEGLU>(p, zo * p.sCo + zi * p.sCi, zo * p.sRo + zi * p.sRi, m0, n0, wr, wc, lane, acc, smem);
}

// Split tail, second pass: 16 blocks of 512 threads per leftover tile (one accumulator row-block rb and
// one column half each, so the partial sums stream through many CUs); thread t sums the tail_s
// partial accumulators it owned in gemm8p_kernel (fixed order) and applies the same epilogue.
template <bool GEGLU, int PB = 8>
__global__ void __launch_bounds__(NT2) gemm8p_tail_epilogue(GemmP p) {
  const int tile = blockIdx.x >> 4, rb = (blockIdx.x >> 1) & 7, h = blockIdx.x & 1;
  int tm, tn;
  tile_coords(p.dp_tiles + tile, p.tiles_m * p.tiles_n, p.tiles_m, p.tiles_n, tm, tn, p.group);
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6, wr = wave >> 2, wc = wave & 3;
  const f32x4* W = reinterpret_cast<const f32x4*>(p.ws) + (int64_t)tile * p.tail_s * (32 * NT2);
  // GeGLU pairs gate cb = h with up cb = h + 2; plain outputs take cb = 2h, 2h + 1
  const int c0 = GEGLU ? h : 2 * h, c1 = GEGLU ? h + 2 : 2 * h + 1;
  // pieces loaded PB at a time (2 PB loads in flight per thread), summed in piece order (deterministic)
  const f32x4* W0 = W + (rb * 4 + c0) * NT2 + t;
  const f32x4* W1 = W + (rb * 4 + c1) * NT2 + t;
  auto sum_pieces = [&](f32x4& a0, f32x4& a1) {
    a0 = a1 = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int z = 0; z < p.tail_s; z += PB) {
      f32x4 v0[PB], v1[PB];
#pragma unroll
      for (int u = 0; u < PB; ++u) {
        const bool ok = z + u < p.tail_s;
        v0[u] = ok ? W0[(int64_t)(z + u) * (32 * NT2)] : f32x4{0.f, 0.f, 0.f, 0.f};
        v1[u] = ok ? W1[(int64_t)(z + u) * (32 * NT2)] : f32x4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int u = 0; u < PB; ++u) {
        a0 += v0[u];
        a1 += v1[u];
      }
    }
  };
  const int64_t m = (int64_t)tm * BT + wr * 128 + rb * 16 + (lane & 15);
  f32x4 a0, a1;
  if (GEGLU) {
    sum_pieces(a0, a1);
    store_geglu4(p, 0, m, (int64_t)tn * (BT / 2) + wc * 32 + h * 16 + 4 * (lane >> 4), a0, a1);
  } else {
    const int64_t n = (int64_t)tn * BT + wc * 64 + 4 * (lane >> 4);
    // the epilogue's side inputs (residual, saved activation, bias) issued with the first pieces, not after the sum
    epi_dispatch(p, [&](auto em) {
      constexpr int EM = decltype(em)::value;
      Side s0, s1;
      epi_load4<EM>(p, 0, 0, m, n + c0 * 16, s0);
      epi_load4<EM>(p, 0, 0, m, n + c1 * 16, s1);
      const u32x2 b0 = epi_load_bias(p, n + c0 * 16), b1 = epi_load_bias(p, n + c1 * 16);
      sum_pieces(a0, a1);
      epi_store4<EM>(p, 0, 0, m, n + c0 * 16, a0, s0, b0);
      epi_store4<EM>(p, 0, 0, m, n + c1 * 16, a1, s1, b1);
    });
  }
}

// -------------------------------------------------------------------------
// Skinny GEMM for M <= 16 (inference denoise steps, B = 1..4): weights are
// streamed once straight into VGPRs (no LDS), a block of W waves per 16 output
// columns, K split into W contiguous ranges (one per wave, loads issued 8 / 4
// chunks ahead of their MFMAs so each lane keeps up to 8 x 16 B of weights in
// flight) and reduced through LDS.  W = 4/8/16 by K so every wave has >= 4
// chunks of 32.  Operands k-contiguous (nn.Linear weight layout).
// -------------------------------------------------------------------------
template <int W, int NC>
__global__ void __launch_bounds__(W * 64) gemm_skinny_kernel(GemmP p) {
  constexpr int SK_WAVES = W;
  __shared__ f32x4 red[SK_WAVES][64];
  __shared__ float redn[SK_WAVES][16];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const bool geglu = p.epi == PZ_EPI_GEGLU;
  const bool nrm = p.nw != nullptr;
  const int64_t ncols = geglu ? p.geglu_I : p.N;
  // NC < 16 output columns per block (more blocks for narrow outputs): the 16 MFMA columns repeat
  // the NC real ones (same addresses, no extra traffic) and only the first NC are stored
  const int64_t n0 = (int64_t)blockIdx.x * NC;
  const int64_t z = blockIdx.y;
  const int64_t zo = z / p.batch_inner, zi = z % p.batch_inner;
  const bf16_t* A = p.A + zo * p.sAo + zi * p.sAi;
  const bf16_t* B = p.B + zo * p.sBo + zi * p.sBi;
  const int64_t m = lane & 15;
  const int64_t nr = n0 + (lane & 15) % NC;
  const bool mok = m < p.M, nok = nr < ncols;
  const int64_t kchunks = p.K / 32;  // K % 32 == 0 required (host checked)
  f32x4 acc = {0.f, 0.f, 0.f, 0.f}, acc2 = {0.f, 0.f, 0.f, 0.f};
  float ss = 0.f;
  const bf16_t* Arow = A + m * p.lda + 8 * (lane >> 4);
  const bf16_t* Brow = B + nr * p.ldb + 8 * (lane >> 4);
  const bf16_t* Brow2 = B + (p.geglu_I + nr) * p.ldb + 8 * (lane >> 4);
  const bf16_t* Wn = p.nw + 8 * (lane >> 4);
  const int64_t per = (kchunks + SK_WAVES - 1) / SK_WAVES;
  const int64_t kb = wave * per, ke = min(kchunks, kb + per);
  int64_t kc = kb;
  auto run = [&](auto U_) {
    constexpr int U = decltype(U_)::value;
    for (; kc + U <= ke; kc += U) {
      bf16x8 a[U], b[U], b2[U], wv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        a[u] = mok ? *reinterpret_cast<const bf16x8*>(Arow + (kc + u) * 32) : bf16x8{};
        b[u] = nok ? *reinterpret_cast<const bf16x8*>(Brow + (kc + u) * 32) : bf16x8{};
        if (geglu) b2[u] = nok ? *reinterpret_cast<const bf16x8*>(Brow2 + (kc + u) * 32) : bf16x8{};
        if (nrm) wv[u] = *reinterpret_cast<const bf16x8*>(Wn + (kc + u) * 32);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (nrm) {  // sum of squares of the raw row; the product takes x * (1 + w), rsqrt applied after
          const u32x4 xa = __builtin_bit_cast(u32x4, a[u]), xw = __builtin_bit_cast(u32x4, wv[u]);
          u32x4 o;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float x0 = __uint_as_float(xa[e] << 16), x1 = __uint_as_float(xa[e] & 0xffff0000u);
            const float w0 = __uint_as_float(xw[e] << 16), w1 = __uint_as_float(xw[e] & 0xffff0000u);
            ss += x0 * x0 + x1 * x1;
            o[e] = pack2bf(x0 * (1.f + w0), x1 * (1.f + w1));
          }
          a[u] = __builtin_bit_cast(bf16x8, o);
        }
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b[u], a[u], acc, 0, 0, 0);
        if (geglu) acc2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b2[u], a[u], acc2, 0, 0, 0);
      }
    }
  };
  run(std::integral_constant<int, 8>{});
  run(std::integral_constant<int, 4>{});
  run(std::integral_constant<int, 1>{});
  // D[n_local = 4*(lane>>4)+r][m = lane&15]
  red[wave][lane] = acc;
  if (nrm) {
    ss += __shfl_xor(ss, 16, 64);
    ss += __shfl_xor(ss, 32, 64);
    if (lane < 16) redn[wave][lane] = ss;
  }
  __syncthreads();
  if (wave == 0) {
    for (int w = 1; w < SK_WAVES; ++w) acc += red[w][lane];
  }
  if (geglu) {
    __syncthreads();
    red[wave][lane] = acc2;
    __syncthreads();
    if (wave == 0)
      for (int w = 1; w < SK_WAVES; ++w) acc2 += red[w][lane];
  }
  if (wave != 0) return;
  const int64_t mm = lane & 15;
  if (mm >= p.M) return;
  float scale = p.alpha;
  if (nrm) {
    float t = 0.f;
    for (int w = 0; w < SK_WAVES; ++w) t += redn[w][mm];
    scale *= rsqrtf(t / (float)p.K + p.neps);
  }
  const int64_t n = n0 + 4 * (lane >> 4);
  const int64_t cofs = zo * p.sCo + zi * p.sCi;
  const int64_t rofs = zo * p.sRo + zi * p.sRi;
  for (int r = 0; r < 4; ++r) {
    const int64_t nn = n + r;
    if (4 * (lane >> 4) + r >= NC || nn >= ncols) continue;
    float x = acc[r] * scale;
    if (geglu) {
      const float g = x, u = acc2[r] * scale;
      if (p.aux) {
        p.aux[mm * p.ld_aux + nn] = f2bf(g);
        p.aux[mm * p.ld_aux + p.geglu_I + nn] = f2bf(u);
      }
      x = gelu_tanh(g) * u;
    } else {
      if (p.bias) x += bf2f(p.bias[nn]);
      if (p.epi == PZ_EPI_GELU || p.epi == PZ_EPI_SILU) {
        if (p.aux) p.aux[mm * p.ld_aux + nn] = f2bf(x);
        x = p.epi == PZ_EPI_GELU ? gelu_tanh(x) : silu(x);
      }
      if (p.resid) x += bf2f(p.resid[rofs + mm * p.ld_resid + nn]);
    }
    if (p.c_fp32) {
      float* Cp = reinterpret_cast<float*>(p.C) + cofs + mm * p.ldc + nn;
      *Cp = p.beta ? *Cp + x : x;
    } else {
      bf16_t* Cp = reinterpret_cast<bf16_t*>(p.C) + cofs + mm * p.ldc + nn;
      *Cp = f2bf(p.beta ? bf2f(*Cp) + x : x);
    }
  }
}

// -------------------------------------------------------------------------
// Small strided fp32-accumulate GEMM for the K=7 / N=7 action/proprio linears
// (SURVEY 2.2 "proprio enc / action dec": 0.03 GF).  One thread per output.
// -------------------------------------------------------------------------
__global__ void gemm_small_kernel(pz_small_gemm_args a) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= a.M * a.N) return;
  const int64_t m = idx / a.N, n = idx % a.N;
  const bf16_t* A = (const bf16_t*)a.A;
  const bf16_t* B = (const bf16_t*)a.B;
  float s = 0.f;
  for (int64_t k = 0; k < a.K; ++k)
    s += bf2f(A[m * a.sAm + k * a.sAk]) * bf2f(B[k * a.sBk + n * a.sBn]);
  s *= a.alpha;
  if (a.bias) s += bf2f(((const bf16_t*)a.bias)[n]);
  bf16_t* C = (bf16_t*)a.C + m * a.ldc + n;
  if (a.beta) s += bf2f(*C);
  *C = f2bf(s);
}

// Long-K / tiny-N case (action decoder, pizero.py:100-103: [rows, 1024] x [7, 1024]^T): one wave
// per output row, lanes split K in 16-B chunks (k-contiguous A and B), butterfly reduction.
constexpr int SMALL_NMAX = 8;
__global__ void __launch_bounds__(256) gemm_small_rowwave_kernel(pz_small_gemm_args a) {
  const int lane = threadIdx.x & 63;
  const int64_t m = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (m >= a.M) return;
  const bf16_t* A = (const bf16_t*)a.A + m * a.sAm;
  const bf16_t* B = (const bf16_t*)a.B;
  float s[SMALL_NMAX];
#pragma unroll
  for (int n = 0; n < SMALL_NMAX; ++n) s[n] = 0.f;
  for (int64_t k = 8 * lane; k < a.K; k += 512) {
    const u32x4 xa = *reinterpret_cast<const u32x4*>(A + k);
    float x[8];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      x[2 * e] = bf2f(xa[e] & 0xffff);
      x[2 * e + 1] = bf2f(xa[e] >> 16);
    }
#pragma unroll
    for (int n = 0; n < SMALL_NMAX; ++n) {
      if (n >= a.N) break;
      const u32x4 wb = *reinterpret_cast<const u32x4*>(B + n * a.sBn + k);
#pragma unroll
      for (int e = 0; e < 4; ++e) s[n] += x[2 * e] * bf2f(wb[e] & 0xffff) + x[2 * e + 1] * bf2f(wb[e] >> 16);
    }
  }
#pragma unroll
  for (int n = 0; n < SMALL_NMAX; ++n) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) s[n] += __shfl_xor(s[n], off);
  }
  if (lane < a.N) {
    float v = 0.f;
#pragma unroll
    for (int n = 0; n < SMALL_NMAX; ++n)
      if (n == lane) v = s[n];
    v *= a.alpha;
    if (a.bias) v += bf2f(((const bf16_t*)a.bias)[lane]);
    bf16_t* C = (bf16_t*)a.C + m * a.ldc + lane;
    if (a.beta) v += bf2f(*C);
    *C = f2bf(v);
  }
}

}  // namespace

// ----------------------------------------------------------------- host ----

static thread_local char g_err[512];
void pz_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

extern "C" const char* pz_last_error(void) { return g_err; }

extern "C" int pz_abi_version(void) { return PZ_ABI_VERSION; }

template <bool AKC, bool BKC, int WM, int TAG = 0>
static int launch_tile(const GemmP& p, int64_t batch, hipStream_t st) {
  const int smem = 4 * TILE_BYTES;
  auto kern = gemm_kernel<AKC, BKC, WM, TAG>;
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, smem);
    attr_set = true;
  }
  static int xb = -1;  // PZ_GEMM_BATCH_XCD=0: 2-D grid (A/B; read once)
  if (xb < 0) {
    const char* e = getenv("PZ_GEMM_BATCH_XCD");
    xb = !(e && e[0] == '0');
  }
  if (xb && p.ksplit == 0 && batch >= 8 && batch % 8 == 0 && (int64_t)p.tiles_m * p.tiles_n * batch < (1LL << 31)) {
    GemmP q = p;
    q.batch_xcd = (int)batch;
    hipLaunchKernelGGL(kern, dim3((unsigned)(p.tiles_m * p.tiles_n * batch)), dim3(NT), smem, st, q);
    PZ_CHECK_LAUNCH();
    return PZ_OK;
  }
  dim3 grid(p.tiles_m * p.tiles_n, (unsigned)batch);
  hipLaunchKernelGGL(kern, grid, dim3(NT), smem, st, p);
  PZ_CHECK_LAUNCH();
  return PZ_OK;
}

template <bool AKC, bool BKC, bool GEGLU>
static int launch256(const GemmP& p, int64_t batch, hipStream_t st) {
  const int smem = 2 * 2 * 256 * 64 * 2;  // 128 KiB for either pipeline
  auto kern = gemm256_kernel<AKC, BKC, GEGLU, BK256>;
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, smem);
    attr_set = true;
  }
  hipLaunchKernelGGL(kern, dim3(p.tiles_m * p.tiles_n, (unsigned)batch), dim3(NT2), smem, st, p);
  PZ_CHECK_LAUNCH();
  return PZ_OK;
}

static bool use_8phase();
static bool use_khalf(bool akc, bool bkc, int64_t m, int64_t n, int64_t k);

namespace {
// skinny-64 split-K: partials summed in the launch (default) or by splitk_epilogue_kernel (PZ_SK64_FUSED=0)
static bool sk64_two_launch() {
  const char* e = getenv("PZ_SK64_FUSED");
  return e && e[0] == '0';
}

enum PathKind { PATH_SKINNY, PATH_256, PATH_TILE, PATH_SPLIT, PATH_GEMV, PATH_SKINNY64, PATH_ROWS, PATH_TALL };
struct Plan {
  PathKind kind;
  bool akc, bkc, geglu;
  int wm, tag, skinny_w, skinny_nc, skinny_mb, splits;
  int64_t ksplit, ldw, tiles_m, tiles_n;
  int dp_tiles, tail_s, tail_kt;  // 8-phase split tail (tail_s == 0: none)
  int rows_w, rows_tnb, rows_tmb;  // row-slab kernel: waves, 16-column / 16-row blocks per tile
  int rows_f8;                     // ... with e4m3 weight codes: 1 = W8A16, 2 = W8A8 (both operands codes)
  int tall_mi;                     // tall-tile kernel: 64 * tall_mi rows per tile (4 | 5)
};

// compute units of the current device (the "wave" of resident 8-phase workgroups: 1 per CU)
int device_cus() {
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

// Wave quantisation of the 8-phase kernel (one 256x256 tile per CU at a time): T = q*G + r tiles
// leave the last round r/G full.  Split each of the r leftover tiles into s K-pieces (s*r <= G)
// so the last round takes ~1/s of a tile time; partial sums go through the fp32 workspace.
// q == 0 (fewer tiles than CUs, e.g. weight gradients of small layers) is the same split.
void plan_tail(Plan& pl, const pz_gemm_args* a) {
  if (a->batch != 1 || !a->workspace || !PZ_ALIGNED(a->workspace, 16)) return;
  const char* e = getenv("PZ_GEMM_TAIL");  // "0": whole tiles only (A/B runs; read per call)
  if (e && e[0] == '0') return;
  const int64_t G = device_cus();
  const int64_t T = pl.tiles_m * pl.tiles_n;
  const int64_t q = T / G, r = T % G;
  const int64_t nk = (a->K + 63) / 64;
  // a leftover round at least half full runs about as fast as its K-pieces would (less contention);
  // after many rounds the workgroups no longer run in lockstep and the leftover tiles fill the gaps
  // (measured: split worse at q = 17, better at q <= 4)
  // (splitting a leftover round exactly half full -- micro-batch 128's SigLIP 1152-wide GEMMs, 640 tiles = 2 rounds +
  // 128 -- measured within noise: profiles/r04/siglip_1152_ab.txt)
  if (r == 0 || (q > 0 && 2 * r >= G) || q > 8) return;
  int64_t s = G / r;
  s = s < 16 ? s : 16;
  if (q == 0) {
    // the whole GEMM is the tail (weight gradients of the 1152-wide SigLIP layers: 70 / 85 / 25 tiles): the pieces
    // may take several rounds when that fills the CUs better.  Cost (us) = rounds(s) / s x nk x 1.8 (a 256 x 256 x 64
    // step at ~4.6 TF/s per CU) + r s x 0.1 (each piece's 256 KiB fp32 partial written and re-read, chip-wide):
    // 70 tiles x 1024 K-tiles -> 3 pieces in one 82 %-full round 635 us, 7 pieces in two 96 %-full rounds 576 us
    const int64_t smax = (int64_t)(a->ws_bytes / (32 * NT2 * 16)) / r;
    auto cost = [&](int64_t s2) { return (double)((r * s2 + G - 1) / G) / (double)s2 * (double)nk * 1.8 + r * s2 * 0.1; };
    double best = cost(s);
    for (int64_t s2 = s + 1; s2 <= 16 && s2 <= nk / 2 && s2 <= smax; ++s2) {
      const double c = cost(s2);
      if (c < best * 0.97) {
        best = c;
        s = s2;
      }
    }
  }
  // no split below 8 K-tiles: a piece writes (and the merge re-reads) a 256 KiB fp32 partial, which a short
  // reduction cannot amortise -- the K = 320 action-expert wgrad (8192 x 1024, 5 K-tiles) took 42.0 us with
  // 2 pieces per leftover tile vs 20.0 us whole (tools/shape_ab.py, profiles/r03/shape_ab.log)
  s = s < nk / 2 ? s : nk / 2;
  if (s < 2 || nk < 8) return;
  const int64_t kt = (nk + s - 1) / s;
  s = (nk + kt - 1) / kt;
  if (s < 2 || r * s * (int64_t)(32 * NT2 * 16) > a->ws_bytes) return;
  pl.dp_tiles = (int)(q * G);
  pl.tail_s = (int)s;
  pl.tail_kt = (int)kt;
}

// row-slab kernel (64 < M <= PZ_ROWS_MAXM, default 512; k-contiguous A and B, batch 1, forward
// epilogues): whole-K 64-row tiles, 16 / 32 / 64 columns wide so the tiles cover >= 128 workgroups;
// 8 waves split K when it has >= 16 chunks (4 for GeGLU).  Taken where it measured faster than the
// 128-tile + split-K pair or the 256-tile kernel (tools/rows_bench.py, profiles/r03/rows_bench.log):
// K <= 2048 and <= 4096 output columns -- B = 1 SigLIP q|k|v 20.9 -> 12.0 us, o 14.6 -> 9.0 us, Gemma
// q|k|v / o at 276 rows 19.8 -> 18.1 us, action expert (320 rows) q|k|v 17.5 -> 11.0, o 16.0 -> 13.4,
// gate|up + GeGLU 32.9 -> 25.8 us; the long-K / wide ones (SigLIP fc1 / fc2, 4096-K down projections,
// the 32768-wide Gemma gate|up) stay on the tile kernels.  PZ_GEMM_ROWS=0: never; =1: any 64 < M <= maxm
// (A/B runs; read per call)
bool plan_rows(Plan& pl, const pz_gemm_args* a, int64_t ncols) {
  const char* er = getenv("PZ_GEMM_ROWS");
  const char* em = getenv("PZ_ROWS_MAXM");
  const int64_t maxm = em ? atoll(em) : 1024;  // (C5's 768 / 789 prefill rows: 21.32 vs 21.52 ms at 512)
  if ((er && er[0] == '0') || a->M <= 64 || a->M > maxm || !pl.akc || !pl.bkc || a->batch != 1 ||
      a->epilogue >= PZ_EPI_DGELU || a->norm_w)
    return false;
  if (!(er && er[0] == '1') && (a->K > 2048 || ncols > 4096)) return false;
  // e4m3 weights with bf16 rows (W8A16): 64-chunks of whole 16-code loads
  if (a->fp8_mode == 2 && (a->K % 64 != 0 || a->ldb % 16 != 0)) return false;
  pl.rows_f8 = a->fp8_mode == 2;
  // 64-row tiles (32-row tiles, twice the workgroups, measured slower on every shape: rows_bench.log)
  const int tmb = 4;
  const int64_t tm = (a->M + 16 * tmb - 1) / (16 * tmb);
  int tnb = pl.geglu ? 2 : 4;
  while (tnb > 1 && tm * ((ncols + 16 * tnb - 1) / (16 * tnb)) < 128) tnb /= 2;
  pl.kind = PATH_ROWS;
  pl.rows_w = (a->K + 63) / 64 >= 16 && !pl.geglu ? 8 : 4;
  const char* ew = getenv("PZ_ROWS_W");  // A/B overrides (read per call): waves 4 | 8, column blocks
  if (ew && (atoi(ew) == 4 || atoi(ew) == 8)) pl.rows_w = atoi(ew);
  const char* et = getenv("PZ_ROWS_TNB");
  if (et && (atoi(et) == 1 || atoi(et) == 2 || (atoi(et) == 4 && !pl.geglu))) tnb = atoi(et);
  pl.rows_tnb = tnb;
  pl.rows_tmb = tmb;
  pl.tiles_m = tm;
  pl.tiles_n = (ncols + 16 * tnb - 1) / (16 * tnb);
  return true;
}

// tall-tile kernel (pz_gemm_tall.hip): 64 < M <= 1024 rows, k-contiguous A and B, batch 1, bf16 operands, forward
// epilogues: one 256- or 320-row tile covers up to 320 rows (the B = 1 prefill's 276 rows in ONE row tile instead of
// the 8-phase kernel's two 256-row tiles), 64 output columns per tile, K split over blockIdx.y until the grid
// reaches ~256 workgroups.  Taken by default where it measured faster (tools/tall_bench.py,
// profiles/r04/tall_bench.log, and inside the B = 1 chunk, profiles/r04/infer_trace_split.txt): <= 320 rows against
// the long-K narrow projections (Gemma down 276 x 2048 x 16384: 49.8 -> 44.8 us isolated, 54.5 -> 44.0 us in the
// chunk incl. the merge; SigLIP fc2 256 x 1152 x 4304: 18.7 -> 18.1 us).  Not the B = 1 GeGLU gate|up: 55.4 vs
// 57.9 us isolated (weights L2/MALL-warm over the repeats) but 65.2 vs 60.7 us in the chunk, where they stream
// cold from HBM; slower on the short-K / narrow shapes the row-slab kernel takes and at 788 rows (the 8-phase
// kernel's 256-row tiles are then mostly full).  PZ_GEMM_TALL=1: every eligible shape, 0: never (A/B runs)
bool plan_tall(Plan& pl, const pz_gemm_args* a, int64_t ncols) {
  const char* e = getenv("PZ_GEMM_TALL");
  if (e && e[0] == '0') return false;
  if (!(e && e[0] == '1') &&
      !(a->M <= 320 && pl.bkc && !pl.geglu && a->K >= 4300 && ncols <= 2048))
    return false;
#ifndef PZ_TALL_AB
  if (!pl.bkc || pl.geglu) return false;  // only the plain k-contiguous form is built (pz_gemm_tall.hip)
#endif
  if (!pl.akc || (!pl.bkc && pl.geglu) || a->batch != 1 || a->fp8_mode != 0 || a->norm_w || a->epilogue >= PZ_EPI_DGELU ||
      a->M <= 64 || a->M > 1024 || a->K % 8 != 0)
    return false;
  const int64_t t5 = (a->M + 319) / 320, t4 = (a->M + 255) / 256;
  pl.tall_mi = t5 * 320 <= t4 * 256 ? 5 : 4;
  pl.tiles_m = pl.tall_mi == 5 ? t5 : t4;
  pl.tiles_n = (ncols + 63) / 64;
  const int64_t bkt = pl.geglu ? 32 : 64;
  const int64_t nk = (a->K + bkt - 1) / bkt;
  const int64_t units = pl.tiles_m * pl.tiles_n;
  int64_t S = (256 + units - 1) / units;
  S = S < nk / 4 ? S : nk / 4;  // >= 4 K-tiles per split
  S = S < 16 ? S : 16;
  if (S >= 2) {
    const int64_t per = (nk + S - 1) / S;
    const int64_t Se = (nk + per - 1) / per;
    const int64_t ldw = pl.geglu ? 2 * a->geglu_inter : (a->N + 3) / 4 * 4;
    if (Se >= 2 && a->workspace && PZ_ALIGNED(a->workspace, 16) && Se * a->M * ldw * 4 <= a->ws_bytes) {
      pl.splits = (int)Se;
      pl.ksplit = per * bkt;
      pl.ldw = ldw;
    }
  }
  pl.kind = PATH_TALL;
  return true;
}

// Kernel choice for a validated argument set (shared by pz_gemm and pz_gemm_kernel_name).
// skinny-64 split-K combined in the launch: S tile-private [64][nc] fp32 slabs per tile fit the workspace (bf16 C,
// forward epilogue)
static bool sk64_fits(const Plan& pl, const pz_gemm_args* a) {
  const int64_t tiles = pl.tiles_n * ((a->M + 63) / 64);
  return (int64_t)pl.splits * tiles * 64 * pl.skinny_nc * 4 <= a->ws_bytes && !a->c_fp32 &&
         a->epilogue < PZ_EPI_DGELU;
}

Plan make_plan(const pz_gemm_args* a) {
  Plan pl{};
  pl.akc = a->a_kcontig != 0;
  pl.bkc = a->b_kcontig != 0;
  pl.geglu = a->epilogue == PZ_EPI_GEGLU;
  const int64_t ncols = pl.geglu ? a->geglu_inter : a->N;
  // fp8 W8A8: the 8-phase 256-tile kernel on code pairs (K, lda, ldb halved by the caller of make_plan); the row-slab
  // shapes (64 < M <= 1024, <= 2048 codes of K in 128-code chunks, <= 4096 columns, no GeGLU: C5's prefill q|k|v / o)
  // take the W8A8 row-slab kernel (PZ_ROWS_W8A8=0: the 8-phase kernel, A/B; read per call)
  if (a->fp8_mode == 1) {
    const char* er8 = getenv("PZ_ROWS_W8A8");
    if (!(er8 && er8[0] == '0') && !pl.geglu && a->M > 64 && a->M <= 1024 && a->K % 64 == 0 && a->K <= 1024 &&
        ncols <= 4096 && a->a_row_scale) {
      const int64_t tm = (a->M + 63) / 64;
      int tnb = 4;
      while (tnb > 1 && tm * ((ncols + 16 * tnb - 1) / (16 * tnb)) < 128) tnb /= 2;
      pl.kind = PATH_ROWS;
      pl.rows_f8 = 2;
      pl.rows_w = a->K / 64 >= 8 ? 8 : 4;
      pl.rows_tnb = tnb;
      pl.rows_tmb = 4;
      pl.tiles_m = tm;
      pl.tiles_n = (ncols + 16 * tnb - 1) / (16 * tnb);
      return pl;
    }
    pl.kind = PATH_256;
    pl.tiles_m = (a->M + BT - 1) / BT;
    pl.tiles_n = (ncols + (pl.geglu ? BT / 2 : BT) - 1) / (pl.geglu ? BT / 2 : BT);
    plan_tail(pl, a);
    return pl;
  }
  // skinny-64 path: 16 < M <= 64 rows (bf16), or any M <= 64 with fp8 weights (W8A16)
  // rows 65..PZ_SK64_MAXM run as 64-row chunks of the same kernel (blockIdx.y)
  const char* emax = getenv("PZ_SK64_MAXM");
  const int64_t sk_maxm = emax ? atoll(emax) : 64;
  const bool sk64_ok = (a->M <= 64 || a->M <= sk_maxm) && pl.akc && pl.bkc && a->K % 64 == 0 && a->batch == 1 &&
                       !a->c_fp32 && a->epilogue < PZ_EPI_DGELU;
  const char* e64 = getenv("PZ_SK64");  // "0": rows 17..64 take the tile kernels (A/B; read per call)
  if (a->fp8_mode == 2 && a->M > 64) {  // W8A16 above 64 rows: the row-slab kernel or nothing (pz_gemm rejects)
    pl.kind = PATH_SKINNY64;
    plan_rows(pl, a, ncols);
    return pl;
  }
  if (a->fp8_mode == 2 || (sk64_ok && a->M > 16 && !(e64 && e64[0] == '0'))) {
    pl.kind = PATH_SKINNY64;
    pl.skinny_mb = a->M > 64 ? 4 : (int)((a->M + 15) / 16);
    pl.skinny_mb = pl.skinny_mb == 3 ? 4 : pl.skinny_mb;
    // 16 real columns per block, 8 waves: every block re-reads the (L2-resident) activation rows, so
    // narrower blocks multiply that traffic -- measured at 50 rows (tools/skinny_bench.py): q|k|v
    // 7.3 vs 16.8 us, gate|up 8.6 vs 25.6 us for 16 vs 4 columns; W = 8 never slower than 4
    pl.skinny_w = a->K / 64 >= 8 ? 8 : 4;
    pl.skinny_nc = 16;
    // narrow outputs (o / down projections: 64 blocks of 16 columns) split K over blockIdx.z so the
    // weight stream spreads over ~256 workgroups; partials summed by splitk_epilogue_kernel
    // (PZ_SK64_SPLIT = 0 disables; no fused norm / GeGLU with a split)
    {
      const char* es = getenv("PZ_SK64_SPLIT");
      const int64_t nblk = (ncols + 15) / 16 * ((a->M + 63) / 64);
      const int64_t kch = a->K / 64;
      if (!(es && es[0] == '0') && !a->norm_w && !pl.geglu && a->workspace && nblk < 128 &&
          kch >= 16) {
        int64_t S = (256 + nblk - 1) / nblk;
        S = S < kch / 8 ? S : kch / 8;
        S = S < 8 ? S : 8;
        const char* esn = getenv("PZ_SK64_S");  // A/B override of the slice count (read per call)
        if (esn && atoi(esn) >= 2 && atoi(esn) <= 8 && atoi(esn) <= kch / 4) S = atoi(esn);
        const int64_t ldw = (a->N + 3) / 4 * 4;
        if (S >= 2 && S * a->M * ldw * 4 <= a->ws_bytes && PZ_ALIGNED(a->workspace, 16)) {
          const int64_t per = (kch + S - 1) / S;
          pl.splits = (int)((kch + per - 1) / per);
          pl.ksplit = per * 64;
          pl.ldw = ldw;
        }
      }
    }
    {  // A/B overrides (read per call): PZ_SK64_NC = 4|8|16 columns per block, PZ_SK64_W = 4|8 waves
      const char* e = getenv("PZ_SK64_NC");
      if (e && (atoi(e) == 4 || atoi(e) == 8 || atoi(e) == 16)) pl.skinny_nc = atoi(e);
      e = getenv("PZ_SK64_W");
      if (e && (atoi(e) == 4 || atoi(e) == 8)) pl.skinny_w = atoi(e);
    }
    pl.tiles_n = (ncols + pl.skinny_nc - 1) / pl.skinny_nc;
    return pl;
  }
  // GEMV path (M <= 8, K % 512 == 0: the B = 1..2 denoise rows): every CU streams its weight slice
  // (pz_gemv.hip); PZ_GEMV=0 falls back to the MFMA skinny kernel below
  if (pz_gemv_supported(a)) {
    pl.kind = PATH_GEMV;
    return pl;
  }
  // skinny path: few rows, weights streamed once (inference denoise / proprio rows)
  if (a->M <= 16 && pl.akc && pl.bkc && a->K % 32 == 0 && !a->c_fp32 && a->epilogue < PZ_EPI_DGELU) {
    const int64_t kch = a->K / 32;
    pl.kind = PATH_SKINNY;
    pl.skinny_w = kch >= 64 ? 16 : (kch >= 32 ? 8 : 4);
    // PZ_SKINNY_MINNC=8|4: fewer columns per block for narrow outputs until the blocks cover the CUs
    // (A/B runs; measured slower at B=1 -- 9.9 vs 8.8 us for the 1024-wide o/down projections -- so
    // every block takes 16 columns by default)
    const char* e = getenv("PZ_SKINNY_MINNC");
    const int min_nc = e ? atoi(e) : 16;
    pl.skinny_nc = 16;
    while (pl.skinny_nc > 4 && pl.skinny_nc / 2 >= min_nc &&
           a->batch * ((ncols + pl.skinny_nc - 1) / pl.skinny_nc) < device_cus())
      pl.skinny_nc /= 2;
    pl.tiles_n = (ncols + pl.skinny_nc - 1) / pl.skinny_nc;
    return pl;
  }
  const int64_t cw = pl.geglu ? BT / 2 : BT;
  if (plan_tall(pl, a, ncols)) return pl;
  // the row-slab kernel before the 256-tile kernels (action-expert gate|up at 320 rows); PZ_ROWS_FIRST=1 for
  // every shape it takes (A/B runs; read per call)
  {
    const char* ef = getenv("PZ_ROWS_FIRST");
    if ((pl.geglu || (ef && ef[0] == '1')) && plan_rows(pl, a, ncols)) return pl;
  }
  // rows from which the 256-tile kernels are tried: 256 for the GeGLU GEMM and long-K GEMMs (prefill
  // at B=1, 276 rows: 64 vs 78 us and 51 vs 56 us measured), 512 otherwise (narrow prefill GEMMs
  // are faster on 128-row tiles); PZ_GEMM_256_MINM overrides (A/B runs)
  const char* mm = getenv("PZ_GEMM_256_MINM");
  const int64_t min_m = mm ? atoll(mm) : ((pl.geglu || a->K >= 8192 || (a->batch > 1 && !pl.akc && !pl.bkc)) ? 256 : 512);
  // at most half a round of 256-tiles at short K (the action expert's 1024- and 1280-row GEMMs at micro-batch 256): the 128-tile
  // kernel (+ split-K) beats the 256-tile split tail, 22-37 vs 29-45 us per launch, except at K 8192
  // (tools/attn_gemm_ab.py, profiles/r05/attn_gemm_ab.log); PZ_GEMM_SMALL256=1 keeps the 256 path (A/B)
  const char* es2 = getenv("PZ_GEMM_SMALL256");
  const bool small_short = !pl.geglu && a->batch == 1 && a->M >= 1024 && a->K <= 4096 &&
                           ((a->M + BT - 1) / BT) * ((ncols + cw - 1) / cw) <= 128 && !(es2 && es2[0] == '1');
  // batched TN GEMMs with >= 256 x 256 outputs per batch entry (the joint attention's dK = dS^T Q and dV = P^T dO,
  // 288 x 256 per sample): the 256-tile kernel, two row tiles per sample, 173 vs 190-203 us (dV of the 5-row action
  // mixture 28.7 vs 40.6 us) against the 128-tile kernel (tools/attn_gemm_ab.py, profiles/r05/attn_gemm_ab_r5s.log)
  const bool batched_tn = a->batch > 1 && !pl.akc && !pl.bkc && a->M >= 256 && ncols >= 256;
  const char* mn = getenv("PZ_GEMM_256_MINN");  // A/B: output columns from which the 256-tile path is tried
  const int64_t min_n = mn ? atoll(mn) : (pl.geglu || batched_tn ? 256 : 512);
  if ((use_8phase() ? a->K % 8 == 0 : a->K % BK256 == 0) && a->M >= min_m && ncols >= min_n && !small_short) {
    const int64_t tm = (a->M + BT - 1) / BT, tn = (ncols + cw - 1) / cw;
    Plan cand = pl;
    cand.kind = PATH_256;
    cand.tiles_m = tm;
    cand.tiles_n = tn;
    if (use_8phase()) plan_tail(cand, a);
    // enough workgroups to fill the chip: whole tiles, or tiles split into K-pieces
    const int64_t units = cand.tail_s ? cand.dp_tiles + (tm * tn - cand.dp_tiles) * cand.tail_s : a->batch * tm * tn;
    const char* mu = getenv("PZ_GEMM_256_MINUNITS");  // A/B: workgroups the 256-tile path must reach
    if (units >= (mu ? atoll(mu) : 160)) return cand;
  }
  if (plan_rows(pl, a, ncols)) return pl;
  pl.kind = PATH_TILE;
  pl.tiles_m = (a->M + BM - 1) / BM;
  pl.tiles_n = (ncols + (pl.geglu ? BN / 2 : BN) - 1) / (pl.geglu ? BN / 2 : BN);
  pl.wm = pl.geglu ? 4 : 2;
  pl.tag = (pl.geglu && pl.akc && a->M >= 2048) ? 1 : 0;
  // split-K when one 128x128 tile per WG leaves most of the 256 CUs idle
  const int64_t tiles = pl.tiles_m * pl.tiles_n;
  const int64_t nk = (a->K + BK - 1) / BK;
  const char* esk = getenv("PZ_SPLITK");  // "0": whole-K tiles only (A/B; read per call)
  if (a->batch == 1 && a->workspace && tiles < 120 && nk >= 4 && !(esk && esk[0] == '0')) {
    int64_t S = (240 + tiles - 1) / tiles;
    S = S < 16 ? S : 16;
    S = S < nk / 2 ? S : nk / 2;
    if (S >= 2) {
      const int64_t ks = ((nk + S - 1) / S) * BK;
      const int64_t Se = (a->K + ks - 1) / ks;
      const int64_t ldw = pl.geglu ? 2 * a->geglu_inter : (a->N + 3) / 4 * 4;
      if (Se >= 2 && Se * a->M * ldw * 4 <= a->ws_bytes && PZ_ALIGNED(a->workspace, 16)) {
        pl.kind = PATH_SPLIT;
        pl.splits = (int)Se;
        pl.ksplit = ks;
        pl.ldw = ldw;
      }
    }
  }
  return pl;
}

const char* bstr(bool b) { return b ? "true" : "false"; }
}  // namespace

extern "C" const char* pz_gemm_kernel_name(const pz_gemm_args* a) {
  static thread_local char buf[160];
  if (!a) return "";
  pz_gemm_args a8;  // W8A8: the planner sees K / lda / ldb in code pairs, as in pz_gemm
  if (a->fp8_mode == 1) {
    a8 = *a;
    a8.K = a->K / 2;
    a8.lda = a->lda / 2;
    a8.ldb = a->ldb / 2;
    a = &a8;
  }
  const Plan pl = make_plan(a);
  switch (pl.kind) {
    case PATH_SKINNY:
      snprintf(buf, sizeof(buf), "gemm_skinny_kernel<%d, %d>", pl.skinny_w, pl.skinny_nc);
      break;
    case PATH_SKINNY64:
      snprintf(buf, sizeof(buf), "gemm_skinny64_kernel<%d, %d, %d, %s>%s", pl.skinny_w, pl.skinny_nc, pl.skinny_mb,
               bstr(a->fp8_mode == 2),
               pl.ksplit > 0 && (sk64_two_launch() || !sk64_fits(pl, a)) ? "+splitk_epilogue_kernel" : "");
      break;
    case PATH_GEMV:
      snprintf(buf, sizeof(buf), "gemv_kernel<M<=%d>", a->M <= 4 ? 4 : 8);
      break;
    case PATH_256:
      if (use_8phase() && pl.tail_s)
        snprintf(buf, sizeof(buf), "%s<%s, %s, %s, %s>+gemm8p_tail_epilogue(tail %lld x %d)",
                 use_khalf(pl.akc, pl.bkc, a->M, a->N, a->K) ? "gemm8k_kernel" : "gemm8p_kernel", bstr(pl.akc), bstr(pl.bkc), bstr(pl.geglu), bstr(a->K % 64 != 0),
                 (long long)(pl.tiles_m * pl.tiles_n - pl.dp_tiles), pl.tail_s);
      else if (use_8phase())
        snprintf(buf, sizeof(buf), "%s<%s, %s, %s, %s>", use_khalf(pl.akc, pl.bkc, a->M, a->N, a->K) ? "gemm8k_kernel" : "gemm8p_kernel",
                 bstr(pl.akc), bstr(pl.bkc), bstr(pl.geglu), bstr(a->K % 64 != 0));
      else
        snprintf(buf, sizeof(buf), "gemm256_kernel<%s, %s, %s, %d>", bstr(pl.akc), bstr(pl.bkc), bstr(pl.geglu),
                 BK256);
      break;
    case PATH_TILE:
      snprintf(buf, sizeof(buf), "gemm_kernel<%s, %s, %d, %d>", bstr(pl.akc), bstr(pl.bkc), pl.wm, pl.tag);
      break;
    case PATH_ROWS:
      if (pl.rows_f8 == 2)
        snprintf(buf, sizeof(buf), "gemm_rows_f8a_kernel<%d, %d, %d>", pl.rows_w, pl.rows_tmb, pl.rows_tnb);
      else
        snprintf(buf, sizeof(buf), "gemm_rows_kernel<%d, %d, %d, %s, %s>", pl.rows_w, pl.rows_tmb, pl.rows_tnb,
                 bstr(pl.geglu), bstr(pl.rows_f8 == 1));
      break;
    case PATH_TALL:
      snprintf(buf, sizeof(buf), "gemm_tall_kernel<%d, %d, %d, %d, %s, %s>%s", pl.tall_mi, pl.geglu ? 4 : 2,
               pl.geglu ? 32 : 64, pl.geglu ? 4 : 3, bstr(pl.geglu), bstr(pl.bkc),
               pl.splits > 1 ? "+splitk_epilogue_kernel" : "");
      break;
    case PATH_SPLIT:
      snprintf(buf, sizeof(buf), "gemm_kernel<%s, %s, %d, %d>+splitk_epilogue_kernel(S=%d)", bstr(pl.akc),
               bstr(pl.bkc), pl.wm, pl.tag, pl.splits);
      break;
  }
  return buf;
}

int pz_splitk_epi_launch(const GemmP& p, int S, hipStream_t st) {
  const int64_t work = p.M * ((p.N + 3) / 4);
  hipLaunchKernelGGL(splitk_epilogue_kernel, dim3((unsigned)((work + 255) / 256)), dim3(256), 0, st, p, S);
  PZ_CHECK_LAUNCH();
  return PZ_OK;
}

template <bool GEGLU>
static int launch8p_f8(const GemmP& p, hipStream_t st) {
  const int smem = 2 * P8_BUF;
  auto kern = p.K % 64 != 0 ? gemm8p_f8_kernel<GEGLU, true> : gemm8p_f8_kernel<GEGLU, false>;
  static bool attr_set[2] = {false, false};
  const int ix = p.K % 64 != 0;
  if (!attr_set[ix]) {
    hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, smem);
    attr_set[ix] = true;
  }
  const int T = p.tiles_m * p.tiles_n;
  const int units = p.tail_s ? p.dp_tiles + (T - p.dp_tiles) * p.tail_s : T;
  hipLaunchKernelGGL(kern, dim3(units, 1), dim3(NT2), smem, st, p);
  PZ_CHECK_LAUNCH();
  if (p.tail_s) {
    launch_tail<GEGLU>(p, T, st);
    PZ_CHECK_LAUNCH();
  }
  return PZ_OK;
}

template <int W, int NC>
static int launch_skinny_nc(const GemmP& p, int64_t tiles_n, int64_t batch, hipStream_t st) {
  hipLaunchKernelGGL((gemm_skinny_kernel<W, NC>), dim3((unsigned)tiles_n, (unsigned)batch), dim3(W * 64), 0, st, p);
  PZ_CHECK_LAUNCH();
  return PZ_OK;
}

template <int W>
static int launch_skinny(const GemmP& p, int nc, int64_t tiles_n, int64_t batch, hipStream_t st) {
  if (nc == 4) return launch_skinny_nc<W, 4>(p, tiles_n, batch, st);
  if (nc == 8) return launch_skinny_nc<W, 8>(p, tiles_n, batch, st);
  return launch_skinny_nc<W, 16>(p, tiles_n, batch, st);
}

template <bool AKC, bool BKC, int WM, int TAG>
static int launch_tile_any(GemmP& p, const Plan& pl, int64_t batch, hipStream_t st) {
  if (pl.kind != PATH_SPLIT) return launch_tile<AKC, BKC, WM, TAG>(p, batch, st);
  int rc = launch_tile<AKC, BKC, WM, TAG>(p, pl.splits, st);
  if (rc != PZ_OK) return rc;
  const int64_t ncols = pl.geglu ? p.geglu_I : p.N;
  const int64_t work = p.M * ((ncols + 3) / 4);
  hipLaunchKernelGGL(splitk_epilogue_kernel, dim3((unsigned)((work + 255) / 256)), dim3(256), 0, st, p,
                     pl.splits);
  PZ_CHECK_LAUNCH();
  return PZ_OK;
}

// main loop of the 256-tile kernels: k-half segments (gemm8k_kernel) when an operand is k-strided,
// region sections (gemm8p_kernel) when both are k-contiguous -- there the k-half images' 64-B row
// pieces cost more than the halved barrier count saves (measured on every Pi0 NT shape) -- and, since the
// two-section loop (round 5), for the micro-batch's NN dgrads (A k-contiguous, B k-strided; >= 16384 rows) with
// >= 4096 output columns or a reduction >= 4096: 2-4 % faster there, 2.5 % slower at 2048 x 2048
// (profiles/r05/nn_main_ab.log; smaller row counts not measured, left on the k-half kernel).  Micro-batch census:
// gate|up dgrad 128.5 vs 136.2 ms, down-proj DGEGLU dgrad 90.5 vs 94.1 ms, all GEMMs 854.6 vs 865.5 ms
// (profiles/r05/census_nn_routing_ab.log; -DPZ_NN_KHALF builds the old routing for that A/B).
// PZ_GEMM_MAIN=quad|khalf forces one (A/B runs; read per call).
static bool use_khalf(bool akc, bool bkc, int64_t m, int64_t n, int64_t k) {
  const char* e = getenv("PZ_GEMM_MAIN");
  if (e && strcmp(e, "quad") == 0) return false;
  if (e && strcmp(e, "khalf") == 0) return true;
#ifndef PZ_NN_KHALF
  if (akc && !bkc && m >= 16384 && (n >= 4096 || k >= 4096)) return false;
#endif
  return !(akc && bkc);
}

// split-tail merge; PZ_TAIL_PB = 4 | 8 partial pieces loaded per round (A/B; read per call)
template <bool GEGLU>
static void launch_tail(const GemmP& p, int T, hipStream_t st) {
  const char* e = getenv("PZ_TAIL_PB");
  if (e && atoi(e) == 4)
    hipLaunchKernelGGL((gemm8p_tail_epilogue<GEGLU, 4>), dim3((T - p.dp_tiles) * 16), dim3(NT2), 0, st, p);
  else
    hipLaunchKernelGGL((gemm8p_tail_epilogue<GEGLU, 8>), dim3((T - p.dp_tiles) * 16), dim3(NT2), 0, st, p);
}

template <bool AKC, bool BKC, bool GEGLU, bool KTAIL>
static int launch8p_k(const GemmP& p, int64_t batch, hipStream_t st) {
  const int smem = 2 * P8_BUF;  // 128 KiB
  const bool kh = use_khalf(AKC, BKC, p.M, p.N, p.K);
  auto kern = kh ? gemm8k_kernel<AKC, BKC, GEGLU, KTAIL> : gemm8p_kernel<AKC, BKC, GEGLU, KTAIL>;
  static bool attr_set[2] = {false, false};
  if (!attr_set[kh]) {
    hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, smem);
    attr_set[kh] = true;
  }
  const int T = p.tiles_m * p.tiles_n;
  const int units = p.tail_s ? p.dp_tiles + (T - p.dp_tiles) * p.tail_s : T;
  hipLaunchKernelGGL(kern, dim3(units, (unsigned)batch), dim3(NT2), smem, st, p);
  PZ_CHECK_LAUNCH();
  if (p.tail_s) {
    launch_tail<GEGLU>(p, T, st);
    PZ_CHECK_LAUNCH();
  }
  return PZ_OK;
}

template <bool AKC, bool BKC, bool GEGLU>
static int launch8p(const GemmP& p, int64_t batch, hipStream_t st) {
  if (p.K % 64 != 0) return launch8p_k<AKC, BKC, GEGLU, true>(p, batch, st);
  return launch8p_k<AKC, BKC, GEGLU, false>(p, batch, st);
}

// large-GEMM kernel: the 8-phase ping-pong (default) or the 2-stage 256 kernel (PZ_GEMM_BIG=2stage, A/B runs)
static bool use_8phase() {
  const char* e = getenv("PZ_GEMM_BIG");  // read per call: A/B runs flip it in-process
  return !(e && strcmp(e, "2stage") == 0);
}

extern "C" int pz_gemm(const pz_gemm_args* a, void* stream) {
  PZ_CHECK_ARG(a != nullptr, "pz_gemm: null args");
  PZ_CHECK_ARG(a->M > 0 && a->N > 0 && a->K > 0, "pz_gemm: bad dims M=%lld N=%lld K=%lld",
               (long long)a->M, (long long)a->N, (long long)a->K);
  PZ_CHECK_ARG(a->A && a->B && a->C, "pz_gemm: null operand");
  PZ_CHECK_ARG(a->batch >= 1 && a->batch_inner >= 1 && a->batch % a->batch_inner == 0,
               "pz_gemm: bad batch %lld/%lld", (long long)a->batch, (long long)a->batch_inner);
  PZ_CHECK_ARG(PZ_ALIGNED(a->A, 16) && PZ_ALIGNED(a->B, 16), "pz_gemm: A/B must be 16-byte aligned");
  PZ_CHECK_ARG(a->lda % 8 == 0 && a->ldb % 8 == 0, "pz_gemm: lda/ldb must be multiples of 8");
  PZ_CHECK_ARG(a->ldc % 4 == 0 && PZ_ALIGNED(a->C, 8), "pz_gemm: ldc %% 4 and C 8-byte alignment");
  PZ_CHECK_ARG(a->sA_outer % 8 == 0 && a->sA_inner % 8 == 0 && a->sB_outer % 8 == 0 &&
                   a->sB_inner % 8 == 0 && a->sC_outer % 4 == 0 && a->sC_inner % 4 == 0,
               "pz_gemm: batch strides must keep 16-byte alignment");
  if (a->a_kcontig) PZ_CHECK_ARG(a->K % 8 == 0, "pz_gemm: k-contiguous A needs K %% 8 == 0");
  else PZ_CHECK_ARG(a->M % 8 == 0, "pz_gemm: k-strided A needs M %% 8 == 0");
  if (a->b_kcontig) PZ_CHECK_ARG(a->K % 8 == 0, "pz_gemm: k-contiguous B needs K %% 8 == 0");
  else PZ_CHECK_ARG(a->N % 8 == 0, "pz_gemm: k-strided B needs N %% 8 == 0");
  const bool geglu = a->epilogue == PZ_EPI_GEGLU;
  if (geglu) {
    PZ_CHECK_ARG(a->b_kcontig && a->geglu_inter > 0 && a->N == 2 * a->geglu_inter && a->batch == 1 &&
                     !a->beta_accum && !a->resid && !a->bias && !a->c_fp32 && a->geglu_inter % 4 == 0,
                 "pz_gemm: GEGLU needs k-contiguous B = [gate; up] (N = 2I), no batch/bias/resid");
  }
  if (a->epilogue == PZ_EPI_GELU || a->epilogue == PZ_EPI_SILU)
    PZ_CHECK_ARG(a->batch == 1, "pz_gemm: activation epilogue is unbatched");
  PZ_CHECK_ARG(a->epilogue >= PZ_EPI_NONE && a->epilogue <= PZ_EPI_DGEGLU, "pz_gemm: unknown epilogue %d",
               (int)a->epilogue);
  PZ_CHECK_ARG(!(a->c_fp32 && a->beta_accum && a->resid), "pz_gemm: fp32 beta accumulation takes no resid");
  if (a->epilogue >= PZ_EPI_DGELU) {
    PZ_CHECK_ARG(a->batch == 1 && a->aux && !a->bias && !a->resid && !a->beta_accum && !a->c_fp32,
                 "pz_gemm: backward epilogues read aux, write bf16 C, unbatched, no bias/resid/beta");
    if (a->epilogue == PZ_EPI_DGEGLU)
      PZ_CHECK_ARG(a->geglu_inter == a->N && a->ldc >= 2 * a->N && a->ld_aux >= 2 * a->N,
                   "pz_gemm: DGEGLU needs N == geglu_inter and [*, 2I] aux / C rows");
  }
  if (a->aux) PZ_CHECK_ARG(a->ld_aux % 4 == 0 && PZ_ALIGNED(a->aux, 8), "pz_gemm: aux alignment");
  PZ_CHECK_ARG(a->ws_bytes >= 0, "pz_gemm: negative ws_bytes");
  PZ_CHECK_ARG(a->fp8_mode >= 0 && a->fp8_mode <= 2, "pz_gemm: fp8_mode %d", (int)a->fp8_mode);
  pz_gemm_args a8;  // fp8 W8A8: K / lda / ldb in code pairs for the planner and the kernel
  if (a->fp8_mode == 1) {
    PZ_CHECK_ARG(a->a_kcontig && a->b_kcontig && a->batch == 1 && !a->norm_w && a->epilogue <= PZ_EPI_SILU &&
                     a->K % 16 == 0 && a->lda % 16 == 0 && a->ldb % 16 == 0,
                 "pz_gemm: fp8 W8A8 needs k-contiguous A [M][K] and B [N][K] codes, batch 1, K / lda / ldb "
                 "%% 16 == 0, a forward epilogue and no fused norm");
    a8 = *a;
    a8.K = a->K / 2;
    a8.lda = a->lda / 2;
    a8.ldb = a->ldb / 2;
    a = &a8;
  }
  if (a->fp8_mode == 2) {
    PZ_CHECK_ARG(a->a_kcontig && a->b_kcontig && a->batch == 1 && a->K % 64 == 0 && !a->c_fp32 &&
                     a->epilogue < PZ_EPI_DGELU && a->ldb % 16 == 0,
                 "pz_gemm: fp8 weights with bf16 rows (W8A16) need k-contiguous A and B, batch 1, "
                 "K %% 64 == 0, ldb %% 16 == 0, bf16 C and a forward epilogue");
    PZ_CHECK_ARG(a->M <= 64 || make_plan(a).kind == PATH_ROWS,
                 "pz_gemm: W8A16 above 64 rows needs a row-slab shape (M <= 1024, K <= 2048, <= 4096 columns)");
  }

  GemmP p;
  memset(&p, 0, sizeof(p));
  p.A = (const bf16_t*)a->A;
  p.B = (const bf16_t*)a->B;
  p.C = a->C;
  p.bias = (const bf16_t*)a->bias;
  p.resid = (const bf16_t*)a->resid;
  p.aux = (bf16_t*)a->aux;
  p.M = a->M; p.N = a->N; p.K = a->K;
  p.lda = a->lda; p.ldb = a->ldb; p.ldc = a->ldc;
  p.ld_resid = a->ld_resid; p.ld_aux = a->ld_aux; p.geglu_I = a->geglu_inter;
  p.batch_inner = a->batch_inner;
  p.sAo = a->sA_outer; p.sAi = a->sA_inner;
  p.sBo = a->sB_outer; p.sBi = a->sB_inner;
  p.sCo = a->sC_outer; p.sCi = a->sC_inner;
  p.sRo = a->sR_outer; p.sRi = a->sR_inner;
  p.epi = a->epilogue;
  p.c_fp32 = a->c_fp32;
  p.beta = a->beta_accum;
  p.alpha = a->alpha;
  p.nw = (const bf16_t*)a->norm_w;
  p.neps = a->norm_eps;
  p.rs = a->fp8_mode == 1 ? a->a_row_scale : nullptr;
  {
    const char* e = getenv("PZ_GEMM_DBG");
    p.dbg = e ? atoi(e) : 0;
    e = getenv("PZ_GEMM_NT");
    p.nt_store = e ? atoi(e) : 0;
    e = getenv("PZ_GEMM_NT_AUX");
    p.nt_aux = p.nt_store || (e && atoi(e) != 0);
  }
  hipStream_t st = (hipStream_t)stream;

  const Plan pl = make_plan(a);
  {
    // 8-phase tile order (tile_coords): super-rows of 2 row tiles instead of 8 for the narrow long-K GEMMs (<= 8
    // column tiles, K >= 16384: the Gemma gate|up dgrad, down forward, down / gate|up wgrads) and the DGEGLU dgrad --
    // measured per shape at micro-batch 256 (profiles/r06/gemm_group_ab.txt: gate|up dgrad 125.8 -> 121.4 ms,
    // DGEGLU 83.7 -> 81.5, down fwd 62.2 -> 61.2, wgrad 127.9 -> 127.0); the GeGLU forward keeps 8 (139.9 vs 142.2).
    // PZ_GEMM_GROUP overrides (A/B; read per call).
    const char* e = getenv("PZ_GEMM_GROUP");
    if (e && atoi(e) >= 1 && atoi(e) <= 64) p.group = atoi(e);
    else p.group = (a->K >= 16384 && pl.tiles_n <= 8) || a->epilogue == PZ_EPI_DGEGLU ? 2 : 8;
  }
  if (pl.kind == PATH_GEMV) return pz_gemv_launch(a, st);
  if (a->norm_w)
    PZ_CHECK_ARG((pl.kind == PATH_SKINNY || pl.kind == PATH_SKINNY64) && PZ_ALIGNED(a->norm_w, 16),
                 "pz_gemm: fused RMSNorm needs the few-row paths (M <= 64, k-contiguous A/B, K %% 32 == 0 "
                 "(M <= 16) or K %% 64 == 0) and a 16-byte aligned weight");
  if (pl.kind == PATH_SKINNY64) {
    p.tiles_n = (int)pl.tiles_n;
    if (pl.ksplit > 0) {
      p.ws = (float*)a->workspace;
      p.ksplit = pl.ksplit;
      p.ldw = pl.ldw;
      // in-launch combine: S tile-private [64][nc] fp32 slabs per tile, bf16 C with a forward epilogue
      p.sk_tk = sk64_fits(pl, a) ? 0 : -1;
    }
    return pz_sk64_launch(p, pl.skinny_w, pl.skinny_nc, pl.skinny_mb, a->fp8_mode == 2, pl.tiles_n, st);
  }
  if (a->fp8_mode == 1 && pl.kind == PATH_ROWS) {  // W8A8 row slab
    p.tiles_m = (int)pl.tiles_m;
    p.tiles_n = (int)pl.tiles_n;
    PZ_CHECK_ARG(PZ_ALIGNED(a->A, 16) && PZ_ALIGNED(a->B, 16), "pz_gemm: W8A8 rows need 16-byte aligned codes");
    return pz_rows_launch(p, pl.rows_w, pl.rows_tnb, false, 2, st);
  }
  if (a->fp8_mode == 1) {
    p.tiles_m = (int)pl.tiles_m;
    p.tiles_n = (int)pl.tiles_n;
    PZ_CHECK_ARG(pl.tiles_m * pl.tiles_n < (1LL << 31), "pz_gemm: grid too large");
    if (pl.tail_s) {
      p.ws = (float*)a->workspace;
      p.dp_tiles = pl.dp_tiles;
      p.tail_s = pl.tail_s;
      p.tail_kt = pl.tail_kt;
    }
    return geglu ? launch8p_f8<true>(p, st) : launch8p_f8<false>(p, st);
  }
  if (pl.kind == PATH_SKINNY) {
    PZ_CHECK_ARG(a->batch < 65536, "pz_gemm: batch too large");
    if (pl.skinny_w == 16) return launch_skinny<16>(p, pl.skinny_nc, pl.tiles_n, a->batch, st);
    if (pl.skinny_w == 8) return launch_skinny<8>(p, pl.skinny_nc, pl.tiles_n, a->batch, st);
    return launch_skinny<4>(p, pl.skinny_nc, pl.tiles_n, a->batch, st);
  }
  p.tiles_m = (int)pl.tiles_m;
  p.tiles_n = (int)pl.tiles_n;
  PZ_CHECK_ARG(pl.tiles_m * pl.tiles_n < (1LL << 31) && a->batch < 65536, "pz_gemm: grid too large");
  if (pl.kind == PATH_ROWS)
    return pz_rows_launch(p, pl.rows_w, pl.rows_tnb, pl.geglu, pl.rows_f8, st);
  if (pl.kind == PATH_TALL) {
    if (pl.splits > 1) {
      p.ws = (float*)a->workspace;
      p.ksplit = pl.ksplit;
      p.ldw = pl.ldw;
    }
    return pz_tall_launch(p, pl.tall_mi, geglu, pl.bkc, pl.splits > 1 ? pl.splits : 1, st);
  }
  if (pl.kind == PATH_256 && use_8phase()) {
    if (pl.tail_s) {
      p.ws = (float*)a->workspace;
      p.dp_tiles = pl.dp_tiles;
      p.tail_s = pl.tail_s;
      p.tail_kt = pl.tail_kt;
    }
    if (geglu) {
      if (a->a_kcontig) return launch8p<true, true, true>(p, a->batch, st);
      return launch8p<false, true, true>(p, a->batch, st);
    }
    if (a->a_kcontig && a->b_kcontig) return launch8p<true, true, false>(p, a->batch, st);
    if (a->a_kcontig && !a->b_kcontig) return launch8p<true, false, false>(p, a->batch, st);
    if (!a->a_kcontig && a->b_kcontig) return launch8p<false, true, false>(p, a->batch, st);
    return launch8p<false, false, false>(p, a->batch, st);
  }
  if (pl.kind == PATH_256) {
    if (geglu) {
      if (a->a_kcontig) return launch256<true, true, true>(p, a->batch, st);
      return launch256<false, true, true>(p, a->batch, st);
    }
    if (a->a_kcontig && a->b_kcontig) return launch256<true, true, false>(p, a->batch, st);
    if (a->a_kcontig && !a->b_kcontig) return launch256<true, false, false>(p, a->batch, st);
    if (!a->a_kcontig && a->b_kcontig) return launch256<false, true, false>(p, a->batch, st);
    return launch256<false, false, false>(p, a->batch, st);
  }
  if (pl.kind == PATH_SPLIT) {
    p.ws = (float*)a->workspace;
    p.ksplit = pl.ksplit;
    p.ldw = pl.ldw;
  }
  if (geglu) {
    if (pl.tag) return launch_tile_any<true, true, 4, 1>(p, pl, a->batch, st);
    if (a->a_kcontig) return launch_tile_any<true, true, 4, 0>(p, pl, a->batch, st);
    return launch_tile_any<false, true, 4, 0>(p, pl, a->batch, st);
  }
  if (a->a_kcontig && a->b_kcontig) return launch_tile_any<true, true, 2, 0>(p, pl, a->batch, st);
  if (a->a_kcontig && !a->b_kcontig) return launch_tile_any<true, false, 2, 0>(p, pl, a->batch, st);
  if (!a->a_kcontig && a->b_kcontig) return launch_tile_any<false, true, 2, 0>(p, pl, a->batch, st);
  return launch_tile_any<false, false, 2, 0>(p, pl, a->batch, st);
}

// q|k|v projection + RoPE + joint Q / K / V scatter in one 8-phase GEMM launch (training / prefill rows:
// mixture.py:162-215 + utils.py:4-16 + joint_model.py:170-257).  PZ_ERR_UNSUPPORTED (no error text) when the
// shape does not take the 8-phase 256-tile kernel: the caller then runs pz_gemm + pz_qkv_rope_split.
extern "C" int pz_gemm_qkv_rope(const pz_qkv_rope_args* a, void* stream) {
  PZ_CHECK_ARG(a && a->x && a->W && a->pos && a->cs && a->k_out && a->v_out && a->M > 0 && a->K > 0,
               "gemm_qkv_rope: bad args");
  PZ_CHECK_ARG(a->nh >= 1 && a->N == (a->nh + 2) * a->hd && a->T > 0 && a->M % a->T == 0,
               "gemm_qkv_rope: N = (nh + 2) * hd, M %% T == 0");
  // head_dim 256 (one 256-column 8-phase tile / 16 skinny blocks per head) and Q written: otherwise not this
  // kernel (no error text)
  if (a->hd != BT || !a->q_out) return PZ_ERR_UNSUPPORTED;
  PZ_CHECK_ARG(PZ_ALIGNED(a->x, 16) && PZ_ALIGNED(a->W, 16) && a->ldx % 8 == 0 && a->ldw % 8 == 0 && a->K % 8 == 0 &&
                   PZ_ALIGNED(a->q_out, 16) && PZ_ALIGNED(a->k_out, 16) && PZ_ALIGNED(a->v_out, 16),
               "gemm_qkv_rope: 16-byte alignment");
  pz_gemm_args g;
  memset(&g, 0, sizeof(g));
  g.M = a->M; g.N = a->N; g.K = a->K;
  g.A = a->x; g.lda = a->ldx; g.a_kcontig = 1;
  g.B = a->W; g.ldb = a->ldw; g.b_kcontig = 1;
  g.C = a->q_out; g.ldc = a->N;
  g.batch = 1; g.batch_inner = 1;
  g.alpha = 1.f;
  g.norm_w = a->norm_w;
  g.norm_eps = a->norm_eps;
  if (a->w_fp8) {
    PZ_CHECK_ARG(a->ldw % 16 == 0, "gemm_qkv_rope: fp8 weights need ldw %% 16 == 0");
    g.fp8_mode = 2;
    g.alpha = a->w_scale;
  }
  const Plan pl = make_plan(&g);  // no workspace: whole tiles only (the tail merge has no RoPE epilogue)
  // few rows (16 < M <= 64: C5's 50-row denoise chunk): the skinny-64 kernel with the RoPE epilogue, the
  // Gemma RMSNorm optionally fused (mixture.py:162-215 + utils.py:4-16 in one launch)
  if (pl.kind == PATH_SKINNY64 && pl.ksplit == 0 && a->K % 64 == 0 && a->N % 256 == 0 && a->M <= 64 &&
      (!a->norm_w || PZ_ALIGNED(a->norm_w, 16))) {
    GemmP p;
    memset(&p, 0, sizeof(p));
    p.group = 8;
    p.A = (const bf16_t*)a->x;
    p.B = (const bf16_t*)a->W;
    p.C = a->q_out;
    p.M = a->M; p.N = a->N; p.K = a->K;
    p.lda = a->ldx; p.ldb = a->ldw; p.ldc = a->N;
    p.batch_inner = 1;
    p.alpha = a->w_fp8 ? a->w_scale : 1.f;
    p.nw = (const bf16_t*)a->norm_w;
    p.neps = a->norm_eps;
    p.rpos = a->pos;
    p.rcs = a->cs;
    p.rq = (bf16_t*)a->q_out;
    p.rk = (bf16_t*)a->k_out;
    p.rv = (bf16_t*)a->v_out;
    p.rT = a->T; p.rnh = a->nh; p.rLq = a->Lq; p.rqoff = a->qoff; p.rLk = a->Lk; p.rkoff = a->koff;
    return pz_sk64_launch(p, pl.skinny_w, 16, pl.skinny_mb, a->w_fp8 != 0, a->N / 16, (hipStream_t)stream);
  }
  if (a->norm_w || a->w_fp8 || !use_8phase() || pl.kind != PATH_256) return PZ_ERR_UNSUPPORTED;
  GemmP p;
  memset(&p, 0, sizeof(p));
  p.group = 8;
  p.A = (const bf16_t*)a->x;
  p.B = (const bf16_t*)a->W;
  p.C = a->q_out;
  p.M = a->M; p.N = a->N; p.K = a->K;
  p.lda = a->ldx; p.ldb = a->ldw; p.ldc = a->N;
  p.batch_inner = 1;
  p.alpha = 1.f;
  p.tiles_m = (int)pl.tiles_m;
  p.tiles_n = (int)pl.tiles_n;
  p.rpos = a->pos;
  p.rcs = a->cs;
  p.rq = (bf16_t*)a->q_out;
  p.rk = (bf16_t*)a->k_out;
  p.rv = (bf16_t*)a->v_out;
  p.rT = a->T; p.rnh = a->nh; p.rLq = a->Lq; p.rqoff = a->qoff; p.rLk = a->Lk; p.rkoff = a->koff;
  return launch8p<true, true, false>(p, 1, (hipStream_t)stream);
}

extern "C" int pz_gemm_small(const pz_small_gemm_args* a, void* stream) {
  PZ_CHECK_ARG(a && a->A && a->B && a->C && a->M > 0 && a->N > 0 && a->K > 0, "pz_gemm_small: bad args");
  if (a->N <= SMALL_NMAX && a->K >= 256 && a->K % 8 == 0 && a->sAk == 1 && a->sBk == 1 && a->sAm % 8 == 0 &&
      a->sBn % 8 == 0 && PZ_ALIGNED(a->A, 16) && PZ_ALIGNED(a->B, 16)) {
    hipLaunchKernelGGL(gemm_small_rowwave_kernel, dim3((unsigned)((a->M + 3) / 4)), dim3(256), 0,
                       (hipStream_t)stream, *a);
    PZ_CHECK_LAUNCH();
    return PZ_OK;
  }
  const int64_t total = a->M * a->N;
  hipLaunchKernelGGL(gemm_small_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, *a);
  PZ_CHECK_LAUNCH();
  return PZ_OK;
}
