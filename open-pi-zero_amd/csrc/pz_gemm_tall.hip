// Tall-tile GEMM: 64 < M <= 1024 rows against wide weights (own translation unit).
//
// Shapes: the B = 1 prefill's Gemma MLP at 276 rows (gate|up 276 x 32768 x 2048 + GeGLU, down
// 276 x 2048 x 16384), SigLIP at 256 rows, C5's 788-row prefill (pizero.py:430-451 / paligemma
// modules.py:86-95 / siglip.py:100-107) -- k-contiguous A [M][K] and B [N][K] (nn.Linear forward).
// The 8-phase kernel tiles them as 256 x 256: M = 276 takes two row tiles, the second holding 20
// rows, so every CU runs a full 256 x 256 x K tile for ~half useful work.  Here ONE row tile covers
// all rows (TR = 64 * MI: 256 or 320), and the columns are split finely (TC = 64 plain, 64 output
// columns = 128 B rows for GeGLU) so the grid still fills the chip; the weights stream from HBM
// once (each weight row is read by one workgroup per row tile), the A rows are L2-resident and
// re-read by every column tile.  Narrow outputs (down / fc2) split K over blockIdx.y: raw fp32
// partials summed in fixed order by splitk_epilogue_kernel (deterministic).
//
// 8 waves as 4 (M) x 2 (N): wave (wr, wc) owns rows 16 MI wr .. + 16 MI, columns 16 NI wc ..
// (GeGLU: NI / 2 gate blocks and the matching up blocks); swapped-operand MFMA
// (mfma_f32_16x16x32_bf16(B, A)) so a lane holds 4 consecutive columns of one row for the shared
// epilogues.  Operands are streamed global -> LDS by LDS-DMA (global_load_lds 16 B per lane, 1 KiB
// per wave-instruction) into an NSTAGE ring of BKT-deep K-tiles with counted vmcnt waits (NSTAGE - 2
// K-tiles stay in flight behind the one being consumed) and one barrier per K-tile.  LDS images are
// [rows][BKT] with the 16-B chunks XOR-swizzled by row (conflict-free ds_read_b128); the swizzle is
// applied to each lane's global source because an LDS-DMA write is lane-linear.  A K tail
// (K % BKT != 0, K % 8 == 0) clamps its source chunks in bounds and zeroes the A fragments past K.
#include "pz_gemm_epi.h"

namespace {

__device__ __forceinline__ void tl_glds16(const bf16_t* src, char* lds_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds_base, 16, 0, 0);
}

template <int BKT>
__device__ __forceinline__ int tl_swz(int r) {
  return BKT == 64 ? ((r >> 1) & 7) : 3 * ((r >> 3) & 1);
}

#define TL_WAIT_VM(n) asm volatile("s_waitcnt vmcnt(" #n ")" ::: "memory")
__device__ __forceinline__ void tl_wait_vm(int n) {  // wave-uniform count -> immediate
  switch (n) {
    case 0: TL_WAIT_VM(0); break;
    case 1: TL_WAIT_VM(1); break;
    case 2: TL_WAIT_VM(2); break;
    case 3: TL_WAIT_VM(3); break;
    case 4: TL_WAIT_VM(4); break;
    case 5: TL_WAIT_VM(5); break;
    case 6: TL_WAIT_VM(6); break;
    case 7: TL_WAIT_VM(7); break;
    case 8: TL_WAIT_VM(8); break;
    case 9: TL_WAIT_VM(9); break;
    case 10: TL_WAIT_VM(10); break;
    case 11: TL_WAIT_VM(11); break;
    case 12: TL_WAIT_VM(12); break;
    case 13: TL_WAIT_VM(13); break;
    case 14: TL_WAIT_VM(14); break;
    case 15: TL_WAIT_VM(15); break;
    case 16: TL_WAIT_VM(16); break;
    case 17: TL_WAIT_VM(17); break;
    case 18: TL_WAIT_VM(18); break;
    case 19: TL_WAIT_VM(19); break;
    case 20: TL_WAIT_VM(20); break;
    case 21: TL_WAIT_VM(21); break;
    case 22: TL_WAIT_VM(22); break;
    case 23: TL_WAIT_VM(23); break;
    default: TL_WAIT_VM(24); break;
  }
}

// k-strided B image [BKT k][64 columns] (128-B k-rows) for ds_read_b64_tr_b16: the 8-B column unit u of k-row k
// sits at u ^ tl_swtr(k) -- conflict-free for the 32 lanes of a transposed read (8 k-rows x 4 units)
__device__ __forceinline__ int tl_swtr(int k) { return 4 * (((k >> 1) & 1) | (((k >> 3) & 1) << 1)); }

// transposed fragment (inline asm: the builtin makes hipcc drain vmcnt -- the in-flight LDS-DMA -- before every read;
// callers wait lgkmcnt(0) before the first use)
__device__ __forceinline__ bf16x8 tl_frag_tr(const char* img, int rb, int kk, int lane) {
  const int q = (lane & 15) >> 2, p = lane & 3;
  s16x8 out;
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int k = kk * 32 + 8 * (lane >> 4) + 4 * t + q;
    const unsigned a = (unsigned)(size_t)(const __attribute__((address_space(3))) char*)(img + k * 128 +
                                                                                         (((4 * rb + p) ^ tl_swtr(k)) << 3));
    s16x4 v;
    asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"(a));
    out[4 * t + 0] = v[0];
    out[4 * t + 1] = v[1];
    out[4 * t + 2] = v[2];
    out[4 * t + 3] = v[3];
  }
  return __builtin_bit_cast(bf16x8, out);
}

template <int MI, int NI, int BKT, int NSTAGE, bool GEGLU>
struct TallCfg {
  static constexpr int TR = 64 * MI;               // tile rows
  static constexpr int TCB = 32 * NI;              // B image rows (GeGLU: gate | up)
  static constexpr int TCO = GEGLU ? TCB / 2 : TCB;  // output columns per tile
  static constexpr int RB = BKT * 2;               // bytes per image row
  static constexpr int IMG_A = TR * RB, IMG_B = TCB * RB, STAGE = IMG_A + IMG_B;
  static constexpr int NA = IMG_A / 1024, NB = IMG_B / 1024;  // 1 KiB DMA instructions per K-tile
  static constexpr int NPW = (NA + NB + 7) / 8;                // per wave (the last one repeated to even out)
  static constexpr int SMEM = NSTAGE * STAGE;
  static_assert(IMG_A % 1024 == 0 && IMG_B % 1024 == 0, "whole DMA instructions");
  static_assert(SMEM <= 160 * 1024, "LDS");
  static_assert((NSTAGE - 2) * NPW <= 24, "vmcnt immediates");
};

// BKC = false: B k-strided [K][N] (nn.Linear dgrad dY . W), plain epilogues only (64-column image of 128-B k-rows)
template <int MI, int NI, int BKT, int NSTAGE, bool GEGLU, bool BKC = true>
__global__ void __launch_bounds__(512, 1) gemm_tall_kernel(GemmP p) {
  using C = TallCfg<MI, NI, BKT, NSTAGE, GEGLU>;
  static_assert(BKC || (!GEGLU && C::TCB == 64), "k-strided B: 64-column plain tiles");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = wave >> 1, wc = wave & 1;
  int tm, tn;
  tile_coords(blockIdx.x, gridDim.x, p.tiles_m, p.tiles_n, tm, tn);
  const int64_t m0 = (int64_t)tm * C::TR, n0 = (int64_t)tn * C::TCO;
  // split-K: K range [kbeg, kend) of this workgroup (kbeg a multiple of BKT)
  const bool split = p.ksplit > 0;
  const int64_t kbeg = split ? (int64_t)blockIdx.y * p.ksplit : 0;
  const int64_t kend = split ? min(p.K, kbeg + p.ksplit) : p.K;
  const int nk = (int)((kend - kbeg + BKT - 1) / BKT);
  const int krem = (int)(kend - kbeg - (int64_t)(nk - 1) * BKT);  // valid k of the last K-tile (8..BKT)
  constexpr int CPR = BKT / 8, RPI = 64 / CPR;  // 16-B chunks per image row, rows per DMA instruction

  // DMA sources: instruction i = wave + 8 s (s < NPW), clamped to the last one (a repeated identical write)
  const bf16_t* src[C::NPW];
  int dst[C::NPW], kl[C::NPW];
#pragma unroll
  for (int s = 0; s < C::NPW; ++s) {
    const int i = min(wave + 8 * s, C::NA + C::NB - 1);
    const bool isA = i < C::NA;
    const int j = isA ? i : i - C::NA;
    dst[s] = (isA ? 0 : C::IMG_A) + j * 1024;
    if (!BKC && !isA) {  // k-strided B: instruction j = k-rows 8j .. 8j + 7 of 128 B (8 columns per lane)
      const int k = 8 * j + (lane >> 3);
      const int lc = (lane & 7) ^ (tl_swtr(k) >> 1);
      const int64_t c = min(n0 + 8 * lc, p.N - 8);
      kl[s] = -1 - k;  // (marks a k-row source: the K tail clamps the row, not a chunk)
      src[s] = p.B + (kbeg + k) * p.ldb + c;
      continue;
    }
    const int r = RPI * j + lane / CPR;                // image row
    const int ch = (lane % CPR) ^ tl_swz<BKT>(r);      // logical 16-B chunk this lane fetches
    kl[s] = 8 * ch;
    int64_t grow;
    if (isA) {
      grow = min(m0 + r, p.M - 1);
    } else if (GEGLU) {  // rows [0, TCO) gate columns, [TCO, 2 TCO) the matching up columns
      const int64_t c = min(n0 + (r % C::TCO), p.geglu_I - 1);
      grow = r < C::TCO ? c : p.geglu_I + c;
    } else {
      grow = min(n0 + r, p.N - 1);
    }
    src[s] = (isA ? p.A + grow * p.lda : p.B + grow * p.ldb) + kbeg + kl[s];
  }
  auto issue = [&](int kt) {
    char* st = smem + (kt % NSTAGE) * C::STAGE;
    const bool last = kt == nk - 1 && krem < BKT;
#pragma unroll
    for (int s = 0; s < C::NPW; ++s) {
      const bf16_t* g;
      if (!BKC && kl[s] < 0) {  // k-strided B row k: past K it re-reads the last valid k-row (A side zeroed)
        const int k = -1 - kl[s];
        g = src[s] + (int64_t)kt * BKT * p.ldb;
        if (last && k >= krem) g -= (int64_t)(k - (krem - 1)) * p.ldb;
      } else {
        g = src[s] + (int64_t)kt * BKT;
        if (last && kl[s] >= krem) g -= kl[s] - (krem - 8);  // past K: an in-bounds chunk (A side zeroed below)
      }
      tl_glds16(g, st + dst[s]);
    }
  };
  auto frag = [&](const char* img, int rb, int kk) {  // rows 16 rb + (lane & 15), k = 32 kk + 8 (lane >> 4)
    const int r = rb * 16 + (lane & 15);
    const int ch = kk * 4 + (lane >> 4);
    return *reinterpret_cast<const bf16x8*>(img + r * C::RB + ((ch ^ tl_swz<BKT>(r)) << 4));
  };

  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // image row of wave column block j: plain 16 (NI wc + j); GeGLU gate j < NI/2 at 16 (NI/2 wc + j), up at +TCO
  auto brow = [&](int j) {
    if (GEGLU) return (j < NI / 2 ? 0 : C::TCO / 16) + (NI / 2) * wc + (j % (NI / 2));
    return NI * wc + j;
  };
  auto compute = [&](int kt) {
    const char* ia = smem + (kt % NSTAGE) * C::STAGE;
    const char* ib = ia + C::IMG_A;
    const bool last = kt == nk - 1 && krem < BKT;
#pragma unroll
    for (int kk = 0; kk < BKT / 32; ++kk) {
      bf16x8 bf[NI];
#pragma unroll
      for (int j = 0; j < NI; ++j) bf[j] = BKC ? frag(ib, brow(j), kk) : tl_frag_tr(ib, NI * wc + j, kk, lane);
      if (!BKC) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        bf16x8 af = frag(ia, wr * MI + i, kk);
        if (last && kk * 32 + 8 * (lane >> 4) >= krem) af = bf16x8{};
#pragma unroll
        for (int j = 0; j < NI; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j], af, acc[i][j], 0, 0, 0);
      }
    }
  };

  // prologue: NSTAGE - 1 K-tiles in flight, wait for the first
  const int pre = min(nk, NSTAGE - 1);
  for (int kt = 0; kt < pre; ++kt) issue(kt);
  tl_wait_vm((pre - 1) * C::NPW);
  __builtin_amdgcn_s_barrier();
  for (int kt = 0; kt < nk; ++kt) {
    const bool more = kt + NSTAGE - 1 < nk;
    if (more) issue(kt + NSTAGE - 1);  // into the slot of kt - 1 (every wave passed the barrier after it)
    compute(kt);
    // retire K-tile kt + 1: the tiles issued after it may stay in flight
    const int after = min(nk - 1, kt + NSTAGE - 1) - (kt + 1);
    tl_wait_vm(after > 0 ? after * C::NPW : 0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }

  if (split) {  // raw partial sums; GeGLU keeps the [gate | up] column layout (cols n, I + n)
    float* W = p.ws + (int64_t)blockIdx.y * p.M * p.ldw;
#pragma unroll
    for (int i = 0; i < MI; ++i) {
      const int64_t m = m0 + (wr * MI + i) * 16 + (lane & 15);
      if (m >= p.M) continue;
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        int64_t n;
        if (GEGLU) {
          const int64_t nl = n0 + ((NI / 2) * wc + (j % (NI / 2))) * 16 + 4 * (lane >> 4);
          if (nl >= p.geglu_I) continue;
          n = j < NI / 2 ? nl : p.geglu_I + nl;
        } else {
          n = n0 + (NI * wc + j) * 16 + 4 * (lane >> 4);
          if (n >= p.N) continue;
        }
        *reinterpret_cast<f32x4*>(W + m * p.ldw + n) = acc[i][j];
      }
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < MI; ++i) {
    const int64_t m = m0 + (wr * MI + i) * 16 + (lane & 15);
    if (GEGLU) {
#pragma unroll
      for (int j = 0; j < NI / 2; ++j)
        store_geglu4(p, 0, m, n0 + ((NI / 2) * wc + j) * 16 + 4 * (lane >> 4), acc[i][j], acc[i][j + NI / 2]);
    } else {
#pragma unroll
      for (int j = 0; j < NI; ++j) store_out4(p, 0, 0, m, n0 + (NI * wc + j) * 16 + 4 * (lane >> 4), acc[i][j]);
    }
  }
}

}  // namespace

template <int MI, int NI, int BKT, int NSTAGE, bool GEGLU, bool BKC = true>
static int launch_tall_k(const GemmP& p, int splits, hipStream_t st) {
  using C = TallCfg<MI, NI, BKT, NSTAGE, GEGLU>;
  auto kern = gemm_tall_kernel<MI, NI, BKT, NSTAGE, GEGLU, BKC>;
  static bool attr_set = false;
  if (!attr_set) {
    hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, C::SMEM);
    attr_set = true;
  }
  hipLaunchKernelGGL(kern, dim3((unsigned)(p.tiles_m * p.tiles_n), (unsigned)splits), dim3(512), C::SMEM, st, p);
  PZ_CHECK_LAUNCH();
  if (splits > 1) return pz_splitk_epi_launch(p, splits, st);
  return PZ_OK;
}

// plain: 64-column tiles, 64-deep K-tiles in a 3-slot ring; GeGLU: 64 output columns (128 B rows), 32-deep
// K-tiles in a 4-slot ring.  mi = 4 (256-row tiles) or 5 (320-row tiles).
// Only the plain k-contiguous form is planned by default; the GeGLU and k-strided-B (NN dgrad) forms measured
// slower on every Pi0 shape (profiles/r04/tall_bench.log) and are compiled only with -DPZ_TALL_AB (A/B builds).
int pz_tall_launch(const GemmP& p, int mi, bool geglu, bool bkc, int splits, hipStream_t st) {
#ifdef PZ_TALL_AB
  if (!bkc) return mi == 4 ? launch_tall_k<4, 2, 64, 3, false, false>(p, splits, st) : launch_tall_k<5, 2, 64, 3, false, false>(p, splits, st);
  if (geglu) return mi == 4 ? launch_tall_k<4, 4, 32, 4, true>(p, splits, st) : launch_tall_k<5, 4, 32, 4, true>(p, splits, st);
#else
  if (!bkc || geglu) return PZ_ERR_UNSUPPORTED;  // not planned (plan_tall)
#endif
  return mi == 4 ? launch_tall_k<4, 2, 64, 3, false>(p, splits, st) : launch_tall_k<5, 2, 64, 3, false>(p, splits, st);
}
