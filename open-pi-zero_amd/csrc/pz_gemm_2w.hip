// Two-resident-workgroup NT GEMM (own translation unit): the forward GEMMs whose epilogue the one-shot
// 8-phase kernel cannot overlap.
//
// The 8-phase kernel (pz_gemm.hip) holds 128 KiB of LDS, so a CU runs ONE 256 x 256 tile at a time and
// the tile's epilogue stores (bias / residual / GELU + saved pre-activation / GeGLU + saved g|u) run while
// its MFMAs idle: measured (tools/epi_probe.py) SigLIP fc1 + GELU 0.246 ms with stores vs 0.137 ms without,
// the Gemma gate|up + GeGLU 2.19 vs 1.69 ms.  Here a tile is 256 x 128 with 4 waves (2 x 2, 128 x 64
// outputs per wave, acc[8][4] as in the 8-phase kernel) and 72 KiB of LDS, so TWO workgroups share a CU
// (one wave of each per SIMD): while one runs its epilogue the other's MFMAs keep the SIMDs busy, and the
// hardware dispatcher hands the next tile to a freed slot at once.
//
// Main loop: k-contiguous A [M][K] and B [N][K] (nn.Linear forward), K % 32 == 0.  A 3-slot ring of
// 32-deep K-tiles (A image [256][32] 16 KiB + B image [128][32] 8 KiB) streamed global -> LDS by LDS-DMA
// (global_load_lds_dwordx4, 1 KiB per wave-instruction, 6 per wave per K-tile), two K-tiles in flight,
// one counted vmcnt + barrier per K-tile.  Images are [row][64 B] with 16-B chunk ch of row r at
// ch ^ (3 * ((r >> 3) & 1)) -- conflict-free ds_read_b128 fragments; the swizzle is applied to each
// lane's global source (an LDS-DMA write is lane-linear).  MFMA operands swapped (lane owns 4
// consecutive output columns of one row).  The k order of the accumulation is the 8-phase kernel's
// (32-wide MFMA steps in ascending k), so whole-tile results are bit-identical to it.
//
// Epilogue (interior tiles): alpha * acc (+ bias) rounded to bf16 into a 256 x 128 LDS image, then 16-B
// row-contiguous chunks: GELU / SiLU (+ saved pre-activation), residual, old C (beta) -- the arithmetic
// of the 8-phase kernel's staged epilogue; GeGLU: [h | g] image then [u].  Edge tiles: per-lane groups.
#include "pz_gemm_epi.h"

namespace {

constexpr int W2_TM = 256, W2_TN = 128, W2_BK = 32, W2_NT = 256;
constexpr int W2_AIMG = W2_TM * W2_BK * 2;  // 16 KiB
constexpr int W2_BIMG = W2_TN * W2_BK * 2;  // 8 KiB
constexpr int W2_SLOT = W2_AIMG + W2_BIMG;  // 24 KiB
constexpr int W2_NSLOT = 3;
constexpr int W2_LDS = W2_NSLOT * W2_SLOT;  // 72 KiB: two workgroups per CU

__device__ __forceinline__ int w2_swz(int r) { return 3 * ((r >> 3) & 1); }

__device__ __forceinline__ void w2_glds16(const bf16_t* src, char* lds_base) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                   (__attribute__((address_space(3))) void*)lds_base, 16, 0, 0);
}

// fragment: rows rb*16 + (lane & 15), k = 8 * (lane >> 4) + [0, 8) of the K-tile
__device__ __forceinline__ bf16x8 w2_frag(const char* img, int rb, int lane) {
  const int r = rb * 16 + (lane & 15);
  const int ch = lane >> 4;
  return *reinterpret_cast<const bf16x8*>(img + r * 64 + ((ch ^ w2_swz(r)) << 4));
}

// bf16 256 x 128 output image, 256-B rows, 16-B chunk index XOR-swizzled by row
__device__ __forceinline__ void w2_put(char* img, int row, int col, u32x2 v) {
  const int ch = col >> 3;
  *reinterpret_cast<u32x2*>(img + row * 256 + ((ch ^ (row & 15)) << 4) + ((col >> 2) & 1) * 8) = v;
}
__device__ __forceinline__ u32x4 w2_get(const char* img, int row, int ch) {
  return *reinterpret_cast<const u32x4*>(img + row * 256 + ((ch ^ (row & 15)) << 4));
}
__device__ __forceinline__ void w2_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
__device__ __forceinline__ void w2_unpack8(const u32x4& w, float (&o)[8]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    o[2 * i] = __uint_as_float(w[i] << 16);
    o[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}
__device__ __forceinline__ u32x4 w2_pack8(const float (&v)[8]) {
  return u32x4{pack2bf(v[0], v[1]), pack2bf(v[2], v[3]), pack2bf(v[4], v[5]), pack2bf(v[6], v[7])};
}

template <bool GEGLU>
__global__ void __launch_bounds__(W2_NT, 2) gemm2w_kernel(GemmP p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  if (p.dbg >= 2 && blockIdx.x < 512) {
    // measurement (PZ_GEMM_DBG = 2 + n): the first-round workgroup in the upper LDS slot of its CU
    // (HW_REG_LDS_ALLOC base != 0) waits n x s_sleep(127) so the two co-resident tiles run out of phase
    const unsigned la = __builtin_amdgcn_s_getreg((31 << 11) | 6);
    if (la & 0x1ff)
      for (int i = 0; i < p.dbg - 2; ++i) __builtin_amdgcn_s_sleep(127);
  }
  int tm, tn;
  tile_coords(blockIdx.x, gridDim.x, p.tiles_m, p.tiles_n, tm, tn);
  const int64_t m0 = (int64_t)tm * W2_TM;
  const int64_t n0 = GEGLU ? (int64_t)tn * (W2_TN / 2) : (int64_t)tn * W2_TN;
  const int t = threadIdx.x, lane = t & 63;
  const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
  const int wr = wave >> 1, wc = wave & 1;

  // DMA sources: wave w stages A rows 64w..64w+63 (4 instructions) and B rows 32w..32w+31 (2)
  const bf16_t* sa[4];
  const bf16_t* sb[2];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = (wave * 4 + i) * 16 + (lane >> 2);
    const int kc = (lane & 3) ^ w2_swz(r);
    int64_t g = m0 + r;
    g = g < p.M ? g : p.M - 1;  // rows past the edge: clamped (finite, never stored)
    sa[i] = p.A + g * p.lda + 8 * kc;
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r = (wave * 2 + i) * 16 + (lane >> 2);
    const int kc = (lane & 3) ^ w2_swz(r);
    int64_t g;
    if (GEGLU) {  // virtual column r: wave (r >> 6), up (r >> 5 & 1), column n0 + (r >> 6) * 32 + (r & 31)
      int64_t c = n0 + (r >> 6) * 32 + (r & 31);
      c = c < p.geglu_I ? c : p.geglu_I - 1;
      g = ((r >> 5) & 1) ? p.geglu_I + c : c;
    } else {
      g = n0 + r;
      g = g < p.N ? g : p.N - 1;
    }
    sb[i] = p.B + g * p.ldb + 8 * kc;
  }
  auto issue = [&](int kt) {
    char* slot = smem + (kt % W2_NSLOT) * W2_SLOT;
    const int64_t k0 = (int64_t)kt * W2_BK;
#pragma unroll
    for (int i = 0; i < 4; ++i) w2_glds16(sa[i] + k0, slot + (wave * 4 + i) * 1024);
#pragma unroll
    for (int i = 0; i < 2; ++i) w2_glds16(sb[i] + k0, slot + W2_AIMG + (wave * 2 + i) * 1024);
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nk = (int)(p.K / W2_BK);
  issue(0);
  if (nk > 1) {
    issue(1);
    asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  w2_sync();
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 2 < nk) issue(kt + 2);  // slot (kt + 2) % 3 = (kt - 1) % 3: its reads ended before the last barrier
    const char* a_img = smem + (kt % W2_NSLOT) * W2_SLOT;
    const char* b_img = a_img + W2_AIMG;
    bf16x8 bf[4], af[8];
#pragma unroll
    for (int j = 0; j < 4; ++j) bf[j] = w2_frag(b_img, wc * 4 + j, lane);
#pragma unroll
    for (int i = 0; i < 8; ++i) af[i] = w2_frag(a_img, wr * 8 + i, lane);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf[j], af[i], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    if (kt + 2 < nk) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");  // tile kt + 1 landed, kt + 2 in flight
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    w2_sync();
  }
  if (p.dbg == 1) return;  // measurement: main loop only

  const int g4 = 4 * (lane >> 4), rl = lane & 15;
  if (GEGLU) {
    if (m0 + W2_TM <= p.M && n0 + W2_TN / 2 <= p.geglu_I) {
      // pass 1: image columns 0..63 = h, 64..127 = g; pass 2: columns 0..63 = u
#pragma unroll
      for (int rb = 0; rb < 8; ++rb)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          float gg[4], hh[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            gg[r] = acc[rb][j][r] * p.alpha;
            hh[r] = gelu_tanh(gg[r]) * (acc[rb][2 + j][r] * p.alpha);
          }
          const int row = wr * 128 + rb * 16 + rl, col = wc * 32 + j * 16 + g4;
          w2_put(smem, row, col, u32x2{pack2bf(hh[0], hh[1]), pack2bf(hh[2], hh[3])});
          w2_put(smem, row, 64 + col, u32x2{pack2bf(gg[0], gg[1]), pack2bf(gg[2], gg[3])});
        }
      w2_sync();
      bf16_t* C = reinterpret_cast<bf16_t*>(p.C) + m0 * p.ldc + n0;
      bf16_t* X = p.aux ? p.aux + m0 * p.ld_aux + n0 : nullptr;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int c = t + i * W2_NT, row = c >> 4, ch = c & 15;
        const u32x4 v = w2_get(smem, row, ch);
        if (ch < 8) *reinterpret_cast<u32x4*>(C + row * p.ldc + ch * 8) = v;
        else if (X) *reinterpret_cast<u32x4*>(X + row * p.ld_aux + (ch - 8) * 8) = v;
      }
      if (!X) return;
      w2_sync();
#pragma unroll
      for (int rb = 0; rb < 8; ++rb)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          float uu[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) uu[r] = acc[rb][2 + j][r] * p.alpha;
          w2_put(smem, wr * 128 + rb * 16 + rl, wc * 32 + j * 16 + g4, u32x2{pack2bf(uu[0], uu[1]), pack2bf(uu[2], uu[3])});
        }
      w2_sync();
      X += p.geglu_I;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int c = t + i * W2_NT, row = c >> 3, ch = c & 7;
        *reinterpret_cast<u32x4*>(X + row * p.ld_aux + ch * 8) = w2_get(smem, row, ch);
      }
      return;
    }
#pragma unroll
    for (int rb = 0; rb < 8; ++rb) {
      const int64_t m = m0 + wr * 128 + rb * 16 + rl;
#pragma unroll
      for (int j = 0; j < 2; ++j) store_geglu4(p, 0, m, n0 + wc * 32 + j * 16 + g4, acc[rb][j], acc[rb][2 + j]);
    }
    return;
  }

  const int64_t nb = n0 + wc * 64 + g4;
  if (m0 + W2_TM <= p.M && n0 + W2_TN <= p.N) {
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
      float bias[4] = {0.f, 0.f, 0.f, 0.f};
      if (p.bias) unpack4(*reinterpret_cast<const u32x2*>(p.bias + nb + cb * 16), bias);
#pragma unroll
      for (int rb = 0; rb < 8; ++rb) {
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = acc[rb][cb][r] * p.alpha + bias[r];
        w2_put(smem, wr * 128 + rb * 16 + rl, wc * 64 + cb * 16 + g4, u32x2{pack2bf(v[0], v[1]), pack2bf(v[2], v[3])});
      }
    }
    w2_sync();
    bf16_t* C = reinterpret_cast<bf16_t*>(p.C) + m0 * p.ldc + n0;
    const bool act = p.epi == PZ_EPI_GELU || p.epi == PZ_EPI_SILU;
    const bool gelu = p.epi == PZ_EPI_GELU;
    if (!act && !p.resid && !p.beta) {  // plain (+ bias): copy the image out
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int c = t + i * W2_NT, row = c >> 4, ch = c & 15;
        *reinterpret_cast<u32x4*>(C + row * p.ldc + ch * 8) = w2_get(smem, row, ch);
      }
      return;
    }
    const bf16_t* X0 = p.beta ? C : nullptr;                                // old C
    const bf16_t* X1 = p.resid ? p.resid + m0 * p.ld_resid + n0 : nullptr;  // residual
    bf16_t* Aux = act && p.aux ? p.aux + m0 * p.ld_aux + n0 : nullptr;
#pragma unroll
    for (int half = 0; half < 4; ++half) {  // 4 batches of 4 chunks: a batch's side loads issued together
      u32x4 a0[4], a1[4], iv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c = t + (half * 4 + i) * W2_NT, row = c >> 4, ch = c & 15;
        iv[i] = w2_get(smem, row, ch);
        a0[i] = X0 ? *reinterpret_cast<const u32x4*>(X0 + row * p.ldc + ch * 8) : u32x4{0u, 0u, 0u, 0u};
        a1[i] = X1 ? *reinterpret_cast<const u32x4*>(X1 + row * p.ld_resid + ch * 8) : u32x4{0u, 0u, 0u, 0u};
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c = t + (half * 4 + i) * W2_NT, row = c >> 4, ch = c & 15;
        float v[8], x0[8], x1[8];
        w2_unpack8(iv[i], v);
        w2_unpack8(a0[i], x0);
        w2_unpack8(a1[i], x1);
        if (act) {
          if (Aux) *reinterpret_cast<u32x4*>(Aux + row * p.ld_aux + ch * 8) = iv[i];
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = gelu ? gelu_tanh(v[e]) : silu(v[e]);
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] += x1[e] + x0[e];  // resid, old C (zeros when absent)
        *reinterpret_cast<u32x4*>(C + row * p.ldc + ch * 8) = w2_pack8(v);
      }
    }
    return;
  }
  // edge tile: one runtime-general group store per (row block, column block)
#pragma unroll 1
  for (int g = 0; g < 32; ++g) {
    const int rb = g >> 2, cb = g & 3;
    f32x4 v = acc[0][0];
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (i == rb && j == cb) v = acc[i][j];
    store_out4_rt(p, 0, 0, m0 + wr * 128 + rb * 16 + rl, nb + cb * 16, v);
  }
}

template <bool GEGLU>
int launch2w(const GemmP& p, hipStream_t st) {
  auto kern = gemm2w_kernel<GEGLU>;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, W2_LDS);
    attr_set = true;
  }
  hipLaunchKernelGGL(kern, dim3((unsigned)(p.tiles_m * p.tiles_n)), dim3(W2_NT), W2_LDS, st, p);
  PZ_CHECK_LAUNCH();
  return PZ_OK;
}

}  // namespace

int pz_2w_launch(const GemmP& p, bool geglu, hipStream_t st) {
  return geglu ? launch2w<true>(p, st) : launch2w<false>(p, st);
}
