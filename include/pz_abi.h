/*
 * pz_abi.h -- C ABI of the MI355X-native Pi0 hot path (libpizero_hip.so).
 *
 * Every entry point takes raw device pointers, int64 sizes/strides and a
 * hipStream_t passed as `void* stream`; it enqueues work on that stream only
 * (no device syncs, no hipMalloc/hipFree -> legal inside hipGraph capture) and
 * returns 0 (PZ_OK) or a PZ_ERR_* code; pz_last_error() then holds a
 * thread-local message.  All tensors are owned by the caller.  bf16 tensors
 * are raw 16-bit storage.  Nothing here knows about torch.
 *
 * The reference (shroglck/open-pi-zero) has no native code: each entry point
 * replaces the PyTorch/ATen ops at the cited reference sites (file:line in
 * the reference tree).
 */
#ifndef PZ_ABI_H
#define PZ_ABI_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PZ_ABI_VERSION 20

enum {
  PZ_OK = 0,
  PZ_ERR_INVALID_ARG = 1,
  PZ_ERR_LAUNCH = 2,
  PZ_ERR_UNSUPPORTED = 3,
};

/* GEMM epilogues */
enum {
  PZ_EPI_NONE = 0,  /* C = alpha*acc (+bias[n]) (+resid[m,n]) (+C if beta_accum)       */
  PZ_EPI_GELU = 1,  /* pre = alpha*acc + bias; aux = pre; C = gelu_tanh(pre) (+resid)   */
  PZ_EPI_GEGLU = 2, /* B = [gate; up] (N = 2I); aux = [g | u]; C[m,n] = gelu(g)*u        */
  PZ_EPI_SILU = 3,  /* pre = alpha*acc + bias; aux = pre; C = silu(pre)                  */
  /* backward epilogues (dgrad GEMM of the layer after the activation; aux is READ):            */
  PZ_EPI_DGELU = 4,  /* C = alpha*acc * gelu_tanh'(aux[m,n])   (aux = saved pre-activation)  */
  PZ_EPI_DSILU = 5,  /* C = alpha*acc * silu'(aux[m,n])                                       */
  PZ_EPI_DGEGLU = 6, /* N = I, aux = saved [g | u] ([M, 2I]); d = alpha*acc:                    */
                     /*   C[m,n] = d*u*gelu'(g), C[m,I+n] = d*gelu(g)  (C may alias aux)       */
};

/*
 * bf16 MFMA GEMM:  C[z](m,n) = epi(alpha * sum_k A[z](m,k) B[z](k,n))
 *   A(m,k) = A[m*lda + k] if a_kcontig else A[k*lda + m]
 *   B(k,n) = B[n*ldb + k] if b_kcontig else B[k*ldb + n]   (b_kcontig = nn.Linear weight)
 *   C(m,n) = C[m*ldc + n]  (bf16, or fp32 if c_fp32)
 *   batch z in [0,batch): operand offset = (z / batch_inner)*s_outer + (z % batch_inner)*s_inner
 * Replaces every nn.Linear / torch.matmul on the path: siglip.py:103-106,164,183-192,22-30;
 * mixture.py:162-218; paligemma/modules.py:86-95; joint_model.py:261,282; vla/modules.py:39-53.
 */
typedef struct pz_gemm_args {
  int64_t M, N, K;
  const void* A; int64_t lda; int32_t a_kcontig;
  const void* B; int64_t ldb; int32_t b_kcontig;
  void* C; int64_t ldc; int32_t c_fp32;
  int64_t batch, batch_inner;
  int64_t sA_outer, sA_inner, sB_outer, sB_inner, sC_outer, sC_inner, sR_outer, sR_inner;
  int32_t epilogue;
  float alpha;
  int32_t beta_accum;
  const void* bias;                   /* bf16 [N] or NULL */
  const void* resid; int64_t ld_resid; /* bf16, may alias C */
  void* aux; int64_t ld_aux;           /* bf16 saved pre-activations or NULL */
  int64_t geglu_inter;                 /* I for PZ_EPI_GEGLU / PZ_EPI_DGEGLU */
  /* optional fp32 scratch (caller-owned, 16-byte aligned): when a batch-1 GEMM has too few
   * output tiles to fill the chip (prefill at B=1) and ws_bytes allows, K is split over
   * workgroups into fp32 slabs and a second kernel sums them and applies the epilogue.
   * NULL / 0 disables the split.  Deterministic (no atomics). */
  void* workspace; int64_t ws_bytes;
  /* optional fused Gemma RMSNorm of the A rows (paligemma/modules.py:7-21): A is the raw x and
   * the product uses x*rsqrt(mean_k(x^2)+norm_eps)*(1+norm_w[k]) (norm_w bf16 [K]).  Only for
   * the few-row paths (M <= 16 with K % 32 == 0, or 16 < M <= 64 with K % 64 == 0; k-contiguous
   * A and B: inference denoise rows);
   * PZ_ERR_ARG otherwise.  NULL disables. */
  const void* norm_w; float norm_eps;
  /* fp8 operands (OCP e4m3fn codes, one byte each; K, lda, ldb count codes):
   *   0 = bf16 A and B;
   *   1 = W8A8: fp8 A [M][K] and B [N][K], both k-contiguous, batch 1, K / lda / ldb % 16 == 0,
   *       forward epilogues (none / GeGLU / GELU / SiLU, bias, resid), no fused norm; the product
   *       is alpha * a_row_scale[m] * sum_k A*B (alpha = the weight scale; a_row_scale fp32 [M]
   *       from pz_fp8_quant_rows, NULL = 1).  Runs the 256-tile 8-phase kernel at the fp8 MFMA rate;
   *   2 = W8A16: bf16 A rows (M <= 64, optional fused RMSNorm), fp8 B [N][K] expanded to bf16 in
   *       registers, product * alpha (= the weight scale); K % 64 == 0, ldb % 16 == 0. */
  int32_t fp8_mode; const float* a_row_scale;
} pz_gemm_args;
int pz_gemm(const pz_gemm_args* args, void* stream);
/* fp8 (OCP e4m3fn) quantisation for fp8_mode 1 / 2 (C5, BASELINE.json configs[4]):
 * pz_fp8_quant_rows: per row r of bf16 x [R, D] (ldx): s = max_k |x[r,k]| / 448 (1 for an all-zero
 *   row), q[r,k] = e4m3(x[r,k] / s) (round to nearest even), row_scale[r] = s.  D % 8 == 0, D <= 16384.
 * pz_fp8_quant_tensor: q[i] = e4m3(x[i] * inv_scale) for n bf16 elements (n % 8 == 0): weights, with
 *   the per-tensor scale max|W| / 448 from pz_fp8_absmax (PZ_ABSMAX_PARTS fp32 partial maxima). */
#define PZ_ABSMAX_PARTS 1024
/* V^T codes for pz_flash_fwd_f8: per-head-dim scales vs [Z][256] = max over the nk keys of |V[:, d]| / 448, codes
 * vt [Z][256][ldt] (k < nk; zero for nk <= k < ldt) from V bf16 rows [Z][.][256] (row stride ldv, sample stride
 * v_bstride).  Replaces nothing in the reference (it has no fp8 path; BASELINE.json configs[4] asks for fp8 attention). */
int pz_fp8_quant_vt(const void* v, int64_t ldv, int64_t v_bstride, int64_t Z, int64_t nk, void* vt, float* vs,
                    int64_t ldt, void* stream);
/* every operand of one pz_flash_fwd_f8 launch in one launch: Q rows q [nqr][256] -> qc / qs and key rows k [nkr][256]
 * -> kc / ks (per-row, as pz_fp8_quant_rows), V -> vt / vs (as pz_fp8_quant_vt) */
int pz_fp8_quant_attn(const void* q, int64_t nqr, const void* k, int64_t nkr, const void* v, int64_t ldv,
                      int64_t v_bstride, int64_t Z, int64_t nk, void* qc, float* qs, void* kc, float* ks, void* vt,
                      float* vs, int64_t ldt, void* stream);
/* fp8 inference: Gemma RMSNorm / LayerNorm whose bf16-rounded output rows are quantised to e4m3 codes q [R][ldq] with
 * per-row scales qscale [R] in the same pass (= pz_rmsnorm_fwd / pz_layernorm_fwd then pz_fp8_quant_rows) -- the A
 * operand of the next W8A8 GEMM (paligemma/modules.py:7-21, siglip.py:211,217) */
int pz_rmsnorm_fwd_f8(const void* x, int64_t ldx, const void* w, void* q, int64_t ldq, float* qscale, int64_t R,
                      int64_t D, float eps, void* stream);
int pz_layernorm_fwd_f8(const void* x, int64_t ldx, const void* w, const void* b, void* q, int64_t ldq, float* qscale,
                        int64_t R, int64_t D, float eps, void* stream);
int pz_fp8_quant_rows(const void* x, int64_t ldx, void* q, int64_t ldq, float* row_scale, int64_t R, int64_t D,
                      void* stream);
int pz_fp8_quant_tensor(const void* x, int64_t n, void* q, float inv_scale, void* stream);
int pz_fp8_absmax(const void* x, int64_t n, float* parts, void* stream);
/* name of the kernel pz_gemm would launch for args (profiling / bench labels); never fails */
const char* pz_gemm_kernel_name(const pz_gemm_args* args);

/* strided fp32-accumulate GEMM for the K=7 / N=7 linears (pizero.py:94-103, vla/modules.py:44):
 * C[m*ldc+n] (+)= alpha*sum_k A[m*sAm+k*sAk]*B[k*sBk+n*sBn] (+bias[n]); bf16 in/out */
typedef struct pz_small_gemm_args {
  int64_t M, N, K;
  const void* A; int64_t sAm, sAk;
  const void* B; int64_t sBk, sBn;
  void* C; int64_t ldc;
  const void* bias;
  float alpha;
  int32_t beta;
} pz_small_gemm_args;
int pz_gemm_small(const pz_small_gemm_args* args, void* stream);

/* Gemma RMSNorm y = x*rsqrt(mean(x^2)+eps)*(1+w), fp32 inside (paligemma/modules.py:7-21).
 * rstd (fp32 [R]) is saved for backward when non-NULL. */
int pz_rmsnorm_fwd(const void* x, int64_t ldx, const void* w, void* y, int64_t ldy, float* rstd,
                   int64_t R, int64_t D, float eps, void* stream);
/* dx = dres + d(rmsnorm)/dx . dy   (dres may alias dx, may be NULL);
 * dw_part fp32 [ceil(R/rows_per_part), D] partial column sums of dy*xhat (NULL: skip) */
int pz_rmsnorm_bwd(const void* dy, int64_t lddy, const void* x, int64_t ldx, const void* w,
                   const float* rstd, const void* dres, void* dx, int64_t lddx, float* dw_part,
                   int64_t R, int64_t D, void* stream);
/* LayerNorm with affine (siglip.py:211,217,290 -> nn.LayerNorm, fp32 under autocast) */
int pz_layernorm_fwd(const void* x, int64_t ldx, const void* w, const void* b, void* y, int64_t ldy,
                     float* mean, float* rstd, int64_t R, int64_t D, float eps, void* stream);
int pz_layernorm_bwd(const void* dy, int64_t lddy, const void* x, int64_t ldx, const void* w,
                     const float* mean, const float* rstd, const void* dres, void* dx, int64_t lddx,
                     float* dw_part, float* db_part, int64_t R, int64_t D, float* dx_part, void* stream);
/* rows_per_part used by the *_bwd partial sums */
int64_t pz_norm_rows_per_part(void);
/* out[n] (+)= sum_p part[p*D + n]  -> bf16 (parameter gradient of a norm weight/bias) */
int pz_reduce_parts(const float* part, int64_t P, int64_t D, void* out, int32_t beta, void* stream);
/* (ABI 15) several pz_reduce_parts in one launch (a SigLIP layer's LayerNorm weight / bias and Linear bias
 * gradients, reduced together once the layer's backward is done): segment i = (part [P][D] fp32, out [D] bf16,
 * beta), D % 4 == 0, 16-byte aligned partials, 8-byte aligned out; any number of segments (8 per launch) */
typedef struct pz_reduce_seg {
  const float* part; int64_t P, D; void* out; int32_t beta;
} pz_reduce_seg;
int pz_reduce_parts_multi(const pz_reduce_seg* segs, int32_t nseg, void* stream);
/* (ABI 15) pz_layernorm_bwd's dx_part (NULL ok): per-part column sums of the bf16 dx, [ceil(R / rows_per_part)][D]
 * fp32 -- reduce_parts of them is the bias gradient of the Linear whose output gradient dx is (SigLIP fc2 /
 * out_proj, siglip.py:183-192 / 103-106 autograd), without re-reading dx.
 * pz_act_bwd_colsum: dpre = dh * act'(pre) (pz_act_bwd, dpre may alias dh) and dbias (+)= the column sums of the
 * bf16 dpre (the fc1 bias gradient) through ws [ws_rows][N] fp32 partials, in one pass over dh / pre. */
int pz_act_bwd_colsum(const void* dh, int64_t lddh, const void* pre, int64_t ldpre, void* dpre, int64_t M, int64_t N,
                      int32_t act, float* ws, int64_t ws_rows, void* dbias, int32_t beta, void* stream);
/* bias gradient: out[n] (+)= sum_m X[m*ld + n] (bf16 X, fp32 workspace ws of >= 64*N floats) */
int pz_colsum(const void* X, int64_t ld, int64_t M, int64_t N, void* out, int32_t beta, float* ws,
              void* stream);
/* sum over a batch of [rows, D] slabs: out (+)= sum_b X[b*stride + r*D + d] (pos-emb grad, siglip.py:76) */
int pz_batch_sum(const void* X, int64_t B, int64_t stride, int64_t n, void* out, int32_t beta, void* stream);

/* RoPE table: cs[pos*D/2*2 ..] = (cos, sin)(pos * inv_freq[i]) fp32 (paligemma/modules.py:24-67) */
int pz_rope_table(float* cs, int64_t max_pos, int64_t head_dim, float theta, void* stream);
/* one mixture's fused QKV projection [B*T, (nh+2*nkv)*hd] -> joint Q [B, Lq, nh*hd] (rows qoff..),
 * joint K, V [B, Lk, nkv*hd] (rows koff..), RoPE applied to Q and K (utils.py:4-16,
 * joint_model.py:170-257: the cat over mixtures without repeat_kv).  q_out NULL -> skip Q. */
int pz_qkv_rope_split(const void* qkv, const int64_t* pos, const float* cs, void* q_out, void* k_out,
                      void* v_out, int64_t B, int64_t T, int64_t nh, int64_t nkv, int64_t hd,
                      int64_t Lq, int64_t qoff, int64_t Lk, int64_t koff, void* stream);
/* q|k|v projection of few rows (M <= 8) with the fused Gemma RMSNorm of x (norm_w NULL: none) and
 * RoPE + scatter as its epilogue (mixture.py:162-215, joint_model.py:170-257, utils.py:4-16): the
 * projection x[M, K] . W[N = (nh + 2) * hd, K]^T is rounded to bf16 like pz_gemm + pz_qkv_rope_split
 * would, then row r = b*T + t is rotated with the table cs at pos[r] and written to
 * q_out[b][qoff + t][nh*hd] (Lq rows per sample), k_out / v_out[b][koff + t][hd] (Lk rows).  One
 * launch for the denoise step's q|k|v (pizero.py:461-481), K % 512 == 0. */
typedef struct pz_qkv_rope_args {
  const void* x; int64_t ldx;
  const void* W; int64_t ldw;
  int64_t M, N, K;
  const void* norm_w; float norm_eps;
  const int64_t* pos; const float* cs;
  void* q_out; void* k_out; void* v_out;
  int64_t T, nh, hd, Lq, qoff, Lk, koff;
  /* (ABI 15) w_fp8 = 1: W holds OCP e4m3 codes [N][K] (ldw in codes) with the per-tensor scale w_scale (the fp8
   * inference weights of C5); pz_gemm_qkv_rope's few-row path only (W8A16), 0 everywhere else */
  int32_t w_fp8; float w_scale;
} pz_qkv_rope_args;
int pz_gemv_qkv_rope(const pz_qkv_rope_args* a, void* stream);
/* The same fused projection + RoPE + scatter for MANY rows (training / prefill, mixture.py:162-215,
 * utils.py:4-16, joint_model.py:170-257): one 8-phase 256-tile MFMA GEMM whose epilogue rounds each head's
 * projection to bf16, rotates Q / K and writes Q / K / V straight into the joint buffers (no [M, N] qkv
 * tensor, no pz_qkv_rope_split launch; bit-identical to that pair).  hd = 256, q_out required.  16 < M <= 64
 * rows (C5's 50-row denoise chunk) take the skinny-64 MFMA kernel with the same epilogue and an optional fused
 * Gemma RMSNorm (norm_w); the 8-phase path takes norm_w NULL.  Returns PZ_ERR_UNSUPPORTED when the shape takes
 * neither kernel: the caller runs pz_gemm + pz_qkv_rope_split instead.  (ABI 14; few-row path ABI 15) */
int pz_gemm_qkv_rope(const pz_qkv_rope_args* a, void* stream);
/* backward of the above: writes d(qkv) (un-rotates dQ/dK, copies dV).  dq NULL -> zero dQ part */
int pz_qkv_rope_split_bwd(const void* dq, const void* dk, const void* dv, const int64_t* pos,
                          const float* cs, void* dqkv, int64_t B, int64_t T, int64_t nh, int64_t nkv,
                          int64_t hd, int64_t Lq, int64_t qoff, int64_t Lk, int64_t koff, void* stream);

/* attention softmax over rows of S (fp32) -> P (bf16, zero padded to ldp):
 * logits = cap>0 ? cap*tanh(scale*s/cap) : scale*s; masked -> excluded (fully masked row ->
 * uniform, like finfo.min in joint_model.py:271 / pizero.py:291); fp32 softmax (joint_model.py:273).
 * mask_mode 0: none; 1: Pi0 block mask from per-sample prefix counts cnt[b] (pizero.py:271-306),
 * query row r -> token qoff + (r % rows_per_batch)/heads, batch r / rows_per_batch;
 * 2: general additive fp32 mask (joint_model.py:271 adds any [B,1,Lq,Lk] mask): logit += mask[b][qtok][j]
 * at mask + b*mask_bstride + (qtok - qoff)*ldm (finfo.min entries absorb the logit exactly as in the
 * reference; a row whose logits are all -inf is uniform).  tcap (bf16, NULL ok) saves tanh for backward. */
typedef struct pz_softmax_args {
  const float* S; int64_t lds;
  void* P; int64_t ldp;
  void* tcap;
  int64_t R, N;
  float scale, cap;
  int32_t mask_mode;
  int64_t rows_per_batch, heads, qoff;
  const int32_t* cnt; int64_t prefix, cond;
  const float* mask; int64_t ldm, mask_bstride;
} pz_softmax_args;
int pz_attn_softmax(const pz_softmax_args* a, void* stream);
/* dS = scale * (1 - t^2) * P * (dP - rowsum(P*dP)), bf16 out zero padded to ldp */
int pz_attn_softmax_bwd(const void* P, const float* dP, int64_t lddp, const void* tcap, void* dS,
                        int64_t ldp, int64_t R, int64_t N, float scale, float cap, void* stream);

/* Fused (flash) attention, the two Pi0 shapes (no L x L tensor in HBM; see csrc/pz_flash.hip):
 *   SigLIP (siglip.py:108-166): H = 16 heads x head_dim 72 per sample, no mask;
 *   joint (joint_model.py:130-304): H = 1, MQA with the 8 query heads stacked as rows
 *     (r = token*8 + head), one K/V head of 256, soft-cap + Pi0 block mask (pizero.py:271-306).
 * Unit z = b*H + h.  Q row r: q + b*q_bstride + h*q_hstride + r*ldq (K, V alike; dQ/dK/dV use the
 * q/k/v strides).  O / dO row r lives in the output group i with g_row0[i] <= r (< g_row0[i+1]):
 * g_o[i] + b*g_bstride[i] + (r - g_row0[i])*g_ld[i] + h*o_hstride (dO: g_do[i], same layout).
 * logits = cap*tanh(scale*q.k/cap) (cap 0: scale*q.k); mask_mode 1: token t = r / rows_per_token
 * sees keys per the Pi0 block mask of cnt[b] (pad rows t in [cnt, prefix) attend uniformly).
 * lse: fp32 [Z*H][nq] log-sum-exp per row (written by fwd, read by bwd).  delta: fp32 [Z*H][nq]
 * rowsum(dO*O) (written by pz_flash_bwd_prep).  Deterministic (no atomics). */
typedef struct pz_flash_args {
  int64_t Z, H, nq, nk, head_dim;
  const void* q; int64_t ldq, q_bstride, q_hstride;
  const void* k; int64_t ldk, k_bstride, k_hstride;
  const void* v; int64_t ldv, v_bstride, v_hstride;
  int32_t n_groups;
  int64_t g_row0[3];
  void* g_o[3];
  int64_t g_bstride[3], g_ld[3];
  int64_t o_hstride;
  float* lse;
  float scale, cap;
  int32_t mask_mode;
  const int32_t* cnt; int64_t prefix, cond, rows_per_token;
  /* backward */
  const void* g_do[3];
  float* delta;
  void* dq; void* dk; void* dv;
  /* optional fp32 scratch (16-byte aligned) for the query-split dK/dV partials; NULL: no split */
  float* ws; int64_t ws_bytes;
  /* mask token of query row r = (r + mask_row0) / rows_per_token (denoise steps: queries start at
   * the action tokens, pizero.py:461-481) */
  int64_t mask_row0;
} pz_flash_args;
int pz_flash_fwd(const pz_flash_args* a, void* stream);
/* Joint attention forward that also exports the softmax (head_dim 256, nk <= 320, mask mode 0/1;
 * joint_model.py:259-292, pizero.py:271-306): O as pz_flash_fwd (no lse), plus P[z][r][0..ldp) =
 * the bf16 row softmax and tcap[z][r][..] = tanh(scale*s/cap) (NULL: not stored) with exactly
 * pz_attn_softmax's conventions (fully masked rows uniform over the nk keys with tcap 0, zeros past
 * nk), so the GEMM-path backward (P / tcap consumers) runs unchanged.  Replaces the S GEMM +
 * pz_attn_softmax + P V GEMM of the reference's eager attention (joint_model.py:261-292). */
/* fp8 attention forward (C5 prefill; joint_model.py:259-292 with e4m3 operands): the shape, mask, soft-cap,
 * output groups and key-split workspace of *a (H == 1, head_dim 256; a->q / k / v are not read), Q codes qc [Z][nq][256]
 * with row scales qs [Z*nq] (pz_fp8_quant_rows), key codes kc [Z][krows][256] with row scales ks [Z*krows], V^T codes
 * vtc [Z][256][ldvt] with head-dim scales vs [Z][256] (pz_fp8_quant_vt; ldvt >= nk rounded up to 128).  S and P V on
 * the fp8 MFMA, P quantised as e4m3(256 p). */
int pz_flash_fwd_f8(const pz_flash_args* a, const void* qc, const float* qs, const void* kc, const float* ks,
                    int64_t krows, const void* vtc, const float* vs, int64_t ldvt, void* stream);
int pz_flash_fwd_probs(const pz_flash_args* a, void* P, void* tcap, int64_t ldp, void* stream);
/* Joint attention backward from the exported softmax (head_dim 256, nk <= 320): dS[z][r][0..ldp) =
 * P (dP - sum_j P dP) scale (1 - tcap^2) in bf16 with dP = dO V^T computed in registers (dO from the
 * g_do groups; a NULL group counts as dO = 0), zeros past nk -- pz_attn_softmax_bwd's output without
 * the fp32 dP tensor.  Replaces the dP GEMM + softmax backward of joint_model.py:261-292's autograd.
 * With a->dq set it also writes dQ = dS K (bf16 dS, K staged like V; the q strides address dQ). */
int pz_flash_bwd_ds(const pz_flash_args* a, const void* P, const void* tcap, void* dS, int64_t ldp, void* stream);
/* delta[z][r] = sum_d dO[r][d] * O[r][d] (fp32) */
int pz_flash_bwd_prep(const pz_flash_args* a, void* stream);
/* dQ and delta (query-parallel), then dK, dV (key-parallel over all query rows of the unit); overwrite */
int pz_flash_bwd(const pz_flash_args* a, void* stream);

/* Decode-shaped joint attention (denoise steps, pizero.py:461-481; joint_model.py:259-292): for each
 * sample b, the T query tokens x nh heads (T*nh <= 1024 rows, MQA) q[(b*Lq + qoff + t)*ldq + h*256 ..]
 * against the nk cached keys/values k/v[b*k_bstride + j*256 ..] (head_dim 256): logits
 * cap*tanh(scale*q.k/cap), the Pi0 block mask for joint query token qtok0 + t (prefix counts cnt[b],
 * prefix / cond sizes; NULL cnt: no mask), fp32 softmax, O[(b*T + t)*ldo + h*256 ..] bf16.  Two
 * launches: per (32-key chunk, 32-row tile) partial (m, l, O) into the fp32 workspace ws
 * (pz_decode_attn_ws_bytes(B, T*nh, nk)), then a fixed-order merge per row.  Deterministic. */
typedef struct pz_decode_attn_args {
  const void* q; int64_t ldq, Lq, qoff;
  const void* k; const void* v; int64_t k_bstride, v_bstride;
  void* o; int64_t ldo;
  int64_t B, nh, T, nk, head_dim;
  float scale, cap;
  const int32_t* cnt; int64_t prefix, cond, qtok0;
  float* ws; int64_t ws_bytes;
} pz_decode_attn_args;
int64_t pz_decode_attn_ws_bytes(int64_t B, int64_t rows, int64_t nk);
int pz_decode_attn(const pz_decode_attn_args* a, void* stream);

/* SigLIP patch embed im2col (siglip.py:42-48,69-74): pixels bf16 [B,3,H,W] -> cols bf16
 * [B*(H/ps)*(W/ps), ldc] with k = c*ps*ps + ky*ps + kx, zero pad k in [3*ps*ps, ldc) */
int pz_patchify(const void* pix, void* cols, int64_t B, int64_t H, int64_t W, int64_t ps, int64_t ldc,
                void* stream);
/* token embed + image merge (pizero.py:376-414) with the joint-model sqrt(hidden) scaling
 * (joint_model.py:348-355) folded in: out[b,i] = text ? table[id]*emb_scale : image ?
 * img[b,k]*img_scale : 0 */
int pz_embed_merge(const int64_t* ids, const void* table, int64_t vocab, const void* img, void* out,
                   int64_t B, int64_t P, int64_t D, int64_t n_img, int64_t image_token, int64_t pad_token,
                   float emb_scale, float img_scale, void* stream);  /* ids outside [0,vocab) -> zero row */
/* dimg[b,k] = dout[b,i]*img_scale for image tokens */
int pz_embed_merge_bwd(const int64_t* ids, const void* dout, void* dimg, int64_t B, int64_t P,
                       int64_t D, int64_t n_img, int64_t image_token, float img_scale, void* stream);

/* SinusoidalPosEmb (vla/modules.py:9-22) from fp32 t[B] -> bf16 [B, D].  mode 0: fp32 math (the fp32
 * oracle); mode 1: the reference's arithmetic in a bf16 model (bf16 arange, every op rounded to bf16) */
int pz_time_embed(const float* t, void* out, int64_t B, int64_t D, float max_period, int32_t mode,
                  void* stream);
/* out[b*H+h] = [temb[b], e1[b*H+h]] (vla/modules.py:46-51), bf16 */
/* (ABI 15) inference form of pz_time_embed + pz_concat_time: the embedding of sample r / H written into columns
 * [0, D) of row r of out (row stride ldo) for B * H rows -- the action encoder's concat input without the
 * separate time-embedding buffer and concat launch (the encoder's first Linear writes columns [D, 2D)) */
int pz_time_embed_rows(const float* t, void* out, int64_t ldo, int64_t B, int64_t H, int64_t D, float max_period,
                       int32_t mode, void* stream);
int pz_concat_time(const void* temb, const void* e1, void* out, int64_t B, int64_t H, int64_t D,
                   void* stream);
/* dtemb not needed (t is data); de1 = dcat[:, D:] */
int pz_split_time_grad(const void* dcat, void* de1, int64_t rows, int64_t D, void* stream);
/* psi_t (pizero.py:597-605): psi = (1-(1-s)t) x0 + t x1 -> bf16 */
int pz_flow_psi(const float* x0, const float* x1, const float* t, void* psi, int64_t B, int64_t HA,
                float sig_min, void* stream);
/* flow-matching MSE (pizero.py:660-661): loss = mean((v - (x1-(1-s)x0))^2) -> fp32 loss[0];
 * dv = grad_scale[0] * 2 (v-d)/numel (bf16). grad_scale is a device fp32 scalar (NULL = 1). */
int pz_flow_loss(const void* v, int64_t ldv, int64_t v_bstride, const float* x0, const float* x1, float* loss,
                 void* dv, const float* grad_scale, int64_t B, int64_t H, int64_t A, float sig_min, void* stream);
/* Euler step (pizero.py:479-481): a += dt*v ; t += dt.  v row (b,h) at v + b*v_bstride + h*ldv */
/* ABI 20 -- one denoise step's glue in two launches instead of six (inference; bit-identical to the separate
 * kernels): pz_action_in = bf16 cast of the fp32 action rows + the action encoder's first Linear (K = A) into
 * cat[:, D:2D] + the time embedding (pz_time_embed_rows) into cat[:, :D]; pz_action_out = the action expert's final
 * RMSNorm + the action decoder Linear (D -> A <= 8) + the Euler update action += dt v, t += dt (pz_euler_step).
 * pizero.py:461-481 with vla/modules.py:15-53 (ActionEncoder, SinusoidalPosEmb) and pizero.py:100-103 */
int pz_action_in(const float* action, int64_t A, const void* w1, const void* b1, const float* t, void* cat,
                 int64_t ldc, int64_t B, int64_t H, int64_t D, float max_period, int32_t mode, void* stream);
int pz_action_out(const void* x, int64_t ldx, const void* norm_w, float eps, const void* wd, const void* bd, int64_t D,
                  int64_t A, float* action, float* t, int64_t B, int64_t H, float dt, void* stream);
int pz_euler_step(float* action, const void* v, int64_t ldv, int64_t v_bstride, float* t, int64_t B, int64_t H,
                  int64_t A, float dt, void* stream);
int pz_clamp(float* x, int64_t n, float lo, float hi, void* stream);

/* elementwise backward of fused MLP epilogues (recompute activations, no extra saves) */
int pz_geglu_bwd(const void* dh, int64_t lddh, const void* gu, int64_t ldgu, void* dgu, void* h_out,
                 int64_t ldh, int64_t M, int64_t I, void* stream);
int pz_act_bwd(const void* dh, int64_t lddh, const void* pre, int64_t ldpre, void* dpre, void* h_out,
               int64_t ldh, int64_t M, int64_t N, int32_t act /* PZ_EPI_GELU | PZ_EPI_SILU */,
               void* stream);

/* flat fused AdamW over bf16 params (train.py:171-198; torch.optim.AdamW semantics),
 * fp32 moments, gradient pre-scaled by *gscale (device scalar: clip coefficient). */
int pz_adamw(void* p, const void* g, float* m, float* v, int64_t n, float lr, float beta1,
             float beta2, float eps, float wd, float bc1, float bc2, const float* gscale, void* stream);
/* sum of squares of bf16 g[0..n): writes exactly PZ_SUMSQ_PARTS fp32 partials to parts[] (no atomics) */
#define PZ_SUMSQ_PARTS 2048
int pz_sumsq(const void* g, int64_t n, float* parts, void* stream);
/* clip_grad_norm_ coefficient (train.py:371-374; torch.nn.utils.clip_grad_norm_):
 * norm = sqrt(sum of parts[0..nparts) in a fixed order), coef = min(1, max_norm/(norm+1e-6)) */
int pz_clip_coef(const float* parts, int64_t nparts, float* coef, float* norm_out, float max_norm,
                 void* stream);

/* Blockwise 8-bit AdamW (bnb.optim.AdamW8bit, train.py:171-175,194-198; restated in
 * oracle/adamw8bit.py) over one contiguous run of bf16 params p / grads g.  seg: nseg rows of 4 int64
 * {element offset in the run, numel, first 256-element block, fp32-state offset or -1}: rows with
 * -1 keep uint8 codes s1 (m, signed map qmap1) / s2 (v, unsigned map qmap2) indexed like p and one
 * fp32 absmax per block (absmax1/2[block]); the others keep fp32 m32/v32 (bnb min_8bit_size).
 * Per element: g *= gscale[0] (NULL: 1); m = b1*m + omb1*g; v = b2*v + omb2*g*g;
 * p += step * m / (sqrt(v) + epsc); p *= decay; requantise with the block's new absmax.  Host
 * precomputes omb = 1-b, step = -lr*sqrt(1-b2^t)/(1-b1^t), epsc = eps*sqrt(1-b2^t), decay = 1-lr*wd
 * (float32).  Every op rounded separately (bit-exact with the oracle).  Deterministic. */
typedef struct pz_adamw8_args {
  void* p; const void* g;
  uint8_t* s1; uint8_t* s2;
  float* absmax1; float* absmax2;
  float* m32; float* v32;
  const int64_t* seg;
  int64_t nseg, nblocks;
  const float* qmap1; const float* qmap2;
  float beta1, beta2, omb1, omb2, step, epsc, decay;
  const float* gscale;
} pz_adamw8_args;
int pz_adamw8bit(const pz_adamw8_args* a, void* stream);

/* deterministic counter-based fill (oracle/synth.py twin): x[i] = off + scale*u(seed, i) */
int pz_fill_uniform(void* x, int32_t out_fp32, int64_t n, uint64_t seed, float off, float scale,
                    void* stream);
/* strided row copy with scale: dst[b*dbs + r*dld + d] = scale*src[b*sbs + r*sld + d] (+ dst if beta)
 * (the sqrt(hidden) embedding scaling of joint_model.py:348-355 for proprio/action rows) */
int pz_copy_rows(const void* src, int64_t sld, int64_t sbs, void* dst, int64_t dld, int64_t dbs, int64_t B,
                 int64_t rows, int64_t D, float scale, int32_t beta, void* stream);
/* bf16 <-> fp32 copies / scaled adds */
int pz_cast_f32_bf16(const float* x, void* y, int64_t n, void* stream);
int pz_cast_bf16_f32(const void* x, float* y, int64_t n, void* stream);

/* test instrument: fill every CU's LDS with `word` (0xffffffff = NaN) on `stream`, so the next kernel's reads of
 * LDS it did not write return NaN (tests/test_train_loop_gpu.py; _lib.call runs it before every launch under
 * PZ_POISON_LDS=1).  Not on any product path. */
int pz_debug_poison_lds(uint32_t word, void* stream);
/* test instrument: `wgs` workgroups that each occupy a CU (96 KiB LDS) for `ticks` of the constant-rate wall clock
 * (hipDeviceAttributeWallClockRate kHz) -- stands in for RCCL kernels sharing the CUs (tools/contention_probe.py). */
int pz_debug_spin(int64_t wgs, int64_t ticks, void* stream);

const char* pz_last_error(void);
int pz_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* PZ_ABI_H */
