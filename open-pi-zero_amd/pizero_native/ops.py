"""Thin torch-tensor front-ends over the C ABI (pointer/size plumbing only).

Every function enqueues HIP kernels on torch's current stream; tensors are
owned by the caller (PyTorch caching allocator), nothing is allocated on the
native side, so every sequence of these calls is hipGraph-capturable.
"""

from __future__ import annotations

import ctypes as C

import torch

from ._lib import (
    PZ_EPI_DGEGLU,
    PZ_EPI_DGELU,
    PZ_EPI_DSILU,
    PZ_EPI_GEGLU,
    PZ_EPI_GELU,
    PZ_EPI_NONE,
    PZ_EPI_SILU,
    PZ_SUMSQ_PARTS,
    AdamW8Args,
    QkvRopeArgs,
    DecodeAttnArgs,
    FlashArgs,
    GemmArgs,
    SmallGemmArgs,
    NativeError,
    SoftmaxArgs,
    call,
    lib,
)

__all__ = ["PZ_EPI_NONE", "PZ_EPI_GELU", "PZ_EPI_GEGLU", "PZ_EPI_SILU", "PZ_EPI_DGELU", "PZ_EPI_DSILU", "PZ_EPI_DGEGLU"]

BF16 = torch.bfloat16


def _st():
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


def _p(t):
    return None if t is None else t.data_ptr()


_PROBE = None


def set_probe(pred):
    """Record (start, end) HIP events around every pz_gemm launch for which pred(M, N, K, epi, batch)
    is true, on the launch stream (bench.py measures the dominant kernel's duration live)."""
    global _PROBE
    _PROBE = None if pred is None else (pred, [])
    return None if _PROBE is None else _PROBE[1]


def gemm(M, N, K, A, lda, a_kc, B, ldb, b_kc, Cm, ldc, *, epi=PZ_EPI_NONE, alpha=1.0, beta=False,
         bias=None, resid=None, ld_resid=0, aux=None, ld_aux=0, geglu_inter=0, batch=1, batch_inner=1,
         sA=(0, 0), sB=(0, 0), sC=(0, 0), sR=(0, 0), norm=None):
    """Raw GEMM: see pz_gemm_args in include/pz_abi.h.  Element strides.  norm = (w, eps): fused
    Gemma RMSNorm of the A rows (few-row path only)."""
    if _PROBE is not None and _PROBE[0](M, N, K, epi, batch):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        _gemm(M, N, K, A, lda, a_kc, B, ldb, b_kc, Cm, ldc, epi, alpha, beta, bias, resid, ld_resid, aux, ld_aux,
              geglu_inter, batch, batch_inner, sA, sB, sC, sR, norm)
        e1.record()
        _PROBE[1].append((e0, e1))
        return
    _gemm(M, N, K, A, lda, a_kc, B, ldb, b_kc, Cm, ldc, epi, alpha, beta, bias, resid, ld_resid, aux, ld_aux,
          geglu_inter, batch, batch_inner, sA, sB, sC, sR, norm)


_WS_BYTES = 160 << 20  # split-K / split-tail fp32 partials (multi-round tails: up to 640 x 256 KiB)
_WS = {}


_WS_SLOT = [0]


class workspace_slot:
    """``with workspace_slot(1):`` -- GEMMs enqueued inside use their own split-K / split-tail scratch (the
    engine's second stream for the action-expert group runs GEMMs concurrently with the main stream's)."""

    def __init__(self, slot):
        self.slot, self.prev = slot, None

    def __enter__(self):
        self.prev = _WS_SLOT[0]
        _WS_SLOT[0] = self.slot

    def __exit__(self, *exc):
        _WS_SLOT[0] = self.prev


def workspace(device=None):
    """Per-device fp32 split-K scratch for pz_gemm (allocated once, before any graph capture
    reuses it; GEMMs are stream-ordered within a stream, so one buffer per stream slot is enough:
    slot 0 = the main stream, slot 1 = the engine's action-expert stream)."""
    dev = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    key = (dev, _WS_SLOT[0])
    ws = _WS.get(key)
    if ws is None:
        ws = torch.empty(_WS_BYTES // 4, dtype=torch.float32, device=dev)
        _WS[key] = ws
    return ws


def _args(M, N, K, A, lda, a_kc, B, ldb, b_kc, Cm, ldc, epi, alpha, beta, bias, resid, ld_resid, aux, ld_aux,
          geglu_inter, batch, batch_inner, sA, sB, sC, sR, ws=None, norm=None):
    a = GemmArgs()
    a.M, a.N, a.K = int(M), int(N), int(K)
    a.A, a.lda, a.a_kcontig = _p(A), int(lda), int(bool(a_kc))
    a.B, a.ldb, a.b_kcontig = _p(B), int(ldb), int(bool(b_kc))
    a.C, a.ldc, a.c_fp32 = _p(Cm), int(ldc), int(Cm.dtype == torch.float32)
    a.batch, a.batch_inner = int(batch), int(batch_inner)
    a.sA_outer, a.sA_inner = int(sA[0]), int(sA[1])
    a.sB_outer, a.sB_inner = int(sB[0]), int(sB[1])
    a.sC_outer, a.sC_inner = int(sC[0]), int(sC[1])
    a.sR_outer, a.sR_inner = int(sR[0]), int(sR[1])
    a.epilogue, a.alpha, a.beta_accum = int(epi), float(alpha), int(bool(beta))
    a.bias, a.resid, a.ld_resid = _p(bias), _p(resid), int(ld_resid)
    a.aux, a.ld_aux, a.geglu_inter = _p(aux), int(ld_aux), int(geglu_inter)
    if ws is not None:
        a.workspace, a.ws_bytes = ws.data_ptr(), ws.numel() * ws.element_size()
    if norm is not None:
        a.norm_w, a.norm_eps = _p(norm[0]), float(norm[1])
    return a


def _gemm(M, N, K, A, lda, a_kc, B, ldb, b_kc, Cm, ldc, epi, alpha, beta, bias, resid, ld_resid, aux, ld_aux,
          geglu_inter, batch, batch_inner, sA, sB, sC, sR, norm=None):
    ws = workspace(Cm.device) if batch == 1 else None
    a = _args(M, N, K, A, lda, a_kc, B, ldb, b_kc, Cm, ldc, epi, alpha, beta, bias, resid, ld_resid, aux, ld_aux,
              geglu_inter, batch, batch_inner, sA, sB, sC, sR, ws, norm)
    call("pz_gemm", C.byref(a), _st())


def gemm_kernel_name(M, N, K, *, a_kc=True, b_kc=True, epi=PZ_EPI_NONE, geglu_inter=0, batch=1, c_fp32=False,
                     workspace_bytes=_WS_BYTES, fp8_mode=0):
    """Name of the kernel pz_gemm dispatches for this problem (bench / profile labels; fp8_mode 1 = W8A8 with row
    scales, 2 = W8A16, K in codes)."""
    a = GemmArgs()
    a.M, a.N, a.K = int(M), int(N), int(K)
    a.a_kcontig, a.b_kcontig, a.c_fp32 = int(a_kc), int(b_kc), int(c_fp32)
    a.batch, a.batch_inner, a.epilogue, a.geglu_inter = int(batch), 1, int(epi), int(geglu_inter)
    a.workspace, a.ws_bytes = (256 if workspace_bytes else None), int(workspace_bytes)
    a.fp8_mode = int(fp8_mode)
    if fp8_mode == 1:
        a.a_row_scale, a.lda, a.ldb = 256, int(K), int(K)
    return lib().pz_gemm_kernel_name(C.byref(a)).decode()


def linear(x, W, out, *, bias=None, resid=None, epi=PZ_EPI_NONE, aux=None, alpha=1.0, beta=False, norm=None):
    """out[M,N] = epi(x[M,K] @ W[N,K]^T): nn.Linear forward (x, out may be row-strided 2-D views).
    norm = (w, eps): x is first Gemma-RMS-normalised inside the GEMM (M <= 16 rows only)."""
    M, K = x.shape
    N = W.shape[0]
    if epi == PZ_EPI_GEGLU:
        I = N // 2
        gemm(M, N, K, x, x.stride(0), True, W, W.stride(0), True, out, out.stride(0), epi=epi,
             aux=aux, ld_aux=0 if aux is None else aux.stride(0), geglu_inter=I, alpha=alpha, norm=norm)
        return out
    gemm(M, N, K, x, x.stride(0), True, W, W.stride(0), True, out, out.stride(0), epi=epi, alpha=alpha,
         beta=beta, bias=bias, resid=resid, ld_resid=0 if resid is None else resid.stride(0), aux=aux,
         ld_aux=0 if aux is None else aux.stride(0), norm=norm)
    return out


# ---------------------------------------------------------------- fp8 (C5) ----
ABSMAX_PARTS = 1024  # include/pz_abi.h PZ_ABSMAX_PARTS
E4M3_MAX = 448.0


def fp8_quant_rows(x, q, row_scale):
    """per-row fp8 e4m3 codes of bf16 x [R, D] (q uint8 [R, D], row_scale fp32 [R] = max|row| / 448)"""
    R, D = x.shape
    call("pz_fp8_quant_rows", _p(x), x.stride(0), _p(q), q.stride(0), _p(row_scale), R, D, _st())


def rmsnorm_f8(x, w, q, qscale, eps):
    """Gemma RMSNorm of x [R, D] straight to e4m3 codes q [R, D] + per-row scales (pz_rmsnorm_fwd_f8)"""
    R, D = x.shape
    call("pz_rmsnorm_fwd_f8", _p(x), x.stride(0), _p(w), _p(q), q.stride(0), _p(qscale), R, D, float(eps), _st())


def layernorm_f8(x, w, b, q, qscale, eps):
    """LayerNorm of x [R, D] straight to e4m3 codes q [R, D] + per-row scales (pz_layernorm_fwd_f8)"""
    R, D = x.shape
    call("pz_layernorm_fwd_f8", _p(x), x.stride(0), _p(w), _p(b), _p(q), q.stride(0), _p(qscale), R, D, float(eps),
         _st())


def fp8_quant_tensor(x, q, scale):
    """q = e4m3(x / scale) elementwise (weights; scale = max|x| / 448 from fp8_weight_scale)"""
    call("pz_fp8_quant_tensor", _p(x), x.numel(), _p(q), 1.0 / float(scale), _st())


def fp8_weight_scale(x):
    """per-tensor weight scale max|x| / 448 (load-time: pz_fp8_absmax partials, host max)"""
    parts = torch.empty(ABSMAX_PARTS, device=x.device, dtype=torch.float32)
    call("pz_fp8_absmax", _p(x), x.numel(), _p(parts), _st())
    m = float(parts.max().item())
    return m / E4M3_MAX if m > 0 else 1.0


def linear_fp8(x, Wq, w_scale, out, *, bias=None, resid=None, epi=PZ_EPI_NONE, aux=None, norm=None,
               x_scale=None):
    """out = epi(x @ W^T) with fp8 e4m3 weights Wq [N, K] (uint8 codes, per-tensor w_scale).
    x_scale None: x bf16 rows (W8A16, M <= 64: codes expanded to bf16 in registers; norm allowed);
    else x uint8 codes [M, K] with per-row scales x_scale (W8A8 on the fp8 MFMA, 256-tile kernel)."""
    M, K = x.shape
    N = Wq.shape[0]
    a = _args(M, N, K, x, x.stride(0), True, Wq, Wq.stride(0), True, out, out.stride(0), epi, w_scale, False, bias,
              resid, 0 if resid is None else resid.stride(0), aux, 0 if aux is None else aux.stride(0),
              N // 2 if epi == PZ_EPI_GEGLU else 0, 1, 1, (0, 0), (0, 0), (0, 0), (0, 0), workspace(out.device),
              norm)
    a.fp8_mode = 2 if x_scale is None else 1
    a.a_row_scale = _p(x_scale)
    call("pz_gemm", C.byref(a), _st())
    return out


def rows_w8a8_ok(M, K, ncols, epi=PZ_EPI_NONE):
    """both operands e4m3 above 64 rows on the W8A8 row-slab kernel (pz_gemm.hip make_plan: 64 < M <= 1024, K % 128
    == 0, K <= 2048, <= 4096 output columns, no GeGLU; PZ_ROWS_W8A8=0 disables: W8A16 as before)"""
    import os

    if os.environ.get("PZ_ROWS_W8A8") == "0":
        return False
    return 64 < M <= 1024 and K % 128 == 0 and K <= 2048 and ncols <= 4096 and epi != PZ_EPI_GEGLU


def rows_w8a16_ok(M, K, ncols):
    """e4m3 weights with bf16 rows above 64 rows: the row-slab kernel's shapes (pz_gemm.hip plan_rows: 64 < M <=
    PZ_ROWS_MAXM (1024), K % 64 == 0, K <= 2048, <= 4096 output columns; PZ_GEMM_ROWS=0 disables)"""
    import os

    if os.environ.get("PZ_GEMM_ROWS") == "0" or os.environ.get("PZ_ROWS_W8A16") == "0":
        return False
    maxm = int(os.environ.get("PZ_ROWS_MAXM", "1024"))
    return 64 < M <= maxm and K % 64 == 0 and (os.environ.get("PZ_GEMM_ROWS") == "1" or (K <= 2048 and ncols <= 4096))


def linear_dgrad(dy, W, dx, *, beta=False, resid=None, epi=PZ_EPI_NONE, aux=None):
    """dx[M,K] (+)= dy[M,N] @ W[N,K] (+ resid).

    Backward epilogues (aux read): PZ_EPI_DGELU / PZ_EPI_DSILU multiply by the activation
    derivative at the saved pre-activation aux[M,K]; PZ_EPI_DGEGLU takes aux = saved [g | u]
    ([M, 2K]) and writes d(gate|up) into dx[M, 2K] (dx may be aux itself)."""
    M, N = dy.shape
    K = W.shape[1]
    gemm(M, K, N, dy, dy.stride(0), True, W, W.stride(0), False, dx, dx.stride(0), beta=beta,
         resid=resid, ld_resid=0 if resid is None else resid.stride(0), epi=epi, aux=aux,
         ld_aux=0 if aux is None else aux.stride(0), geglu_inter=K if epi == PZ_EPI_DGEGLU else 0)
    return dx


def _split_k(M, N, K):
    """Split the token (reduction) dim when the output has too few 256x256 tiles to fill 256 CUs."""
    tiles = ((N + 255) // 256) * ((K + 255) // 256)
    if tiles >= 160 or M < 4096 or N < 512 or K < 512 or M % 8 == 0:
        return 1  # (M % 8 == 0: the 8-phase kernel splits K itself -- pz_gemm "split tail")
    best = 1
    for s in (2, 4, 8):  # fewest splits that reach ~1 wave of 256-thread... 240+ workgroups
        if M % (s * 64) == 0:
            best = s
            if tiles * s >= 240:
                break
    return best


def linear_wgrad(dy, x, dW, *, beta=False):
    """dW[N,K] (+)= dy[M,N]^T @ x[M,K]   (split-K over tokens into fp32 slabs when the output is small)."""
    M, N = dy.shape
    K = x.shape[1]
    S = _split_k(M, N, K) if dW.is_contiguous() else 1
    if S == 1:
        gemm(N, K, M, dy, dy.stride(0), False, x, x.stride(0), False, dW, dW.stride(0), beta=beta)
        return dW
    Mc = M // S
    slabs = torch.empty(S, N, K, device=dW.device, dtype=torch.float32)
    gemm(N, K, Mc, dy, dy.stride(0), False, x, x.stride(0), False, slabs, K, batch=S,
         sA=(Mc * dy.stride(0), 0), sB=(Mc * x.stride(0), 0), sC=(N * K, 0))
    reduce_parts(slabs.view(S, N * K), dW.view(-1), beta=beta)
    return dW


def small_linear(x, W, out, *, bias=None, beta=False):
    """out[M,N] = x[M,K] W[N,K]^T for tiny K or N (7-dim action/proprio)."""
    M, K = x.shape
    N = W.shape[0]
    a = SmallGemmArgs()
    a.M, a.N, a.K = M, N, K
    a.A, a.sAm, a.sAk = _p(x), x.stride(0), x.stride(1)
    a.B, a.sBk, a.sBn = _p(W), W.stride(1), W.stride(0)
    a.C, a.ldc, a.bias, a.alpha, a.beta = _p(out), out.stride(0), _p(bias), 1.0, int(beta)
    call("pz_gemm_small", C.byref(a), _st())
    return out


def small_gemm(M, N, K, A, sAm, sAk, B, sBk, sBn, out, ldc, *, beta=False, bias=None):
    a = SmallGemmArgs()
    a.M, a.N, a.K = M, N, K
    a.A, a.sAm, a.sAk = _p(A), sAm, sAk
    a.B, a.sBk, a.sBn = _p(B), sBk, sBn
    a.C, a.ldc, a.bias, a.alpha, a.beta = _p(out), ldc, _p(bias), 1.0, int(beta)
    call("pz_gemm_small", C.byref(a), _st())
    return out


def rmsnorm(x, w, y, rstd, eps):
    R, D = x.shape
    call("pz_rmsnorm_fwd", _p(x), x.stride(0), _p(w), _p(y), y.stride(0), _p(rstd), R, D, float(eps), _st())
    return y


def rmsnorm_bwd(dy, x, w, rstd, dx, dres=None, dw_part=None):
    R, D = x.shape
    call("pz_rmsnorm_bwd", _p(dy), dy.stride(0), _p(x), x.stride(0), _p(w), _p(rstd), _p(dres), _p(dx),
         dx.stride(0), _p(dw_part), R, D, _st())
    return dx


def layernorm(x, w, b, y, mean, rstd, eps):
    R, D = x.shape
    call("pz_layernorm_fwd", _p(x), x.stride(0), _p(w), _p(b), _p(y), y.stride(0), _p(mean), _p(rstd), R, D,
         float(eps), _st())
    return y


def layernorm_bwd(dy, x, w, mean, rstd, dx, dres=None, dw_part=None, db_part=None, dx_part=None):
    """dx_part: per-part column sums of the bf16 dx (reduce_parts -> the bias gradient of the Linear whose output
    gradient dx is)"""
    R, D = x.shape
    call("pz_layernorm_bwd", _p(dy), dy.stride(0), _p(x), x.stride(0), _p(w), _p(mean), _p(rstd), _p(dres),
         _p(dx), dx.stride(0), _p(dw_part), _p(db_part), R, D, _p(dx_part), _st())
    return dx


def act_bwd_colsum(dh, pre, dpre, act, ws, dbias, beta=False):
    """dpre = dh * act'(pre) (dpre may alias dh) and dbias (+)= colsum(dpre) in one pass; ws fp32 [rows >= 16, N]"""
    M, N = pre.shape
    call("pz_act_bwd_colsum", _p(dh), dh.stride(0), _p(pre), pre.stride(0), _p(dpre), M, N, int(act), _p(ws),
         ws.numel() // N, _p(dbias), int(beta), _st())
    return dpre


_RPP = None


def rows_per_part():
    global _RPP
    if _RPP is None:
        from ._lib import lib

        _RPP = int(lib().pz_norm_rows_per_part())
    return _RPP


def reduce_parts(part, out, beta=False):
    P, D = part.shape
    call("pz_reduce_parts", _p(part), P, D, _p(out), int(beta), _st())
    return out


def reduce_parts_multi(items, beta=False):
    """[(part [P, D] fp32, out [D] bf16)]: every out (+)= the column sums of its part, one launch"""
    from ._lib import ReduceSeg

    if not items:
        return
    segs = (ReduceSeg * len(items))()
    for s, (part, out) in zip(segs, items):
        s.part, s.P, s.D, s.out, s.beta = _p(part), part.shape[0], part.shape[1], _p(out), int(beta)
    call("pz_reduce_parts_multi", C.cast(segs, C.c_void_p), len(items), _st())


def colsum(X, out, ws, beta=False):
    M, N = X.shape
    call("pz_colsum", _p(X), X.stride(0), M, N, _p(out), int(beta), _p(ws), _st())
    return out


def batch_sum(X, B, stride, n, out, beta=False):
    call("pz_batch_sum", _p(X), B, stride, n, _p(out), int(beta), _st())
    return out


def rope_table(cs, max_pos, head_dim, theta):
    call("pz_rope_table", _p(cs), max_pos, head_dim, float(theta), _st())
    return cs


def qkv_rope_split(qkv, pos, cs, q_out, k_out, v_out, B, T, nh, nkv, hd, Lq, qoff, Lk, koff):
    call("pz_qkv_rope_split", _p(qkv), _p(pos), _p(cs), _p(q_out), _p(k_out), _p(v_out), B, T, nh, nkv, hd,
         Lq, qoff, Lk, koff, _st())


def qkv_rope_split_bwd(dq, dk, dv, pos, cs, dqkv, B, T, nh, nkv, hd, Lq, qoff, Lk, koff):
    call("pz_qkv_rope_split_bwd", _p(dq), _p(dk), _p(dv), _p(pos), _p(cs), _p(dqkv), B, T, nh, nkv, hd, Lq,
         qoff, Lk, koff, _st())


def gemv_qkv_rope(x, W, pos, cs, q_out, k_out, v_out, T, nh, hd, Lq, qoff, Lk, koff, norm=None):
    """Few-row q|k|v projection (+ fused RMSNorm) with RoPE and the Q / K / V scatter as its epilogue."""
    a = QkvRopeArgs()
    a.x, a.ldx = _p(x), x.stride(0)
    a.W, a.ldw = _p(W), W.stride(0)
    a.M, a.N, a.K = x.shape[0], W.shape[0], x.shape[1]
    if norm is not None:
        a.norm_w, a.norm_eps = _p(norm[0]), float(norm[1])
    a.pos, a.cs = _p(pos), _p(cs)
    a.q_out, a.k_out, a.v_out = _p(q_out), _p(k_out), _p(v_out)
    a.T, a.nh, a.hd, a.Lq, a.qoff, a.Lk, a.koff = T, nh, hd, Lq, qoff, Lk, koff
    call("pz_gemv_qkv_rope", C.byref(a), _st())


PZ_ERR_UNSUPPORTED = 3  # include/pz_abi.h


def gemm_qkv_rope(x, W, pos, cs, q_out, k_out, v_out, T, nh, hd, Lq, qoff, Lk, koff, norm=None, w_scale=None):
    """q|k|v projection with RoPE and the joint Q / K / V scatter fused into the GEMM's epilogue
    (pz_gemm_qkv_rope): the 8-phase kernel for many rows, the skinny-64 kernel for 16 < M <= 64 (norm = (w, eps):
    fused Gemma RMSNorm; w_scale: W is e4m3 codes, W8A16 -- few-row path only).  Returns False (nothing launched) when the shape takes neither --
    the caller then runs linear + qkv_rope_split (same bits)."""
    a = QkvRopeArgs()
    a.x, a.ldx = _p(x), x.stride(0)
    a.W, a.ldw = _p(W), W.stride(0)
    a.M, a.N, a.K = x.shape[0], W.shape[0], x.shape[1]
    if norm is not None:
        a.norm_w, a.norm_eps = _p(norm[0]), float(norm[1])
    if w_scale is not None:  # W = e4m3 codes (uint8 [N, K]) with a per-tensor scale: few-row W8A16 path
        a.w_fp8, a.w_scale = 1, float(w_scale)
    a.pos, a.cs = _p(pos), _p(cs)
    a.q_out, a.k_out, a.v_out = _p(q_out), _p(k_out), _p(v_out)
    a.T, a.nh, a.hd, a.Lq, a.qoff, a.Lk, a.koff = T, nh, hd, Lq, qoff, Lk, koff
    rc = lib().pz_gemm_qkv_rope(C.byref(a), _st())
    if rc == PZ_ERR_UNSUPPORTED:
        return False
    if rc != 0:
        raise NativeError(f"pz_gemm_qkv_rope failed (rc={rc}): {lib().pz_last_error().decode(errors='replace')}")
    return True


def decode_attn(q, Lq, qoff, k, v, o, B, nh, T, nk, scale, cap, cnt, prefix, cond, qtok0):
    """Few-query joint attention (denoise): q [B, Lq, nh*hd] rows qoff.., k/v [B, Lk, hd], o [B*T, nh*hd]."""
    a = DecodeAttnArgs()
    a.q, a.ldq, a.Lq, a.qoff = _p(q), q.shape[-1], Lq, qoff
    a.k, a.v = _p(k), _p(v)
    a.k_bstride, a.v_bstride = k.stride(0), v.stride(0)
    a.o, a.ldo = _p(o), o.stride(0)
    a.B, a.nh, a.T, a.nk, a.head_dim = B, nh, T, nk, k.shape[-1]
    a.scale, a.cap = float(scale), float(cap)
    a.cnt, a.prefix, a.cond, a.qtok0 = _p(cnt), prefix, cond, qtok0
    need = lib().pz_decode_attn_ws_bytes(B, T * nh, nk)
    ws = workspace(o.device)  # the GEMM split-K scratch: stream-ordered, not in use between kernels
    if ws.numel() * 4 < need:
        raise ValueError(f"decode_attn: {B} samples x {nk} keys need {need} B of workspace (> {ws.numel() * 4})")
    a.ws, a.ws_bytes = _p(ws), ws.numel() * 4
    call("pz_decode_attn", C.byref(a), _st())


def attn_softmax(S, lds, P, ldp, R, N, scale, cap=0.0, tcap=None, mask_mode=0, rows_per_batch=1, heads=1,
                 qoff=0, cnt=None, prefix=0, cond=0, mask=None, ldm=0, mask_bstride=0):
    a = SoftmaxArgs()
    a.S, a.lds, a.P, a.ldp, a.tcap = _p(S), lds, _p(P), ldp, _p(tcap)
    a.R, a.N, a.scale, a.cap, a.mask_mode = R, N, float(scale), float(cap), mask_mode
    a.rows_per_batch, a.heads, a.qoff = rows_per_batch, heads, qoff
    a.cnt, a.prefix, a.cond = _p(cnt), prefix, cond
    a.mask, a.ldm, a.mask_bstride = _p(mask), ldm, mask_bstride
    call("pz_attn_softmax", C.byref(a), _st())


def attn_softmax_bwd(P, dP, lddp, tcap, dS, ldp, R, N, scale, cap):
    call("pz_attn_softmax_bwd", _p(P), _p(dP), lddp, _p(tcap), _p(dS), ldp, R, N, float(scale), float(cap),
         _st())


def flash_args(Z, H, nq, nk, hd, q, q_strides, k, k_strides, v, v_strides, groups, o_hstride, lse, scale,
               cap=0.0, mask_mode=0, cnt=None, prefix=0, cond=0, rows_per_token=1, dgroups=None, delta=None,
               dq=None, dk=None, dv=None, mask_row0=0, key_split=False):
    """pz_flash_args (include/pz_abi.h).  *_strides = (ld, bstride, hstride) in elements; groups =
    [(row0, O tensor, bstride, ld), ...] (dgroups: the dO tensors of the same groups).  key_split:
    hand the forward the workspace so launches with few query blocks split the keys."""
    a = FlashArgs()
    a.Z, a.H, a.nq, a.nk, a.head_dim = int(Z), int(H), int(nq), int(nk), int(hd)
    a.q, (a.ldq, a.q_bstride, a.q_hstride) = _p(q), tuple(int(x) for x in q_strides)
    a.k, (a.ldk, a.k_bstride, a.k_hstride) = _p(k), tuple(int(x) for x in k_strides)
    a.v, (a.ldv, a.v_bstride, a.v_hstride) = _p(v), tuple(int(x) for x in v_strides)
    a.n_groups = len(groups)
    for i, (r0, o, bs, ld) in enumerate(groups):
        a.g_row0[i], a.g_o[i], a.g_bstride[i], a.g_ld[i] = int(r0), _p(o), int(bs), int(ld)
        if dgroups is not None:
            a.g_do[i] = _p(dgroups[i])
    a.o_hstride = int(o_hstride)
    a.lse = _p(lse)
    a.scale, a.cap, a.mask_mode = float(scale), float(cap), int(mask_mode)
    a.cnt, a.prefix, a.cond, a.rows_per_token = _p(cnt), int(prefix), int(cond), int(rows_per_token)
    a.mask_row0 = int(mask_row0)
    a.delta, a.dq, a.dk, a.dv = _p(delta), _p(dq), _p(dk), _p(dv)
    if dq is not None or key_split:  # fp32 scratch: dK/dV query-split / forward key-split partials
        ws = flash_workspace(q.device)
        a.ws, a.ws_bytes = ws.data_ptr(), ws.numel() * ws.element_size()
    return a


_FLASH_WS_BYTES = 320 << 20
_FLASH_WS = {}


def flash_workspace(device):
    """Per-device fp32 scratch of the fused attention backward (8 query splits x dK, dV of a
    64-sample micro-batch = 295 MB); allocated once, stream-ordered like the GEMM workspace."""
    dev = torch.device(device)
    ws = _FLASH_WS.get(dev)
    if ws is None:
        ws = torch.empty(_FLASH_WS_BYTES // 4, dtype=torch.float32, device=dev)
        _FLASH_WS[dev] = ws
    return ws


def flash_fwd(a):
    call("pz_flash_fwd", C.byref(a), _st())


def fp8_quant_vt(v, Z, nk, vt, vs):
    """V^T e4m3 codes vt [Z, 256, ldt] (zero past nk) and per-head-dim scales vs [Z, 256] of bf16 V [Z, rows, 256]"""
    call("pz_fp8_quant_vt", _p(v), v.stride(1), v.stride(0), Z, nk, _p(vt), _p(vs), vt.shape[2], _st())


def fp8_quant_attn(q, k, v, Z, nk, qc, qs, kc, ks, vt, vs):
    """pz_fp8_quant_attn: Q rows q [R, 256] and key rows k [Rk, 256] per row, V [Z, rows, 256] per head dim (V^T codes
    vt [Z, 256, ldt]) -- the operands of flash_fwd_f8 in one launch"""
    call("pz_fp8_quant_attn", _p(q), q.shape[0], _p(k), k.shape[0], _p(v), v.stride(1), v.stride(0), Z, nk, _p(qc),
         _p(qs), _p(kc), _p(ks), _p(vt), _p(vs), vt.shape[2], _st())


def flash_fwd_f8(a, qc, qs, kc, ks, krows, vt, vs):
    """fp8 attention forward (pz_flash_fwd_f8): shape / mask / outputs from the pz_flash_args a"""
    call("pz_flash_fwd_f8", C.byref(a), _p(qc), _p(qs), _p(kc), _p(ks), int(krows), _p(vt), _p(vs), vt.shape[2], _st())


def flash_bwd_ds(a, P, tcap, dS, ldp):
    """dS of the joint attention from the exported softmax P / tanh(cap) and dO (a.g_do groups);
    pz_flash_bwd_ds."""
    call("pz_flash_bwd_ds", C.byref(a), _p(P), _p(tcap), _p(dS), int(ldp), _st())


def flash_fwd_probs(a, P, tcap, ldp):
    """Joint fused forward that also stores the bf16 softmax P and tanh(cap) [Z, nq, ldp] (the
    GEMM-path backward's inputs); pz_flash_fwd_probs."""
    call("pz_flash_fwd_probs", C.byref(a), _p(P), _p(tcap), int(ldp), _st())


def flash_bwd(a):
    """dQ (+ delta = rowsum(dO * O)), then dK/dV (overwritten); a.delta is fp32 scratch [Z*H, nq]."""
    call("pz_flash_bwd", C.byref(a), _st())


def siglip_flash_args(qkv, O, lse, B, nh, hd, N, dO=None, delta=None, dqkv=None):
    """SigLIP attention in place on the fused q|k|v projection rows [B*N, 3*nh*hd]; O [B*N, nh*hd]."""
    W = qkv.stride(0)
    H = nh * hd
    strides = (W, N * W, hd)
    return flash_args(B, nh, N, N, hd, qkv, strides, qkv[:, H:], strides, qkv[:, 2 * H:], strides,
                      [(0, O, N * O.stride(0), O.stride(0))], hd, lse, hd ** -0.5,
                      dgroups=None if dO is None else [dO], delta=delta,
                      dq=dqkv, dk=None if dqkv is None else dqkv[:, H:], dv=None if dqkv is None else dqkv[:, 2 * H:])


def patchify(pix, cols, ps):
    B, _, H, W = pix.shape
    call("pz_patchify", _p(pix), _p(cols), B, H, W, ps, cols.stride(0), _st())


def embed_merge(ids, table, img, out, n_img, image_token, pad_token, emb_scale, img_scale):
    B, P = ids.shape
    D = table.shape[1]
    call("pz_embed_merge", _p(ids), _p(table), table.shape[0], _p(img), _p(out), B, P, D, n_img, image_token,
         pad_token,
         float(emb_scale), float(img_scale), _st())


def embed_merge_bwd(ids, dout, dimg, n_img, image_token, img_scale):
    B, P = ids.shape
    D = dout.shape[-1]
    call("pz_embed_merge_bwd", _p(ids), _p(dout), _p(dimg), B, P, D, n_img, image_token, float(img_scale),
         _st())


def time_embed(t, out, max_period, ref_bf16=False):
    B, D = out.shape
    call("pz_time_embed", _p(t), _p(out), B, D, float(max_period), int(bool(ref_bf16)), _st())


def time_embed_rows(t, out, H, max_period, ref_bf16=False):
    """time embedding of sample r // H into out[r, :] (a column slice of the concat input), B * H rows"""
    rows, D = out.shape
    call("pz_time_embed_rows", _p(t), _p(out), out.stride(0), rows // H, H, D, float(max_period), int(bool(ref_bf16)),
         _st())


def concat_time(temb, e1, out, B, H, D):
    call("pz_concat_time", _p(temb), _p(e1), _p(out), B, H, D, _st())


def split_time_grad(dcat, de1, rows, D):
    call("pz_split_time_grad", _p(dcat), _p(de1), rows, D, _st())


def flow_psi(x0, x1, t, psi, sig_min):
    B = x0.shape[0]
    call("pz_flow_psi", _p(x0), _p(x1), _p(t), _p(psi), B, x0[0].numel(), float(sig_min), _st())


def flow_loss(v, ldv, vbs, x0, x1, loss, dv, grad_scale, B, H, A, sig_min):
    call("pz_flow_loss", _p(v), ldv, vbs, _p(x0), _p(x1), _p(loss), _p(dv), _p(grad_scale), B, H, A,
         float(sig_min), _st())


def action_in(action, W1, b1, t, cat, B, H, D, max_period, ref_bf16=False):
    """cat[:, :D] = time embedding, cat[:, D:2D] = bf16(action) @ W1^T + b1 (one launch; inference)"""
    A = action.shape[-1]
    call("pz_action_in", _p(action), A, _p(W1), _p(b1), _p(t), _p(cat), cat.stride(0), B, H, D, float(max_period),
         int(bool(ref_bf16)), _st())


def action_out(x, norm_w, eps, Wd, bd, action, t, B, H, dt):
    """action += dt * (RMSNorm(x) @ Wd^T + bd) (bf16 v), t += dt: the denoise step's tail in one launch"""
    D = x.shape[1]
    call("pz_action_out", _p(x), x.stride(0), _p(norm_w), float(eps), _p(Wd), _p(bd), D, Wd.shape[0], _p(action),
         _p(t), B, H, float(dt), _st())


def euler_step(action, v, ldv, vbs, t, B, H, A, dt):
    call("pz_euler_step", _p(action), _p(v), ldv, vbs, _p(t), B, H, A, float(dt), _st())


def copy_rows(src, sld, sbs, dst, dld, dbs, B, rows, D, scale=1.0, beta=False):
    call("pz_copy_rows", _p(src), sld, sbs, _p(dst), dld, dbs, B, rows, D, float(scale), int(beta), _st())


def clamp_(x, lo, hi):
    call("pz_clamp", _p(x), x.numel(), float(lo), float(hi), _st())


def geglu_bwd(dh, gu, dgu, h_out, M, I):
    call("pz_geglu_bwd", _p(dh), dh.stride(0), _p(gu), gu.stride(0), _p(dgu), _p(h_out),
         0 if h_out is None else h_out.stride(0), M, I, _st())


def act_bwd(dh, pre, dpre, h_out, act):
    M, N = pre.shape
    call("pz_act_bwd", _p(dh), dh.stride(0), _p(pre), pre.stride(0), _p(dpre), _p(h_out),
         0 if h_out is None else h_out.stride(0), M, N, int(act), _st())


def adamw(p, g, m, v, lr, b1, b2, eps, wd, bc1, bc2, gscale=None):
    call("pz_adamw", _p(p), _p(g), _p(m), _p(v), p.numel(), float(lr), float(b1), float(b2), float(eps),
         float(wd), float(bc1), float(bc2), _p(gscale), _st())


def adamw8bit(run, g, qmap1, qmap2, lr, b1, b2, eps, wd, t, gscale=None):
    """One bnb-style 8-bit AdamW step over a contiguous run (optim.FusedAdamW._prepare_8bit layout).
    Host precomputes the float32 constants exactly as oracle/adamw8bit.py does."""
    import numpy as np

    f = np.float32
    c1 = f(1.0 - b1 ** t)
    c2 = f(np.sqrt(1.0 - b2 ** t))
    a = AdamW8Args()
    a.p, a.g = _p(run["flat"]), _p(g)
    a.s1, a.s2 = _p(run["s1"]), _p(run["s2"])
    a.absmax1, a.absmax2 = _p(run["absmax1"]), _p(run["absmax2"])
    a.m32, a.v32 = _p(run["m32"]), _p(run["v32"])
    a.seg, a.nseg, a.nblocks = _p(run["seg"]), run["nseg"], run["nblocks"]
    a.qmap1, a.qmap2 = _p(qmap1), _p(qmap2)
    a.beta1, a.beta2 = float(f(b1)), float(f(b2))
    a.omb1, a.omb2 = float(f(1.0 - b1)), float(f(1.0 - b2))
    a.step = float(f(f(-lr) * c2 / c1))
    a.epsc = float(f(f(eps) * c2))
    a.decay = float(f(1.0 - lr * wd)) if wd > 0 else 1.0
    a.gscale = _p(gscale)
    call("pz_adamw8bit", C.byref(a), _st())


def sumsq(g, parts):
    """writes PZ_SUMSQ_PARTS fp32 partial sums of g*g into parts[0:PZ_SUMSQ_PARTS]"""
    assert parts.dtype == torch.float32 and parts.numel() >= PZ_SUMSQ_PARTS
    call("pz_sumsq", _p(g), g.numel(), _p(parts), _st())


def clip_coef(parts, coef, norm_out, max_norm):
    """norm = sqrt(sum(parts)) (fixed order), coef = min(1, max_norm / (norm + 1e-6))"""
    call("pz_clip_coef", _p(parts), parts.numel(), _p(coef), _p(norm_out), float(max_norm), _st())


def fill_uniform(x, seed, off, scale):
    call("pz_fill_uniform", _p(x), int(x.dtype == torch.float32), x.numel(), C.c_uint64(seed & (2**64 - 1)),
         float(off), float(scale), _st())
    return x


def cast_to_bf16(x, y):
    call("pz_cast_f32_bf16", _p(x), _p(y), x.numel(), _st())


def debug_poison_lds(word=0xFFFFFFFF):
    """Test instrument: fill every CU's LDS with ``word`` (0xffffffff = NaN) on the current stream."""
    call("pz_debug_poison_lds", C.c_uint32(int(word) & 0xFFFFFFFF), _st())


def debug_spin(wgs, ticks):
    """Test instrument: ``wgs`` workgroups each holding a CU for ``ticks`` wall-clock ticks, on the current stream."""
    call("pz_debug_spin", int(wgs), int(ticks), _st())
