"""Per-kernel numerics on the MI355X vs a plain PyTorch fp32 reference of the same op.

Tolerances: bf16 inputs are identical on both sides; the HIP kernels
accumulate in fp32 and round the output once to bf16, so errors are bounded by
~1 bf16 ulp of the output (2^-8 relative) plus fp32 summation-order noise.
"""

import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

dev = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _native():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import pizero_native

    pizero_native.lib()
    torch.manual_seed(0)


def bf(*shape, scale=1.0):
    return (torch.randn(*shape, device=dev) * scale).to(torch.bfloat16)


def close(out, ref, rtol=1.6e-2, atol=1e-2):
    out, ref = out.float(), ref.float()
    err = (out - ref).abs()
    tol = atol + rtol * ref.abs()
    bad = (err > tol).sum().item()
    assert bad == 0, f"{bad} mismatches, max err {err.max().item():.4g}, max ref {ref.abs().max().item():.4g}"


@pytest.mark.parametrize("M,N,K", [(128, 128, 64), (300, 200, 136), (4416, 2560, 2048), (7, 36, 72), (1, 2048, 2048),
                                   (5, 1024, 4096), (276, 2560, 2048)])
def test_linear_forward(M, N, K):
    from pizero_native import ops

    x, W = bf(M, K), bf(N, K, scale=K ** -0.5)
    b = bf(N)
    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    ops.linear(x, W, out, bias=b)
    close(out, x.float() @ W.float().t() + b.float())


@pytest.mark.parametrize("M,N,K", [(256, 192, 128), (4416, 1152, 2048), (281, 256, 2248)])
def test_dgrad_and_wgrad_layouts(M, N, K):
    from pizero_native import ops

    dy, W, x = bf(M, N), bf(N, K, scale=N ** -0.5), bf(M, K)
    dx = torch.empty(M, K, device=dev, dtype=torch.bfloat16)
    ops.linear_dgrad(dy, W, dx)
    close(dx, dy.float() @ W.float())
    dW = torch.empty(N, K, device=dev, dtype=torch.bfloat16)
    ops.linear_wgrad(dy, x, dW)
    close(dW, dy.float().t() @ x.float(), atol=0.05 * math.sqrt(M) / 16)
    dW2 = dW.clone()
    ops.linear_wgrad(dy, x, dW2, beta=True)
    close(dW2, 2 * (dy.float().t() @ x.float()), atol=0.1 * math.sqrt(M) / 16)


def test_all_four_layouts_batched_fp32_out():
    from pizero_native import ops

    Bt, M, N, K = 3, 96, 80, 104
    A = bf(Bt, M, K)
    Bm = bf(Bt, N, K)
    ref = A.float() @ Bm.float().transpose(1, 2)
    for akc in (True, False):
        for bkc in (True, False):
            Aop = A if akc else A.transpose(1, 2).contiguous()
            Bop = Bm if bkc else Bm.transpose(1, 2).contiguous()
            C = torch.zeros(Bt, M, N, device=dev, dtype=torch.float32)
            ops.gemm(M, N, K, Aop, K if akc else M, akc, Bop, K if bkc else N, bkc, C, N, batch=Bt,
                     batch_inner=1, sA=(M * K, 0), sB=(N * K, 0), sC=(M * N, 0))
            close(C, ref, rtol=1e-4, atol=1e-3)


@pytest.mark.parametrize("K", [2208, 40, 200])
def test_batched_tn_256_tile(K):
    """Batched TN GEMMs with >= 256 x 256 outputs per entry (the joint attention's dK = dS^T Q, dV = P^T dO: 288 x 256
    per sample, K = vlm rows x heads 2208 or the action mixture's 40 with beta accumulation) take the 256-tile kernel:
    two row tiles per sample, the second with 32 rows; bf16 out, then accumulated (beta) -- vs fp32 torch"""
    from pizero_native import ops

    Bt, M, N = 96, 288, 256  # >= 160 workgroups (2 row tiles x 96): the 256-tile path's fill threshold
    assert ops.gemm_kernel_name(M, N, K, a_kc=False, b_kc=False, batch=Bt).startswith("gemm8k_kernel<false, false")
    At = bf(Bt, K, M, scale=0.5)  # k-strided A (dS / P as stored: [rows x heads][keys])
    Bk = bf(Bt, K, N, scale=0.5)  # k-strided B (Q / dO)
    ref = At.float().transpose(1, 2) @ Bk.float()
    C = torch.empty(Bt, M, N, device=dev, dtype=torch.bfloat16)
    kw = dict(batch=Bt, sA=(M * K, 0), sB=(N * K, 0), sC=(M * N, 0))
    ops.gemm(M, N, K, At, M, False, Bk, N, False, C, N, **kw)
    close(C, ref, atol=3e-2 * math.sqrt(K) / 8)
    ops.gemm(M, N, K, At, M, False, Bk, N, False, C, N, beta=True, **kw)
    close(C, 2 * ref, atol=6e-2 * math.sqrt(K) / 8)


@pytest.mark.parametrize("xcd", ["1", "0"])
def test_batched_xcd_grouped_layouts(xcd):
    """batch % 8 == 0 launches of the 128-tile kernel take the XCD-grouped 1-D grid (a batch entry's tiles
    on one XCD; PZ_GEMM_BATCH_XCD=0 = the 2-D grid): every layout (the TN one of the 288 x 256 shape = the joint
    attention's dK takes the 256-tile kernel), fp32 and bf16 outputs, beta accumulation -- run in a subprocess
    because the switch is read once per process"""
    import subprocess
    import sys

    code = r"""
import torch, sys
sys.path.insert(0, 'open-pi-zero_amd')
import pizero_native
from pizero_native import ops
pizero_native.lib()
torch.manual_seed(0)
dev = 'cuda'
for (Bt, M, N, K) in ((16, 288, 256, 200), (8, 96, 80, 104)):
    A = (torch.randn(Bt, M, K, device=dev) * 0.5).to(torch.bfloat16)
    Bm = (torch.randn(Bt, N, K, device=dev) * 0.5).to(torch.bfloat16)
    ref = A.float() @ Bm.float().transpose(1, 2)
    for akc in (True, False):
        for bkc in (True, False):
            Aop = A if akc else A.transpose(1, 2).contiguous()
            Bop = Bm if bkc else Bm.transpose(1, 2).contiguous()
            C = torch.zeros(Bt, M, N, device=dev)
            ops.gemm(M, N, K, Aop, K if akc else M, akc, Bop, K if bkc else N, bkc, C, N, batch=Bt, batch_inner=1,
                     sA=(M * K, 0), sB=(N * K, 0), sC=(M * N, 0))
            assert (C - ref).abs().max().item() < 1e-3 * ref.abs().max().item() + 1e-3, (Bt, M, N, K, akc, bkc)
            Cb = torch.empty(Bt, M, N, device=dev, dtype=torch.bfloat16)
            ops.gemm(M, N, K, Aop, K if akc else M, akc, Bop, K if bkc else N, bkc, Cb, N, batch=Bt, batch_inner=1,
                     sA=(M * K, 0), sB=(N * K, 0), sC=(M * N, 0))
            ops.gemm(M, N, K, Aop, K if akc else M, akc, Bop, K if bkc else N, bkc, Cb, N, batch=Bt, batch_inner=1,
                     sA=(M * K, 0), sB=(N * K, 0), sC=(M * N, 0), beta=True)
            assert ((Cb.float() - 2 * ref).abs() <= 2e-2 * (2 * ref).abs() + 2e-2).all(), (Bt, M, N, K, akc, bkc)
print('OK')
"""
    import os

    env = dict(os.environ, PZ_GEMM_BATCH_XCD=xcd)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "-c", code], cwd=root, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and "OK" in r.stdout, r.stdout + r.stderr


@pytest.mark.parametrize("K", [1024, 4304, 40])
@pytest.mark.parametrize("akc,bkc", [(True, True), (True, False), (False, True), (False, False)])
def test_gemm256_layouts_with_tails(akc, bkc, K):
    """Large shapes take the 256x256 LDS-DMA kernel; M/N not multiples of the tile, K tail
    (4304 = SigLIP MLP width: 67 full K-tiles + 16; 40: a single partial K-tile)."""
    from pizero_native import ops

    M, N = 2600, 4104
    assert ops.gemm_kernel_name(M, N, K, a_kc=akc, b_kc=bkc).startswith(("gemm8p_kernel", "gemm8k_kernel"))
    A = bf(M, K, scale=0.5)
    Bm = bf(N, K, scale=0.5)
    ref = A.float() @ Bm.float().t()
    Aop = A if akc else A.t().contiguous()
    Bop = Bm if bkc else Bm.t().contiguous()
    C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    bias = bf(N)
    ops.gemm(M, N, K, Aop, K if akc else M, akc, Bop, K if bkc else N, bkc, C, N, bias=bias)
    close(C, ref + bias.float(), atol=3e-2)
    Cf = torch.zeros(M, N, device=dev, dtype=torch.float32)
    ops.gemm(M, N, K, Aop, K if akc else M, akc, Bop, K if bkc else N, bkc, Cf, N, beta=True)
    ops.gemm(M, N, K, Aop, K if akc else M, akc, Bop, K if bkc else N, bkc, Cf, N, beta=True)
    close(Cf, 2 * ref, rtol=1e-3, atol=1e-2)


@pytest.mark.parametrize("K", [64, 128, 192, 136, 320])
def test_gemm8p_two_section_short_k(K):
    """The two-section main loop (both operands k-contiguous) at 1, 2 and 3 K-tiles, where its prologue issues fewer
    pieces and its counted waits drop to vmcnt(2) / (0); 136 = two full K-tiles + an 8-deep tail, 320 = 5 tiles;
    plain + bias and the GeGLU epilogue (saved g|u) vs fp32 torch."""
    from pizero_native import ops

    M, N = 2600, 4104
    assert ops.gemm_kernel_name(M, N, K, a_kc=True, b_kc=True).startswith("gemm8p_kernel")
    A, Bm, bias = bf(M, K, scale=0.5), bf(N, K, scale=0.5), bf(N)
    C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    ops.gemm(M, N, K, A, K, True, Bm, K, True, C, N, bias=bias)
    close(C, A.float() @ Bm.float().t() + bias.float(), atol=3e-2)
    I = 2052
    W = bf(2 * I, K, scale=K ** -0.5)
    h = torch.empty(M, I, device=dev, dtype=torch.bfloat16)
    gu = torch.empty(M, 2 * I, device=dev, dtype=torch.bfloat16)
    ops.linear(A, W, h, epi=ops.PZ_EPI_GEGLU, aux=gu)
    ref = A.float() @ W.float().t()
    close(gu, ref)
    close(h, torch.nn.functional.gelu(ref[:, :I], approximate="tanh") * ref[:, I:])


@pytest.mark.parametrize("K", [64, 136, 2056])
def test_gemm8p_two_section_kstrided_b(K):
    """Micro-batch-sized NN dgrads (A k-contiguous, B k-strided, >= 16384 rows, >= 4096 output columns) take the
    two-section loop with B read through transposed loads: 1 K-tile, 2 + tail, 32 + tail; bias, then fp32 beta
    accumulation, vs fp32 torch."""
    from pizero_native import ops

    M, N = 16400, 4104
    assert ops.gemm_kernel_name(M, N, K, a_kc=True, b_kc=False).startswith("gemm8p_kernel<true, false")
    A, Bm, bias = bf(M, K, scale=0.5), bf(N, K, scale=0.5), bf(N)
    Bop = Bm.t().contiguous()
    ref = A.float() @ Bm.float().t()
    C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    ops.gemm(M, N, K, A, K, True, Bop, N, False, C, N, bias=bias)
    close(C, ref + bias.float(), atol=3e-2)
    Cf = torch.zeros(M, N, device=dev, dtype=torch.float32)
    ops.gemm(M, N, K, A, K, True, Bop, N, False, Cf, N, beta=True)
    ops.gemm(M, N, K, A, K, True, Bop, N, False, Cf, N, beta=True)
    close(Cf, 2 * ref, rtol=1e-3, atol=1e-2)


def test_gemm256_geglu_with_tail():
    from pizero_native import ops

    M, K, I = 2000, 512, 4100
    x = bf(M, K)
    W = bf(2 * I, K, scale=K ** -0.5)
    h = torch.empty(M, I, device=dev, dtype=torch.bfloat16)
    gu = torch.empty(M, 2 * I, device=dev, dtype=torch.bfloat16)
    ops.linear(x, W, h, epi=ops.PZ_EPI_GEGLU, aux=gu)
    ref = x.float() @ W.float().t()
    close(gu, ref)
    close(h, torch.nn.functional.gelu(ref[:, :I], approximate="tanh") * ref[:, I:])


@pytest.mark.parametrize("M,N,K", [(1000, 1280, 2056), (4352, 4096, 1024)])
@pytest.mark.parametrize("akc,bkc", [(True, True), (True, False), (False, True), (False, False)])
def test_gemm8p_split_tail(akc, bkc, M, N, K):
    """Wave-quantisation split: leftover tiles (all 20 of a 4x5 grid; 16 after one full round of 256)
    run as K-pieces into the fp32 workspace, summed + epilogued by gemm8p_tail_epilogue.
    Covers bias, residual, beta accumulation and a K tail (2056 = 32 K-tiles + 8) in the last piece."""
    import os

    from pizero_native import ops

    name = ops.gemm_kernel_name(M, N, K, a_kc=akc, b_kc=bkc)
    assert name.startswith(("gemm8p_kernel", "gemm8k_kernel")) and "tail" in name, name
    A = bf(M, K, scale=0.5)
    Bm = bf(N, K, scale=0.5)
    ref = A.float() @ Bm.float().t()
    Aop = A if akc else A.t().contiguous()
    Bop = Bm if bkc else Bm.t().contiguous()
    lda, ldb = (K if akc else M), (K if bkc else N)
    bias, R = bf(N), bf(M, N)
    C = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    ops.gemm(M, N, K, Aop, lda, akc, Bop, ldb, bkc, C, N, bias=bias, resid=R, ld_resid=N)
    close(C, ref + bias.float() + R.float(), atol=3e-2)
    C0 = torch.empty_like(C)
    os.environ["PZ_GEMM_TAIL"] = "0"
    try:
        ops.gemm(M, N, K, Aop, lda, akc, Bop, ldb, bkc, C0, N, bias=bias, resid=R, ld_resid=N)
    finally:
        os.environ.pop("PZ_GEMM_TAIL")
    close(C, C0, atol=3e-2)
    Cb = R.clone()
    ops.gemm(M, N, K, Aop, lda, akc, Bop, ldb, bkc, Cb, N, beta=True)
    close(Cb, ref + R.float(), atol=3e-2)
    C2 = torch.empty_like(C)
    ops.gemm(M, N, K, Aop, lda, akc, Bop, ldb, bkc, C2, N, bias=bias, resid=R, ld_resid=N)
    assert torch.equal(C, C2)  # fixed-order partial sums: deterministic


def test_wgrad_small_output_uses_split_tail():
    """weight gradient of a 1152x1152 layer over 16384 tokens: 25 output tiles split into K-pieces"""
    from pizero_native import ops

    M, N, K = 16384, 1152, 1152
    dy, x = bf(M, N, scale=0.3), bf(M, K, scale=0.3)
    assert "tail" in ops.gemm_kernel_name(N, K, M, a_kc=False, b_kc=False)
    dW = torch.empty(N, K, device=dev, dtype=torch.bfloat16)
    ops.linear_wgrad(dy, x, dW)
    close(dW, dy.float().t() @ x.float(), atol=5e-2)


@pytest.mark.parametrize("M", [4, 700, 17664])
def test_backward_activation_epilogues(M):
    """dgrad GEMMs with the activation derivative fused (DGELU / DSILU from the saved pre-activation,
    DGEGLU from saved [g | u] written back in place) vs torch autograd of the same ops in fp32."""
    from pizero_native import ops

    I, H = 1024, 512
    dy = bf(M, H, scale=0.5)
    W = bf(H, I, scale=I ** -0.5)  # next layer's weight [out=H, in=I]
    pre = bf(M, I)
    for epi, f in ((ops.PZ_EPI_DGELU, lambda x: torch.nn.functional.gelu(x, approximate="tanh")),
                   (ops.PZ_EPI_DSILU, torch.nn.functional.silu)):
        x = pre.float().requires_grad_()
        f(x).backward(dy.float() @ W.float())
        out = torch.empty(M, I, device=dev, dtype=torch.bfloat16)
        ops.linear_dgrad(dy, W, out, epi=epi, aux=pre)
        close(out, x.grad, atol=2e-2)
    gu = bf(M, 2 * I)
    g, u = (t.float().requires_grad_() for t in (gu[:, :I], gu[:, I:]))
    (torch.nn.functional.gelu(g, approximate="tanh") * u).backward(dy.float() @ W.float())
    buf = gu.clone()
    ops.linear_dgrad(dy, W, buf, epi=ops.PZ_EPI_DGEGLU, aux=buf)  # in place over the saved g|u
    close(buf[:, :I], g.grad, atol=2e-2)
    close(buf[:, I:], u.grad, atol=2e-2)


def test_epilogues_gelu_resid_geglu_silu():
    from pizero_native import ops

    M, K, I = 300, 256, 192
    x = bf(M, K)
    W = bf(2 * I, K, scale=K ** -0.5)
    h = torch.empty(M, I, device=dev, dtype=torch.bfloat16)
    gu = torch.empty(M, 2 * I, device=dev, dtype=torch.bfloat16)
    ops.linear(x, W, h, epi=ops.PZ_EPI_GEGLU, aux=gu)
    ref = x.float() @ W.float().t()
    close(gu, ref)
    g, u = ref[:, :I], ref[:, I:]
    close(h, torch.nn.functional.gelu(g, approximate="tanh") * u)
    # skinny path (M <= 16) for the same op
    h2 = torch.empty(5, I, device=dev, dtype=torch.bfloat16)
    ops.linear(x[:5], W, h2, epi=ops.PZ_EPI_GEGLU)
    close(h2, (torch.nn.functional.gelu(g, approximate="tanh") * u)[:5])
    # gelu + bias + residual
    b = bf(I)
    r = bf(M, I)
    pre = torch.empty(M, I, device=dev, dtype=torch.bfloat16)
    o = torch.empty(M, I, device=dev, dtype=torch.bfloat16)
    ops.linear(x, W[:I], o, bias=b, epi=ops.PZ_EPI_GELU, aux=pre, resid=r)
    p = x.float() @ W[:I].float().t() + b.float()
    close(pre, p)
    close(o, torch.nn.functional.gelu(p, approximate="tanh") + r.float(), atol=2e-2)
    ops.linear(x, W[:I], o, bias=b, epi=ops.PZ_EPI_SILU, aux=pre)
    close(o, torch.nn.functional.silu(p))


@pytest.mark.parametrize("M,N,K", [(256, 1152, 4304), (276, 2048, 16384), (100, 300, 1024), (276, 2560, 2048)])
def test_split_k_forward_epilogues(M, N, K, monkeypatch):
    """Few-tile batch-1 GEMMs (B=1 prefill) run split-K + epilogue pass (or, long K, the 256-tile
    kernel's K-pieces + tail epilogue) when the row-slab kernel is off; same results as one pass."""
    from pizero_native import ops

    monkeypatch.setenv("PZ_GEMM_ROWS", "0")
    monkeypatch.setenv("PZ_GEMM_TALL", "0")  # (the tall-tile kernel has its own test)

    name = ops.gemm_kernel_name(M, N, K, epi=ops.PZ_EPI_GELU)
    assert "splitk" in name or "tail" in name, name
    x, W, b, r = bf(M, K), bf(N, K, scale=K ** -0.5), bf(N), bf(M, N)
    ref = x.float() @ W.float().t() + b.float()
    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    pre = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    ops.linear(x, W, out, bias=b, resid=r)
    close(out, ref + r.float(), atol=2e-2)
    ops.linear(x, W, out, bias=b, epi=ops.PZ_EPI_GELU, aux=pre)
    close(pre, ref)
    close(out, torch.nn.functional.gelu(ref, approximate="tanh"))
    out32 = torch.ones(M, N, device=dev, dtype=torch.float32)
    ops.gemm(M, N, K, x, K, True, W, K, True, out32, N, beta=True)
    close(out32, 1.0 + x.float() @ W.float().t(), rtol=1e-3, atol=1e-3)
    I = N // 2 // 4 * 4
    if I * 2 == N:
        h = torch.empty(M, I, device=dev, dtype=torch.bfloat16)
        gu = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        name = ops.gemm_kernel_name(M, N, K, epi=ops.PZ_EPI_GEGLU, geglu_inter=I)
        assert "splitk" in name or "tail" in name, name
        ops.linear(x, W, h, epi=ops.PZ_EPI_GEGLU, aux=gu)
        raw = x.float() @ W.float().t()
        close(gu, raw)
        close(h, torch.nn.functional.gelu(raw[:, :I], approximate="tanh") * raw[:, I:])


@pytest.mark.parametrize("M,N,K", [(256, 3456, 1152), (256, 1152, 4304), (276, 2048, 2048), (320, 1024, 4096),
                                   (100, 300, 1032), (512, 520, 200), (65, 2560, 1024)])
@pytest.mark.parametrize("variant", ["auto", "w4", "w8", "tnb1", "tnb2", "tnb4"])
def test_rows_kernel_forward_epilogues(M, N, K, variant, monkeypatch):
    """Row-slab GEMM (64 < M <= 512, whole K per workgroup, no split-K pass): every forward epilogue, K tails
    (K % 64 != 0), row / column edges, each wave count and tile width."""
    from pizero_native import ops

    monkeypatch.setenv("PZ_GEMM_ROWS", "1")  # every 64 < M <= 512 shape (default: K <= 2048, <= 4096 columns)
    monkeypatch.setenv("PZ_GEMM_TALL", "0")  # (planned before the row-slab kernel where it measured faster)
    knob = {"w4": ("PZ_ROWS_W", "4"), "w8": ("PZ_ROWS_W", "8"), "tnb1": ("PZ_ROWS_TNB", "1"),
            "tnb2": ("PZ_ROWS_TNB", "2"), "tnb4": ("PZ_ROWS_TNB", "4")}.get(variant)
    if knob:
        monkeypatch.setenv(*knob)
    assert ops.gemm_kernel_name(M, N, K).startswith("gemm_rows_kernel"), ops.gemm_kernel_name(M, N, K)
    x, W, b, r = bf(M, K), bf(N, K, scale=K ** -0.5), bf(N), bf(M, N)
    ref = x.float() @ W.float().t() + b.float()
    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    pre = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    ops.linear(x, W, out, bias=b, resid=r)
    close(out, ref + r.float(), atol=2e-2)
    ops.linear(x, W, out, bias=b, epi=ops.PZ_EPI_GELU, aux=pre)
    close(pre, ref)
    close(out, torch.nn.functional.gelu(ref, approximate="tanh"))
    ops.linear(x, W, out, bias=b, epi=ops.PZ_EPI_SILU)
    close(out, torch.nn.functional.silu(ref))
    out32 = torch.ones(M, N, device=dev, dtype=torch.float32)
    ops.gemm(M, N, K, x, K, True, W, K, True, out32, N, beta=True)
    close(out32, 1.0 + x.float() @ W.float().t(), rtol=1e-3, atol=1e-3)
    # row-strided views (ld > K / ld > N), as the engine passes them
    xs = bf(M, K + 8)[:, :K]
    xs.copy_(x)
    outs = torch.empty(M, N + 4, device=dev, dtype=torch.bfloat16)[:, :N]
    ops.linear(xs, W, outs, bias=b)
    close(outs, ref)
    I = N // 2 // 4 * 4
    if I * 2 == N:
        monkeypatch.setenv("PZ_ROWS_FIRST", "1")  # GeGLU shapes that the 256-tile path would otherwise take
        name = ops.gemm_kernel_name(M, N, K, epi=ops.PZ_EPI_GEGLU, geglu_inter=I)
        assert name.startswith("gemm_rows_kernel") and name.endswith("true, false>"), name
        h = torch.empty(M, I, device=dev, dtype=torch.bfloat16)
        gu = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        ops.linear(x, W, h, epi=ops.PZ_EPI_GEGLU, aux=gu)
        raw = x.float() @ W.float().t()
        close(gu, raw)
        close(h, torch.nn.functional.gelu(raw[:, :I], approximate="tanh") * raw[:, I:])


@pytest.mark.parametrize("K", [96, 1024, 2048, 4096, 4128])
def test_skinny_widths(K, monkeypatch):
    """M <= 16 rows: W = 4/8/16 waves per block, 8/4/1-chunk unroll tails (MFMA skinny kernel)."""
    from pizero_native import ops

    monkeypatch.setenv("PZ_GEMV", "0")
    for M in (1, 4, 16):
        x, W, b = bf(M, K), bf(1040, K, scale=K ** -0.5), bf(1040)
        out = torch.empty(M, 1040, device=dev, dtype=torch.bfloat16)
        assert "skinny" in ops.gemm_kernel_name(M, 1040, K)
        ops.linear(x, W, out, bias=b)
        close(out, x.float() @ W.float().t() + b.float())


@pytest.mark.parametrize("min_nc", ["16", "4"])
@pytest.mark.parametrize("N", [1024, 1040, 2560, 4100])
def test_skinny_column_blocks(N, min_nc, monkeypatch):
    """PZ_SKINNY_MINNC=4: narrow outputs take 8 or 4 columns per block; ragged last block."""
    from pizero_native import ops

    monkeypatch.setenv("PZ_SKINNY_MINNC", min_nc)
    monkeypatch.setenv("PZ_GEMV", "0")
    K = 2048
    for M in (1, 4, 16):
        x, W, r = bf(M, K), bf(N, K, scale=K ** -0.5), bf(M, N)
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        name = ops.gemm_kernel_name(M, N, K)
        assert name.startswith("gemm_skinny_kernel<16, "), name
        ops.linear(x, W, out, resid=r)
        close(out, x.float() @ W.float().t() + r.float())


def _rms_ref(x, w, eps):
    """paligemma/modules.py:7-21 in fp32, rounded to bf16 like the unfused path"""
    xf = x.float()
    return (xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps) * (1 + w.float())).to(torch.bfloat16)


@pytest.mark.parametrize("gemv", ["1", "0"])
@pytest.mark.parametrize("K,N", [(1024, 2560), (2048, 1024)])
def test_skinny_fused_rmsnorm(K, N, gemv, monkeypatch):
    """Gemma RMSNorm fused into the few-row GEMM (inference denoise q|k|v and gate|up) vs
    rmsnorm -> GEMM in fp32; also the GeGLU epilogue."""
    from pizero_native import ops

    monkeypatch.setenv("PZ_GEMV", gemv)
    eps = 1e-6
    for M in (1, 4, 16, 50, 64):  # 50 / 64: the skinny-64 kernel (C5 denoise rows)
        x = bf(M, K, scale=3.0)
        w = bf(K, scale=0.5)
        W = bf(N, K, scale=K ** -0.5)
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        ops.linear(x, W, out, norm=(w, eps))
        # the fused path rounds x * (1 + w) to bf16 (rsqrt applied to the fp32 sums) where the unfused
        # one rounds the normalised row: ~1 bf16 ulp of the output apart
        close(out, _rms_ref(x, w, eps).float() @ W.float().t(), rtol=2e-2, atol=4e-2)
        I = N // 2
        h = torch.empty(M, I, device=dev, dtype=torch.bfloat16)
        ops.linear(x, W, h, epi=ops.PZ_EPI_GEGLU, norm=(w, eps))
        raw = _rms_ref(x, w, eps).float() @ W.float().t()
        close(h, torch.nn.functional.gelu(raw[:, :I], approximate="tanh") * raw[:, I:], rtol=3e-2, atol=6e-2)
    with pytest.raises(RuntimeError):  # many rows: not a few-row path
        x = bf(65, K)
        ops.linear(x, W, torch.empty(65, N, device=dev, dtype=torch.bfloat16), norm=(w, eps))


@pytest.mark.parametrize("K", [1024, 2048, 4096])
def test_gemv_epilogues(K):
    """few-row GEMV path (M <= 8, K % 512 == 0): every epilogue vs fp32 torch"""
    from pizero_native import ops

    F = torch.nn.functional
    for M in (1, 4, 5, 8):
        assert ops.gemm_kernel_name(M, 1024, K).startswith("gemv_kernel"), ops.gemm_kernel_name(M, 1024, K)
        x = bf(M, K)
        for N in (1024, 1040, 2560):
            W, b, r = bf(N, K, scale=K ** -0.5), bf(N), bf(M, N)
            ref = x.float() @ W.float().t()
            out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            ops.linear(x, W, out, bias=b, resid=r)
            close(out, ref + b.float() + r.float())
            aux = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            ops.linear(x, W, out, bias=b, epi=ops.PZ_EPI_GELU, aux=aux)
            close(aux, ref + b.float())
            close(out, F.gelu(ref + b.float(), approximate="tanh"))
            ops.linear(x, W, out, epi=ops.PZ_EPI_SILU)
            close(out, F.silu(ref))
            o32 = torch.zeros(M, N, device=dev)
            ops.gemm(M, N, K, x, K, True, W, K, True, o32, N, beta=True)
            ops.gemm(M, N, K, x, K, True, W, K, True, o32, N, beta=True)
            close(o32, 2 * ref, rtol=1e-3, atol=1e-3)
        I = 4096
        Wg = bf(2 * I, K, scale=K ** -0.5)
        raw = x.float() @ Wg.float().t()
        h = torch.empty(M, I, device=dev, dtype=torch.bfloat16)
        gu = torch.empty(M, 2 * I, device=dev, dtype=torch.bfloat16)
        ops.linear(x, Wg, h, epi=ops.PZ_EPI_GEGLU, aux=gu)
        close(gu, raw)
        close(h, F.gelu(raw[:, :I], approximate="tanh") * raw[:, I:], rtol=3e-2, atol=3e-2)


@pytest.mark.parametrize("M,T", [(4, 4), (8, 4), (1, 1)])
def test_gemv_qkv_rope_matches_unfused(M, T):
    """pz_gemv_qkv_rope == RMSNorm-fused q|k|v GEMM + pz_qkv_rope_split (same rounding points)"""
    from pizero_native import ops

    K, nh, hd = 1024, 8, 256
    B = M // T
    N = (nh + 2) * hd
    x, W, w = bf(M, K, scale=2.0), bf(N, K, scale=K ** -0.5), bf(K, scale=0.3)
    pos = torch.randint(0, 200, (B, T), device=dev, dtype=torch.int64)
    cs = torch.empty(301 * hd, device=dev)
    ops.rope_table(cs, 300, hd, 100.0)
    Lq, Lk, qoff, koff = T + 2, 290, 1, 277
    q1 = torch.zeros(B, Lq, nh * hd, device=dev, dtype=torch.bfloat16)
    k1 = torch.zeros(B, Lk, hd, device=dev, dtype=torch.bfloat16)
    v1 = torch.zeros_like(k1)
    q2, k2, v2 = q1.clone(), k1.clone(), v1.clone()
    ops.gemv_qkv_rope(x, W, pos, cs, q1, k1, v1, T, nh, hd, Lq, qoff, Lk, koff, norm=(w, 1e-6))
    qkv = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    ops.linear(x, W, qkv, norm=(w, 1e-6))
    ops.qkv_rope_split(qkv, pos, cs, q2, k2, v2, B, T, nh, 1, hd, Lq, qoff, Lk, koff)
    close(q1, q2, rtol=2e-2, atol=2e-2)
    close(k1, k2, rtol=2e-2, atol=2e-2)
    close(v1, v2, rtol=2e-2, atol=2e-2)
    assert q1[:, :qoff].abs().max() == 0 and k1[:, :koff].abs().max() == 0  # only the target rows written


def test_small_gemm():
    from pizero_native import ops

    x, W, b = bf(20, 7), bf(64, 7), bf(64)
    out = torch.empty(20, 64, device=dev, dtype=torch.bfloat16)
    ops.small_linear(x, W, out, bias=b)
    close(out, x.float() @ W.float().t() + b.float())
    # long-K, N=7 (action decoder): one wave per row; output rows padded to 8 like the engine's
    for M, K in ((4, 1024), (257, 1024), (3, 264)):
        x, W, b = bf(M, K), bf(7, K, scale=K ** -0.5), bf(7)
        out = torch.zeros(M, 8, device=dev, dtype=torch.bfloat16)
        ops.small_linear(x, W, out[:, :7], bias=b)
        close(out[:, :7], x.float() @ W.float().t() + b.float())
        assert out[:, 7].abs().max().item() == 0
        ops.small_linear(x, W, out[:, :7], bias=b, beta=True)
        close(out[:, :7], 2 * (x.float() @ W.float().t() + b.float()), atol=2e-2)


@pytest.mark.parametrize("kern", ["row", "wave"])
@pytest.mark.parametrize("D", [1024, 2048, 64])
def test_rmsnorm_fwd_bwd(D, kern, monkeypatch):
    """both backward kernels: row-per-step (default) and wave-per-row (PZ_NORM_BWD=wave)"""
    from pizero_native import ops

    monkeypatch.setenv("PZ_NORM_BWD", kern)

    R = 333
    x = bf(R, D)
    w = bf(D, scale=0.1)
    y = torch.empty_like(x)
    rstd = torch.empty(R, device=dev)
    ops.rmsnorm(x, w, y, rstd, 1e-6)
    xr = x.float().requires_grad_()
    wr = w.float().requires_grad_()
    yr = xr * torch.rsqrt(xr.pow(2).mean(-1, keepdim=True) + 1e-6) * (1 + wr)
    close(y, yr)
    dy = bf(R, D)
    yr.backward(dy.float())
    dres = bf(R, D)
    dx = torch.empty_like(x)
    rpp = ops.rows_per_part()
    part = torch.empty((R + rpp - 1) // rpp, D, device=dev)
    ops.rmsnorm_bwd(dy, x, w, rstd, dx, dres=dres, dw_part=part)
    close(dx, xr.grad + dres.float(), atol=2e-2)
    dw = torch.empty(D, device=dev, dtype=torch.bfloat16)
    ops.reduce_parts(part, dw)
    close(dw, wr.grad, atol=0.1)


@pytest.mark.parametrize("kern", ["row", "wave"])
def test_layernorm_fwd_bwd(kern, monkeypatch):
    from pizero_native import ops

    monkeypatch.setenv("PZ_NORM_BWD", kern)

    R, D = 300, 1152
    x = bf(R, D) * 3 + 1
    w, b = bf(D) * 0.1 + 1, bf(D) * 0.1
    y = torch.empty_like(x)
    mean, rstd = torch.empty(R, device=dev), torch.empty(R, device=dev)
    ops.layernorm(x, w, b, y, mean, rstd, 1e-6)
    xr, wr, br = (t.float().requires_grad_() for t in (x, w, b))
    yr = torch.nn.functional.layer_norm(xr, (D,), wr, br, 1e-6)
    close(y, yr)
    dy = bf(R, D)
    yr.backward(dy.float())
    dx = torch.empty_like(x)
    rpp = ops.rows_per_part()
    P = (R + rpp - 1) // rpp
    pw, pb = torch.empty(P, D, device=dev), torch.empty(P, D, device=dev)
    ops.layernorm_bwd(dy, x, w, mean, rstd, dx, dw_part=pw, db_part=pb)
    close(dx, xr.grad, atol=2e-2)
    dw, db = torch.empty(D, device=dev, dtype=torch.bfloat16), torch.empty(D, device=dev, dtype=torch.bfloat16)
    ops.reduce_parts(pw, dw)
    ops.reduce_parts(pb, db)
    close(dw, wr.grad, atol=0.1)
    close(db, br.grad, atol=0.1)
    db2 = torch.empty(D, device=dev, dtype=torch.bfloat16)
    ws = torch.empty(64 * D, device=dev)
    ops.colsum(dy, db2, ws)
    close(db2, dy.float().sum(0), atol=0.1)
    if kern == "row":  # fused column sums of the bf16 dx (+ residual gradient): the next Linear's bias gradient
        dres = bf(R, D)
        dx2, pd = torch.empty_like(x), torch.empty(P, D, device=dev)
        ops.layernorm_bwd(dy, x, w, mean, rstd, dx2, dres=dres, dw_part=pw, db_part=pb, dx_part=pd)
        close(dx2, xr.grad + dres.float(), atol=3e-2)
        s1, s2 = torch.empty(D, device=dev, dtype=torch.bfloat16), torch.empty(D, device=dev, dtype=torch.bfloat16)
        ops.reduce_parts(pd, s1)
        ops.colsum(dx2, s2, ws)
        close(s1, dx2.float().sum(0), atol=0.1)
        assert (s1.float() - s2.float()).abs().max().item() <= 2 * 2 ** -7 * s2.float().abs().max().item() + 1e-3


def test_reduce_parts_multi_matches_single():
    """pz_reduce_parts_multi (a layer's partial-sum reductions in one launch, > 8 segments = two launches) is
    bit-identical to one pz_reduce_parts per segment, beta included."""
    from pizero_native import ops

    shapes = [(1024, 1152), (1104, 2048), (3, 4), (64, 4304), (1024, 1152), (17, 256), (1, 8), (300, 1152), (5, 12)]
    items, refs = [], []
    for P, D in shapes:
        part = torch.randn(P, D, device=dev)
        out1 = bf(D)
        out2 = out1.clone()
        ops.reduce_parts(part, out1, beta=True)
        items.append((part, out2))
        refs.append(out1)
    ops.reduce_parts_multi(items, beta=True)
    for (part, o), r in zip(items, refs):
        assert torch.equal(o, r), part.shape


@pytest.mark.parametrize("M,N,act", [(16384, 4304, "gelu"), (300, 1152, "gelu"), (320, 4096, "silu"), (17, 64, "gelu")])
def test_act_bwd_colsum_matches_unfused(M, N, act):
    """pz_act_bwd_colsum (GELU / SiLU backward + the bias gradient in one pass, SigLIP fc1) vs pz_act_bwd + pz_colsum:
    dpre bit-identical, the column sums within fp32 summation-order noise, beta accumulation."""
    from pizero_native import ops

    a = ops.PZ_EPI_GELU if act == "gelu" else ops.PZ_EPI_SILU
    dh, pre = bf(M, N), bf(M, N) * 2
    d1, d2 = dh.clone(), dh.clone()
    ops.act_bwd(d1, pre, d1, None, a)
    ws = torch.empty(256, N, device=dev)
    b2 = torch.full((N,), 0.5, device=dev, dtype=torch.bfloat16)
    ops.act_bwd_colsum(d2, pre, d2, a, ws, b2, beta=True)  # in place, as the engine calls it
    assert torch.equal(d1, d2)
    ref = 0.5 + d1.float().sum(0)
    close(b2, ref, rtol=2e-2, atol=0.05 + 1e-4 * math.sqrt(M))


@pytest.mark.parametrize("M,N", [(16384, 1152), (17664, 2048), (300, 4304), (5, 7), (1000, 40), (64, 3456), (257, 1024)])
def test_colsum_and_reduce_parts_shapes(M, N):
    """bias / norm-weight gradient reductions (vectorised and scalar dispatch paths), with and without beta"""
    from pizero_native import ops

    X = bf(M, N)
    ref = X.float().sum(0)
    out = torch.empty(N, device=dev, dtype=torch.bfloat16)
    ws = torch.empty(64 * N, device=dev)
    ops.colsum(X, out, ws)
    close(out, ref, atol=0.05 + 2e-3 * math.sqrt(M))
    prev = bf(N)
    out2 = prev.clone()
    ops.colsum(X, out2, ws, beta=True)
    close(out2, ref + prev.float(), atol=0.05 + 2e-3 * math.sqrt(M))
    # fixed-order reduction: bitwise identical on a second launch
    out3 = torch.empty_like(out)
    ops.colsum(X, out3, ws)
    assert torch.equal(out, out3)
    P = (M + 63) // 64
    part = torch.randn(P, N, device=dev)
    r = torch.empty(N, device=dev, dtype=torch.bfloat16)
    ops.reduce_parts(part, r)
    close(r, part.sum(0), atol=1e-2 * math.sqrt(P))


def _block_mask(cnt, P, C, Lq_off, Lq, L):
    m = torch.zeros(len(cnt), Lq, L, dtype=torch.bool)
    for b, c in enumerate(cnt):
        for qi in range(Lq):
            i = Lq_off + qi
            for j in range(L):
                if i < P:
                    ok = i < c and j < c
                elif i < P + C:
                    ok = j < c or (P <= j < P + C)
                else:
                    ok = j < c or j >= P
                m[b, qi, j] = ok
    return m


def test_softmax_block_mask_softcap_fwd_bwd():
    from pizero_native import ops

    B, P, C, H, nh = 2, 12, 1, 4, 8
    L = P + C + H
    Lp = 24
    cnt = torch.tensor([10, 7], dtype=torch.int32, device=dev)
    R = B * L * nh
    S = torch.randn(R, Lp, device=dev) * 40
    S[:, L:] = float("nan")  # padded logit columns are never written by the S GEMM
    Pm = torch.empty(R, Lp, device=dev, dtype=torch.bfloat16)
    tc = torch.empty(R, Lp, device=dev, dtype=torch.bfloat16)
    ops.attn_softmax(S, Lp, Pm, Lp, R, L, 1 / 16, cap=50.0, tcap=tc, mask_mode=1, rows_per_batch=L * nh, heads=nh,
                     qoff=0, cnt=cnt, prefix=P, cond=C)
    allowed = _block_mask(cnt.tolist(), P, C, 0, L, L).to(dev)  # [B, L, L]
    allowed = allowed[:, :, None, :].expand(B, L, nh, L).reshape(R, L)
    s = (S[:, :L] / 16).requires_grad_()
    lg = torch.tanh(s / 50) * 50
    lg = lg + torch.where(allowed, 0.0, torch.finfo(torch.float32).min)
    ref = torch.softmax(lg, -1)
    close(Pm[:, :L], ref, atol=2e-3)
    assert (Pm[:, L:] == 0).all()
    dP = torch.randn(R, Lp, device=dev)
    ref.backward(dP[:, :L])
    dS = torch.empty(R, Lp, device=dev, dtype=torch.bfloat16)
    ops.attn_softmax_bwd(Pm, dP, Lp, tc, dS, Lp, R, L, 1 / 16, 50.0)
    valid = allowed.any(-1)  # fully-masked rows: gradient unused downstream
    close(dS[valid, :L], s.grad[valid] / 16, atol=3e-3)
    assert (dS[:, L:] == 0).all() and not tc.isnan().any()


def test_qkv_rope_split_roundtrip():
    from pizero_native import ops

    B, T, nh, nkv, hd, theta = 2, 5, 8, 1, 256, 100.0
    qkv = bf(B * T, (nh + 2 * nkv) * hd)
    pos = torch.arange(1, T + 1, device=dev).repeat(B, 1)
    cs = torch.empty(64 * hd, device=dev)
    ops.rope_table(cs, 63, hd, theta)
    Lq, Lk, off = 9, 12, 3
    q = torch.zeros(B, Lq, nh * hd, device=dev, dtype=torch.bfloat16)
    k = torch.zeros(B, Lk, nkv * hd, device=dev, dtype=torch.bfloat16)
    v = torch.zeros_like(k)
    ops.qkv_rope_split(qkv, pos, cs, q, k, v, B, T, nh, nkv, hd, Lq, off, Lk, off)
    inv = 1.0 / (theta ** (torch.arange(0, hd, 2, device=dev).float() / hd))
    f = pos[:, :, None].float() * inv
    emb = torch.cat([f, f], -1)
    cos, sin = emb.cos(), emb.sin()
    x = qkv.float().view(B, T, nh + 2 * nkv, hd)

    def rot(t):
        return t * cos[:, :, None] + torch.cat([-t[..., hd // 2:], t[..., : hd // 2]], -1) * sin[:, :, None]

    close(q[:, off:off + T].view(B, T, nh, hd), rot(x[:, :, :nh]))
    close(k[:, off:off + T].view(B, T, nkv, hd), rot(x[:, :, nh:nh + nkv]))
    assert torch.equal(v[:, off:off + T].view(B, T, nkv, hd), x[:, :, nh + nkv:].to(torch.bfloat16))
    dqkv = torch.empty_like(qkv)
    ops.qkv_rope_split_bwd(q, k, v, pos, cs, dqkv, B, T, nh, nkv, hd, Lq, off, Lk, off)
    close(dqkv, qkv, atol=2e-2)  # rotation is orthogonal: bwd(fwd(x)) = x


def test_fill_uniform_matches_numpy_generator():
    from oracle.synth import synth_tensor, tensor_seed
    from pizero_native import ops

    x = torch.empty(100003, device=dev, dtype=torch.float32)
    ops.fill_uniform(x, tensor_seed("w.test"), 0.25, 0.5)
    ref = synth_tensor("w.test", (100003,), 0.25, 0.5)
    np.testing.assert_array_equal(x.cpu().numpy(), ref)


def test_adamw_matches_torch():
    from pizero_native import ops

    n = 10000
    p = bf(n)
    g = bf(n)
    m = torch.zeros(n, device=dev)
    v = torch.zeros(n, device=dev)
    pr = p.float().clone().requires_grad_()
    opt = torch.optim.AdamW([pr], lr=1e-2, weight_decay=0.01)
    for step in range(1, 4):
        pr.grad = g.float()
        opt.step()
        ops.adamw(p, g, m, v, 1e-2, 0.9, 0.999, 1e-8, 0.01, 1 - 0.9 ** step, 1 - 0.999 ** step)
    close(p, pr.detach(), atol=1e-2)
    parts = torch.empty(ops.PZ_SUMSQ_PARTS, device=dev)
    ops.sumsq(g, parts)
    assert abs(parts.sum().item() - (g.float() ** 2).sum().item()) < 1e-3 * parts.sum().item()


def test_wgrad_split_k_matches_single_pass():
    from pizero_native import ops

    M, N, K = 8192, 1024, 768  # small output, long token reduction -> K split inside pz_gemm (split tail)
    assert "tail" in ops.gemm_kernel_name(N, K, M, a_kc=False, b_kc=False)
    dy, x = bf(M, N), bf(M, K)
    dW = torch.empty(N, K, device=dev, dtype=torch.bfloat16)
    ops.linear_wgrad(dy, x, dW)
    ref = dy.float().t() @ x.float()
    close(dW, ref, atol=0.05 * math.sqrt(M) / 16)
    ops.linear_wgrad(dy, x, dW, beta=True)
    close(dW, 2 * ref, atol=0.1 * math.sqrt(M) / 16)


@pytest.mark.parametrize("mode", [False, True])
def test_time_embed_rows_matches_embed_plus_concat(mode):
    """pz_time_embed_rows (inference: the embedding written into the concat input's first D columns, H rows per
    sample) is bit-identical to pz_time_embed + pz_concat_time."""
    from pizero_native import ops

    B, H, D = 3, 50, 1024
    t = torch.rand(B, device=dev)
    e1 = bf(B * H, D)
    temb = torch.empty(B, D, device=dev, dtype=torch.bfloat16)
    ops.time_embed(t, temb, 4.0, ref_bf16=mode)
    cat1 = torch.empty(B * H, 2 * D, device=dev, dtype=torch.bfloat16)
    ops.concat_time(temb, e1, cat1, B, H, D)
    cat2 = torch.empty(B * H, 2 * D, device=dev, dtype=torch.bfloat16)
    cat2[:, D:].copy_(e1)
    ops.time_embed_rows(t, cat2[:, :D], H, 4.0, ref_bf16=mode)
    assert torch.equal(cat1, cat2)


def test_time_embed_modes_match_reference():
    """pz_time_embed mode 0 = the reference SinusoidalPosEmb in fp32; mode 1 = the reference's bf16
    arithmetic (bf16 arange rounds odd indices above 256, every op rounded; vla/modules.py:15-22)
    -- both against the reference's own outputs (tests/golden/time_embed.npz)."""
    from pizero_native import ops
    from tests.oracle_helpers import load_golden

    g = load_golden("time_embed")
    for P in (100, 10000):
        for mode, key, tkey in ((0, f"fp32_{P}", "t"), (1, f"bf16_{P}", f"t_bf16_{P}")):
            t = torch.from_numpy(g[tkey]).to(dev)
            out = torch.empty(t.numel(), 1024, device=dev, dtype=torch.bfloat16)
            ops.time_embed(t, out, float(P), ref_bf16=bool(mode))
            err = (out.float().cpu() - torch.from_numpy(g[key])).abs()
            assert err.max().item() <= 8e-3 and err.mean().item() <= 6e-4, (P, mode, err.max().item(), err.mean().item())
        # mode 1 tracks the bf16 reference more closely than the fp32 kernel does
        t = torch.from_numpy(g[f"t_bf16_{P}"]).to(dev)
        outs = []
        for mode in (0, 1):
            o = torch.empty(t.numel(), 1024, device=dev, dtype=torch.bfloat16)
            ops.time_embed(t, o, float(P), ref_bf16=bool(mode))
            outs.append((o.float().cpu() - torch.from_numpy(g[f"bf16_{P}"])).abs().mean().item())
        assert outs[1] < outs[0], outs


@pytest.mark.parametrize("mode", ["mfma", "mfma_wg64"])
@pytest.mark.parametrize("B,T,cnts,P", [(1, 4, [270], 276), (2, 4, [276, 259], 276), (1, 2, [100], 276),
                                          (2, 1, [5, 276], 276), (1, 50, [788], 788), (2, 13, [276, 200], 276),
                                          (3, 4, [300, 20, 311], 311), (1, 4, [7], 7)])
def test_decode_attn_matches_reference(B, T, cnts, P, mode, monkeypatch):
    """pz_decode_attn (denoise attention: T action tokens x 8 heads vs the cached keys, MQA) vs fp32 torch
    with the Gemma soft-cap and the Pi0 block mask (joint_model.py:259-292, pizero.py:271-306); T = 50 at
    P = 788 is C5's chunk (400 query rows = 13 row tiles), T = 13 a ragged last tile, 3 samples with 316 keys, 12 keys =
    one partial chunk.  mode "mfma": the key-split MFMA kernel (P.V on the matrix cores) + fixed-order merge (default);
    "mfma_wg64": several chunks per workgroup (online softmax across chunks) + merge"""
    from pizero_native import ops

    if mode == "mfma_wg64":
        monkeypatch.setenv("PZ_DECODE_WG", "4")
    C, nh, hd = 1, 8, 256
    nk = P + C + T
    Lp = (nk + 7) // 8 * 8
    q = bf(B, T, nh * hd)
    k, v = bf(B, Lp, hd), bf(B, Lp, hd)
    cnt = torch.tensor(cnts, device=dev, dtype=torch.int32)
    o = torch.empty(B * T, nh * hd, device=dev, dtype=torch.bfloat16)
    ops.decode_attn(q, T, 0, k, v, o, B, nh, T, nk, 1 / 16.0, 50.0, cnt, P, C, P + C)
    o2 = torch.empty_like(o)
    for _ in range(2):  # same inputs again: bitwise the same output, written by every call (deterministic merge)
        o2.fill_(float("nan"))
        ops.decode_attn(q, T, 0, k, v, o2, B, nh, T, nk, 1 / 16.0, 50.0, cnt, P, C, P + C)
        torch.cuda.synchronize()
        assert torch.equal(o2, o)
    qf = q.float().view(B, T, nh, hd)
    s = torch.einsum("bthd,bjd->bhtj", qf, k.float()[:, :nk]) / 16.0
    s = 50.0 * torch.tanh(s / 50.0)
    j = torch.arange(nk, device=dev)
    allowed = (j[None, :] < cnt[:, None]) | (j[None, :] >= P)  # action rows (pizero.py:296-306)
    s = s.masked_fill(~allowed[:, None, None, :], float("-inf"))
    ref = torch.einsum("bhtj,bjd->bthd", torch.softmax(s, -1), v.float()[:, :nk]).reshape(B * T, nh * hd)
    close(o, ref, rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("B,T,off,K", [(1, 50, 789, 1024), (10, 5, 277, 1024), (6, 5, 277, 2048), (4, 16, 20, 1024)])
@pytest.mark.parametrize("norm", [False, True])
@pytest.mark.parametrize("fp8", [False, True])
def test_gemm_qkv_rope_few_rows_bit_identical(B, T, off, K, norm, fp8):
    """pz_gemm_qkv_rope's few-row path (16 < M <= 64: C5's 50-row denoise chunk): the skinny-64 kernel with the
    rotation pairs of a head in one block, RoPE + Q / K / V scatter in the epilogue, RMSNorm optionally fused,
    bf16 or e4m3 (W8A16) weights -- bit-identical to pz_gemm (skinny-64, same fused norm / same fp8 codes) +
    pz_qkv_rope_split."""
    from pizero_native import ops

    nh, hd = 8, 256
    L = off + T + 3
    Lp = (L + 7) // 8 * 8
    M = B * T
    x, W = bf(M, K), bf((nh + 2) * hd, K, scale=K ** -0.5)
    nw = bf(K, scale=0.1) if norm else None
    nrm = (nw, 1e-6) if norm else None
    if fp8:  # the e4m3 codes + per-tensor scale of prepare_fp8, and the bf16 weights they decode to
        sc = ops.fp8_weight_scale(W)
        Wq = torch.empty(W.shape, device=dev, dtype=torch.uint8)
        ops.fp8_quant_tensor(W, Wq, sc)
        W = (Wq.view(torch.float8_e4m3fn).float() * float(sc)).to(torch.bfloat16)
    pos = (torch.arange(T, device=dev) + off).repeat(B).contiguous()
    cs = torch.empty((L + 9) * hd, device=dev, dtype=torch.float32)
    ops.rope_table(cs, L + 8, hd, 10000.0)
    outs = []
    for fused in (True, False):
        Q = torch.full((B, T, nh * hd), 7.0, device=dev, dtype=torch.bfloat16)
        Kj = torch.full((B, Lp, hd), 7.0, device=dev, dtype=torch.bfloat16)
        Vj = torch.full((B, Lp, hd), 7.0, device=dev, dtype=torch.bfloat16)
        if fused:
            assert ops.gemm_qkv_rope(x, Wq if fp8 else W, pos, cs, Q, Kj, Vj, T, nh, hd, T, 0, Lp, off, norm=nrm,
                                     w_scale=sc if fp8 else None)
        else:
            qkv = torch.empty(M, (nh + 2) * hd, device=dev, dtype=torch.bfloat16)
            if fp8:
                ops.linear_fp8(x, Wq, sc, qkv, norm=nrm)
            else:
                ops.linear(x, W, qkv, norm=nrm)
            ops.qkv_rope_split(qkv, pos, cs, Q, Kj, Vj, B, T, nh, 1, hd, T, 0, Lp, off)
        outs.append((Q, Kj, Vj))
    torch.cuda.synchronize()
    for nm, a, b in zip("QKV", *outs):
        assert torch.equal(a, b), (nm, int((a != b).sum()), float((a.float() - b.float()).abs().max()))
    assert (outs[0][1][:, :off] == 7.0).all() and (outs[0][1][:, off + T:] == 7.0).all()  # only rows off..off+T-1
    # and against torch fp32 (the reference's rotate_half form, utils.py:4-16)
    xf = x.float()
    if norm:
        xf = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + 1e-6) * (1.0 + nw.float())
    qkv = (xf @ W.float().t()).view(B, T, nh + 2, hd)
    c = cs.view(-1, hd)[pos.view(B, T)]
    co, si = c[..., 0::2], c[..., 1::2]
    cos, sin = torch.cat([co, co], -1)[:, :, None], torch.cat([si, si], -1)[:, :, None]
    rot = lambda t: torch.cat([-t[..., hd // 2:], t[..., : hd // 2]], -1)  # noqa: E731
    qk = qkv[:, :, : nh + 1] * cos + rot(qkv[:, :, : nh + 1]) * sin
    tol = 5e-2 if fp8 else 3e-2  # fp8: the reference uses the decoded weights (rounded to bf16 here)
    close(outs[0][0].view(B, T, nh, hd), qk[:, :, :nh], atol=tol)
    close(outs[0][1][:, off:off + T], qk[:, :, nh], atol=tol)
    close(outs[0][2][:, off:off + T], qkv[:, :, nh + 1], atol=tol)


@pytest.mark.parametrize("B,T,off", [(16, 276, 0), (64, 276, 0), (16, 5, 276)])
def test_gemm_qkv_rope_bit_identical_to_gemm_plus_split(B, T, off):
    """pz_gemm_qkv_rope (q|k|v GEMM with RoPE + joint Q/K/V scatter in the 8-phase epilogue, N1) against
    pz_gemm + pz_qkv_rope_split on the same bf16 inputs: bit-identical joint buffers, incl. a partial last
    row tile (B=16: 4416 rows) and the benched micro-batch (17664 rows).  Shapes the 8-phase kernel does
    not take (B=16 x 5 expert rows) return False and launch nothing."""
    from pizero_native import ops

    nh, hd, K = 8, 256, 2048
    L, Lp = 281, 288
    M = B * T
    x, W = bf(M, K), bf((nh + 2) * hd, K, scale=K ** -0.5)
    pos = (torch.arange(T, device=dev) + 1 + off).repeat(B).contiguous()
    cs = torch.empty((L + 9) * hd, device=dev, dtype=torch.float32)
    ops.rope_table(cs, L + 8, hd, 10000.0)
    outs = []
    for fused in (True, False):
        Q = torch.full((B, L, nh * hd), 7.0, device=dev, dtype=torch.bfloat16)
        Kj = torch.full((B, Lp, hd), 7.0, device=dev, dtype=torch.bfloat16)
        Vj = torch.full((B, Lp, hd), 7.0, device=dev, dtype=torch.bfloat16)
        done = fused and ops.gemm_qkv_rope(x, W, pos, cs, Q, Kj, Vj, T, nh, hd, L, off, Lp, off)
        if fused and T < 256:
            assert not done  # 80 rows: neither an 8-phase nor a few-row (<= 64) shape
        if not done:
            qkv = torch.empty(M, (nh + 2) * hd, device=dev, dtype=torch.bfloat16)
            ops.linear(x, W, qkv)
            ops.qkv_rope_split(qkv, pos, cs, Q, Kj, Vj, B, T, nh, 1, hd, L, off, Lp, off)
        outs.append((Q, Kj, Vj))
    torch.cuda.synchronize()
    for nm, a, b in zip("QKV", *outs):
        if not torch.equal(a, b):
            bad = (a != b).nonzero()
            print(f"{nm}: {bad.shape[0]} mismatches, first {bad[:4].tolist()}, fused {a[tuple(bad[0])].item()} "
                  f"vs split {b[tuple(bad[0])].item()}")
        assert torch.equal(a, b), (nm, float((a.float() - b.float()).abs().max()))
    if T >= 256:  # the rows the fused epilogue did not own are untouched
        assert (outs[0][0][:, T + off:] == 7.0).all() and (outs[0][1][:, T + off:] == 7.0).all()


@pytest.mark.parametrize("M,N,K", [(276, 2048, 2048), (256, 4304, 1152), (256, 1152, 4304), (320, 1024, 4096),
                                   (97, 200, 72)])
def test_gemm_tall_forward_epilogues(M, N, K, monkeypatch):
    """Tall-tile GEMM (pz_gemm_tall.hip, PZ_GEMM_TALL=1: one 256- / 320-row tile over 64 < M <= 1024 rows, K split
    over blockIdx.y + fixed-order split-K sum): bias + residual, GELU + saved pre-activation and fp32 beta
    accumulation against torch fp32; K tails (K % 64 != 0), ragged rows / columns.  (The GeGLU and k-strided-B
    forms are built only with -DPZ_TALL_AB: the planner never takes them.)"""
    from pizero_native import ops

    monkeypatch.setenv("PZ_GEMM_TALL", "1")
    x = bf(M, K)
    assert not ops.gemm_kernel_name(M, 2 * N, K, epi=ops.PZ_EPI_GEGLU, geglu_inter=N).startswith("gemm_tall_kernel")
    W, b, r = bf(N, K, scale=K ** -0.5), bf(N), bf(M, N)
    assert ops.gemm_kernel_name(M, N, K).startswith("gemm_tall_kernel"), ops.gemm_kernel_name(M, N, K)
    ref = x.float() @ W.float().t()
    o = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    ops.linear(x, W, o, bias=b, resid=r)
    close(o, ref + b.float() + r.float(), atol=2e-2)
    o, pre = torch.empty(M, N, device=dev, dtype=torch.bfloat16), torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    ops.linear(x, W, o, bias=b, epi=ops.PZ_EPI_GELU, aux=pre)
    close(pre, ref + b.float())
    close(o, torch.nn.functional.gelu(ref + b.float(), approximate="tanh"))
    c = torch.ones(M, N, device=dev, dtype=torch.float32)
    ops.gemm(M, N, K, x, K, True, W, K, True, c, N, beta=True)
    close(c, 1.0 + ref, rtol=1e-3, atol=1e-3)
    assert not ops.gemm_kernel_name(M, N, K, b_kc=False).startswith("gemm_tall_kernel")


@pytest.mark.parametrize("M", [256, 4096])
def test_siglip_mlp_row_pitch_bitwise(M):
    """SigLIP's 4304-wide MLP activations at the engine's 4352-element row pitch (engine.Engine._sig_rows):
    every GEMM that reads or writes them -- fc1 forward + GELU (output and saved pre-activation), fc2 forward
    (K = 4304: the K-tail clamps its loads into the row), the fc2 dgrad writing d(fc1 out), the fc1 dgrad and
    both weight gradients reading them -- gives bitwise the contiguous result, and the pad columns are neither
    read (NaN there changes nothing) nor written (they stay NaN)."""
    from pizero_native import ops

    D, F, P = 1152, 4304, 4352

    def padded(t):
        buf = torch.full((t.shape[0], P), float("nan"), device=dev, dtype=t.dtype)
        buf[:, :F].copy_(t)
        return buf, buf[:, :F]

    x, dy = bf(M, D), bf(M, D)
    w1, w2 = bf(F, D, scale=0.05), bf(D, F, scale=0.05)
    b1, b2 = bf(F), bf(D)
    # fc1 forward + GELU, output and pre-activation at the padded pitch
    h0, a0 = torch.empty(M, F, device=dev, dtype=torch.bfloat16), torch.empty(M, F, device=dev, dtype=torch.bfloat16)
    ops.linear(x, w1, h0, bias=b1, epi=ops.PZ_EPI_GELU, aux=a0)
    hb, h1 = padded(torch.zeros(M, F, device=dev, dtype=torch.bfloat16))
    ab, a1 = padded(torch.zeros(M, F, device=dev, dtype=torch.bfloat16))
    ops.linear(x, w1, h1, bias=b1, epi=ops.PZ_EPI_GELU, aux=a1)
    assert torch.equal(h1, h0) and torch.equal(a1, a0)
    assert torch.isnan(hb[:, F:].float()).all() and torch.isnan(ab[:, F:].float()).all()
    # fc2 forward reading the padded rows (K = 4304)
    y0, y1 = torch.empty(M, D, device=dev, dtype=torch.bfloat16), torch.empty(M, D, device=dev, dtype=torch.bfloat16)
    ops.linear(h0, w2, y0, bias=b2, resid=x)
    ops.linear(h1, w2, y1, bias=b2, resid=x)
    assert torch.equal(y1, y0)
    # fc2 dgrad into padded rows; fc1 dgrad and both weight gradients reading them
    g0 = torch.empty(M, F, device=dev, dtype=torch.bfloat16)
    ops.linear_dgrad(dy, w2, g0)
    gb, g1 = padded(torch.zeros(M, F, device=dev, dtype=torch.bfloat16))
    ops.linear_dgrad(dy, w2, g1)
    assert torch.equal(g1, g0) and torch.isnan(gb[:, F:].float()).all()
    d0, d1 = torch.empty(M, D, device=dev, dtype=torch.bfloat16), torch.empty(M, D, device=dev, dtype=torch.bfloat16)
    ops.linear_dgrad(g0, w1, d0)
    ops.linear_dgrad(g1, w1, d1)
    assert torch.equal(d1, d0)
    wg0, wg1 = torch.empty(D, F, device=dev, dtype=torch.bfloat16), torch.empty(D, F, device=dev, dtype=torch.bfloat16)
    ops.linear_wgrad(dy, h0, wg0)  # fc2 weight gradient: dy^T h
    ops.linear_wgrad(dy, h1, wg1)
    assert torch.equal(wg1, wg0)
    v0, v1 = torch.empty(F, D, device=dev, dtype=torch.bfloat16), torch.empty(F, D, device=dev, dtype=torch.bfloat16)
    ops.linear_wgrad(g0, x, v0)
    ops.linear_wgrad(g1, x, v1)
    assert torch.equal(v1, v0)


@pytest.mark.parametrize("case", ["long_k_narrow", "dgeglu", "geglu_fwd"])
def test_gemm_tile_order_group_bitwise(case, monkeypatch):
    """The 8-phase kernels' tile order (tile_coords super-row height: the planner takes 2 for narrow long-K GEMMs and
    the DGEGLU dgrad, 8 otherwise; PZ_GEMM_GROUP overrides) changes which workgroup computes a tile, never its
    arithmetic: every group height gives the same bits, also with a ragged last super-row (11 row tiles) and a split
    tail; against torch fp32 too."""
    from pizero_native import ops

    torch.manual_seed(3)
    outs = []
    for grp in ("", "8", "3", "1", "16"):
        monkeypatch.setenv("PZ_GEMM_GROUP", grp)
        torch.manual_seed(3)
        if case == "long_k_narrow":  # K >= 16384, <= 8 column tiles: group 2 by default
            M, N, K = 2816, 1024, 16384
            x, W = bf(M, K, scale=0.5), bf(N, K, scale=K ** -0.5)
            out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            ops.linear(x, W, out)
            ref = x.float() @ W.float().t()
        elif case == "dgeglu":  # down-proj dgrad with d(gate|up) in place over the saved g|u: group 2 by default
            M, I, H = 2816, 2048, 512
            dy, W = bf(M, H, scale=0.5), bf(H, I, scale=I ** -0.5)
            out = bf(M, 2 * I)
            ops.linear_dgrad(dy, W, out, epi=ops.PZ_EPI_DGEGLU, aux=out)
            ref = None
        else:  # GeGLU forward: group 8 by default
            M, K, I = 2816, 512, 1024
            x, W = bf(M, K), bf(2 * I, K, scale=K ** -0.5)
            out = torch.empty(M, I, device=dev, dtype=torch.bfloat16)
            ops.linear(x, W, out, epi=ops.PZ_EPI_GEGLU)
            r = x.float() @ W.float().t()
            ref = torch.nn.functional.gelu(r[:, :I], approximate="tanh") * r[:, I:]
        torch.cuda.synchronize()
        outs.append(out.clone())
        if ref is not None and grp == "":
            close(out, ref, atol=2e-2)
    for o in outs[1:]:
        assert torch.equal(o, outs[0])
