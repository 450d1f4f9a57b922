"""Fused (flash) attention kernels vs a plain PyTorch fp32 reference of the same attention.

SigLIP shape (siglip.py:108-166: 16 heads x 72, 256 tokens, no mask) read in place from the fused
q|k|v rows, and the joint MQA shape (joint_model.py:130-304: 8 query heads stacked as rows, one
K/V head of 256, soft-cap 50, Pi0 block mask incl. pad rows, pizero.py:271-306) scattered into
per-mixture output buffers.  Tolerance: P is rounded to bf16 before the PV product (as the
reference's autocast softmax(...).to(bf16) does), outputs are bf16: ~1e-2 relative.
"""

import math

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


def close(out, ref, rtol=2e-2, atol=2e-2):
    out, ref = out.float(), ref.float()
    err = (out - ref).abs()
    bad = (err > atol + rtol * ref.abs()).sum().item()
    assert bad == 0, f"{bad} mismatches, max err {err.max().item():.4g}"


def joint_mask(cnt, P, C, L):
    """[B, L, L] bool allowed + [B, L] dead-row flags (pizero.py:271-306 semantics)."""
    B = len(cnt)
    i = torch.arange(L).view(L, 1)
    j = torch.arange(L).view(1, L)
    allowed = torch.zeros(B, L, L, dtype=torch.bool)
    dead = torch.zeros(B, L, dtype=torch.bool)
    for b, c in enumerate(cnt):
        vlm = (i < P) & (i < c) & (j < c)
        prop = (i >= P) & (i < P + C) & ((j < c) | ((j >= P) & (j < P + C)))
        act = (i >= P + C) & ((j < c) | (j >= P))
        allowed[b] = vlm | prop | act
        dead[b] = (torch.arange(L) < P) & (torch.arange(L) >= c)
    return allowed, dead


def ref_attention(q, k, v, scale, cap=0.0, allowed=None, dead=None):
    """q [B, H, Lq, D], k/v [B, H, Lk, D] fp32; allowed [B, Lq, Lk]; dead [B, Lq] -> uniform rows"""
    s = (q @ k.transpose(-1, -2)) * scale
    if cap > 0:
        s = cap * torch.tanh(s / cap)
    if allowed is not None:
        s = s.masked_fill(~allowed[:, None], float("-inf"))
        s = torch.where(dead[:, None, :, None], torch.zeros_like(s), s)
    lse = torch.logsumexp(s, -1)
    p = torch.softmax(s, -1)
    return p @ v, lse


@pytest.mark.parametrize("unit,sig,B", [("0", "0", 3), ("1", "0", 3), ("1", "1", 3), ("1", "1", 40)])
def test_flash_fwd_siglip(unit, sig, B, monkeypatch):
    """the SigLIP forward kernel families: 2 workgroups per unit (few units), one workgroup per unit, and the
    persistent pipelined kernel (B = 40: 640 units over the CUs, several units per workgroup with a ragged
    last round, XCD-grouped unit order)"""
    from pizero_native import ops

    monkeypatch.setenv("PZ_FLASH_UNIT", unit)
    monkeypatch.setenv("PZ_FLASH_SIG", sig)

    nh, hd, N = 16, 72, 256
    qkv = (torch.randn(B * N, 3 * nh * hd, device=dev) * 1.5).to(torch.bfloat16)
    O = torch.empty(B * N, nh * hd, device=dev, dtype=torch.bfloat16)
    lse = torch.empty(B * nh, N, device=dev)
    ops.flash_fwd(ops.siglip_flash_args(qkv, O, lse, B, nh, hd, N))
    x = qkv.float().view(B, N, 3, nh, hd).permute(2, 0, 3, 1, 4)  # [3, B, nh, N, hd]
    ref, rlse = ref_attention(x[0], x[1], x[2], hd ** -0.5)
    close(O.view(B, N, nh, hd).permute(0, 2, 1, 3), ref)
    close(lse.view(B, nh, N), rlse, rtol=1e-3, atol=1e-3)


@pytest.mark.parametrize("key_split", [False, True])
@pytest.mark.parametrize("cnt", [[276, 276, 276], [276, 250, 9]])
def test_flash_fwd_joint_block_mask(cnt, key_split):
    from pizero_native import ops

    B, P, C, Hc, nh, hd = len(cnt), 276, 1, 4, 8, 256
    L = P + C + Hc
    Lp = (L + 7) // 8 * 8
    Q = (torch.randn(B, L * nh, hd, device=dev) * 2).to(torch.bfloat16)
    K = torch.zeros(B, Lp, hd, device=dev, dtype=torch.bfloat16)
    V = torch.zeros(B, Lp, hd, device=dev, dtype=torch.bfloat16)
    K[:, :L] = (torch.randn(B, L, hd, device=dev) * 2).to(torch.bfloat16)
    V[:, :L] = torch.randn(B, L, hd, device=dev).to(torch.bfloat16)
    Ov = torch.empty(B * P, nh * hd, device=dev, dtype=torch.bfloat16)
    Oe = torch.empty(B * (C + Hc), nh * hd, device=dev, dtype=torch.bfloat16)
    lse = torch.empty(B, L * nh, device=dev)
    cnt_t = torch.tensor(cnt, device=dev, dtype=torch.int32)
    a = ops.flash_args(B, 1, L * nh, L, hd, Q, (hd, L * nh * hd, 0), K, (hd, Lp * hd, 0), V, (hd, Lp * hd, 0),
                       [(0, Ov, P * nh * hd, hd), (P * nh, Oe, (C + Hc) * nh * hd, hd)], 0, lse, 1 / math.sqrt(hd),
                       cap=50.0, mask_mode=1, cnt=cnt_t, prefix=P, cond=C, rows_per_token=nh, key_split=key_split)
    ops.flash_fwd(a)
    allowed, dead = joint_mask(cnt, P, C, L)
    q = Q.float().view(B, L, nh, hd).permute(0, 2, 1, 3)
    k = K.float()[:, None, :L]
    v = V.float()[:, None, :L]
    ref, rlse = ref_attention(q, k, v, 1 / math.sqrt(hd), 50.0, allowed.to(dev), dead.to(dev))
    ref = ref.permute(0, 2, 1, 3)  # [B, L, nh, hd]
    close(Ov.view(B, P, nh, hd), ref[:, :P])
    close(Oe.view(B, C + Hc, nh, hd), ref[:, P:])
    close(lse.view(B, L, nh), rlse.permute(0, 2, 1), rtol=1e-3, atol=2e-3)


@pytest.mark.parametrize("cnt", [[276, 276, 276], [276, 250, 9]])
def test_flash_fwd_probs_joint_block_mask(cnt):
    """pz_flash_fwd_probs (training-default joint forward): O, and the exported bf16 softmax P and
    tanh(cap) with pz_attn_softmax's conventions (dead rows uniform over L keys with tcap 0, zeros in
    the L..Lp pad columns), against torch fp32 (the LDS-DMA ring kernel)"""
    from pizero_native import ops

    B, P, C, Hc, nh, hd = len(cnt), 276, 1, 4, 8, 256
    L = P + C + Hc
    Lp = (L + 7) // 8 * 8
    Q = (torch.randn(B, L * nh, hd, device=dev) * 2).to(torch.bfloat16)
    K = torch.zeros(B, Lp, hd, device=dev, dtype=torch.bfloat16)
    V = torch.zeros(B, Lp, hd, device=dev, dtype=torch.bfloat16)
    K[:, :L] = (torch.randn(B, L, hd, device=dev) * 2).to(torch.bfloat16)
    V[:, :L] = torch.randn(B, L, hd, device=dev).to(torch.bfloat16)
    Ov = torch.empty(B * P, nh * hd, device=dev, dtype=torch.bfloat16)
    Oe = torch.empty(B * (C + Hc), nh * hd, device=dev, dtype=torch.bfloat16)
    Pm = torch.full((B, L * nh, Lp), float("nan"), device=dev, dtype=torch.bfloat16)
    tc = torch.full_like(Pm, float("nan"))
    cnt_t = torch.tensor(cnt, device=dev, dtype=torch.int32)
    a = ops.flash_args(B, 1, L * nh, L, hd, Q, (hd, L * nh * hd, 0), K, (hd, Lp * hd, 0), V, (hd, Lp * hd, 0),
                       [(0, Ov, P * nh * hd, hd), (P * nh, Oe, (C + Hc) * nh * hd, hd)], 0, None, 1 / math.sqrt(hd),
                       cap=50.0, mask_mode=1, cnt=cnt_t, prefix=P, cond=C, rows_per_token=nh)
    ops.flash_fwd_probs(a, Pm, tc, Lp)
    allowed, dead = joint_mask(cnt, P, C, L)
    allowed, dead = allowed.to(dev), dead.to(dev)
    q = Q.float().view(B, L, nh, hd).permute(0, 2, 1, 3)
    k = K.float()[:, None, :L]
    v = V.float()[:, None, :L]
    ref, _ = ref_attention(q, k, v, 1 / math.sqrt(hd), 50.0, allowed, dead)
    ref = ref.permute(0, 2, 1, 3)
    close(Ov.view(B, P, nh, hd), ref[:, :P])
    close(Oe.view(B, C + Hc, nh, hd), ref[:, P:])
    s = (q @ k.transpose(-1, -2)) / math.sqrt(hd)  # [B, nh, L, L]
    th = torch.tanh(s / 50.0)
    x = (50.0 * th).masked_fill(~allowed[:, None], float("-inf"))
    pr = torch.softmax(x, -1)
    pr = torch.where(dead[:, None, :, None], torch.full_like(pr, 1.0 / L), pr)
    th = torch.where(dead[:, None, :, None], torch.zeros_like(th), th)
    got_p = Pm.float().view(B, L, nh, Lp).permute(0, 2, 1, 3)
    got_t = tc.float().view(B, L, nh, Lp).permute(0, 2, 1, 3)
    close(got_p[..., :L], pr, rtol=1e-2, atol=1e-3)
    close(got_t[..., :L], th, rtol=1e-2, atol=2e-3)
    assert (got_p[..., L:] == 0).all() and (got_t[..., L:] == 0).all()
    # rows sum to 1 within bf16 rounding
    assert (got_p.sum(-1) - 1).abs().max().item() < 2e-2


@pytest.mark.parametrize("skip_action", [False, True])
def test_flash_bwd_ds_matches_softmax_backward(skip_action):
    """pz_flash_bwd_ds (dP = dO V^T in registers + the soft-cap softmax backward from the exported P /
    tanh(cap)) against torch fp32 of pz_attn_softmax_bwd's formula on the same P / tcap; a mixture
    without dO (the last layer's skipped prefix) contributes dP = 0"""
    from pizero_native import ops

    cnt = [276, 250]
    B, P, C, Hc, nh, hd = len(cnt), 276, 1, 4, 8, 256
    L = P + C + Hc
    Lp = (L + 7) // 8 * 8
    Q = (torch.randn(B, L * nh, hd, device=dev) * 2).to(torch.bfloat16)
    K = torch.zeros(B, Lp, hd, device=dev, dtype=torch.bfloat16)
    V = torch.zeros(B, Lp, hd, device=dev, dtype=torch.bfloat16)
    K[:, :L] = (torch.randn(B, L, hd, device=dev) * 2).to(torch.bfloat16)
    V[:, :L] = torch.randn(B, L, hd, device=dev).to(torch.bfloat16)
    Ov = torch.empty(B * P, nh * hd, device=dev, dtype=torch.bfloat16)
    Oe = torch.empty(B * (C + Hc), nh * hd, device=dev, dtype=torch.bfloat16)
    dOv = torch.randn(B * P, nh * hd, device=dev).to(torch.bfloat16)
    dOe = torch.randn(B * (C + Hc), nh * hd, device=dev).to(torch.bfloat16)
    Pm = torch.empty(B, L * nh, Lp, device=dev, dtype=torch.bfloat16)
    tc = torch.empty_like(Pm)
    dS = torch.full_like(Pm, float("nan"))
    cnt_t = torch.tensor(cnt, device=dev, dtype=torch.int32)
    groups = [(0, Ov, P * nh * hd, hd), (P * nh, Oe, (C + Hc) * nh * hd, hd)]
    kw = dict(cap=50.0, mask_mode=1, cnt=cnt_t, prefix=P, cond=C, rows_per_token=nh)
    a = ops.flash_args(B, 1, L * nh, L, hd, Q, (hd, L * nh * hd, 0), K, (hd, Lp * hd, 0), V, (hd, Lp * hd, 0), groups,
                       0, None, 1 / math.sqrt(hd), **kw)
    ops.flash_fwd_probs(a, Pm, tc, Lp)
    dgroups = [dOv, None] if skip_action else [dOv, dOe]
    a = ops.flash_args(B, 1, L * nh, L, hd, Q, (hd, L * nh * hd, 0), K, (hd, Lp * hd, 0), V, (hd, Lp * hd, 0), groups,
                       0, None, 1 / math.sqrt(hd), dgroups=dgroups, **kw)
    ops.flash_bwd_ds(a, Pm, tc, dS, Lp)
    dO = torch.cat([dOv.float().view(B, P * nh, hd),
                    (torch.zeros_like(dOe) if skip_action else dOe).float().view(B, (C + Hc) * nh, hd)], 1)
    dP = dO @ V.float().transpose(1, 2)  # [B, L*nh, Lp]
    p, t = Pm.float(), tc.float()
    dot = (p[..., :L] * dP[..., :L]).sum(-1, keepdim=True)
    ref = p * (dP - dot) / math.sqrt(hd) * (1 - t * t)
    ref[..., L:] = 0
    close(dS, ref, rtol=2e-2, atol=2e-2 * ref.abs().max().item() / 8)
    assert (dS[..., L:] == 0).all()
    # with dq: the same dS plus dQ = dS K (the bf16 dS the batched dQ GEMM would read)
    dS2 = torch.full_like(Pm, float("nan"))
    dQ = torch.full_like(Q, float("nan"))
    a = ops.flash_args(B, 1, L * nh, L, hd, Q, (hd, L * nh * hd, 0), K, (hd, Lp * hd, 0), V, (hd, Lp * hd, 0), groups,
                       0, None, 1 / math.sqrt(hd), dgroups=dgroups, dq=dQ, **kw)
    ops.flash_bwd_ds(a, Pm, tc, dS2, Lp)
    assert torch.equal(dS2, dS)
    refq = dS.float() @ K.float()
    close(dQ, refq, rtol=2e-2, atol=2e-2 * refq.abs().max().item() / 8)



@pytest.mark.parametrize("B,cnt", [(1, [276]), (2, [276, 100])])
def test_flash_fwd_denoise_key_split(B, cnt):
    """Inference denoise shape: only the action rows query (mask_row0 = first action row), keys =
    the cached prefix + proprio + the chunk; the key-split forward (one workgroup per key block +
    merge) against the fp32 reference."""
    from pizero_native import ops

    P, C, Hc, nh, hd = 276, 1, 4, 8, 256
    L = P + C + Hc
    Lp = (L + 7) // 8 * 8
    Q = (torch.randn(B, Hc * nh, hd, device=dev) * 2).to(torch.bfloat16)
    K = torch.zeros(B, Lp, hd, device=dev, dtype=torch.bfloat16)
    V = torch.zeros(B, Lp, hd, device=dev, dtype=torch.bfloat16)
    K[:, :L] = (torch.randn(B, L, hd, device=dev) * 2).to(torch.bfloat16)
    V[:, :L] = torch.randn(B, L, hd, device=dev).to(torch.bfloat16)
    O = torch.full((B * Hc, nh * hd), float("nan"), device=dev, dtype=torch.bfloat16)
    cnt_t = torch.tensor(cnt, device=dev, dtype=torch.int32)
    a = ops.flash_args(B, 1, Hc * nh, L, hd, Q, (hd, Hc * nh * hd, 0), K, (hd, Lp * hd, 0), V, (hd, Lp * hd, 0),
                       [(0, O, Hc * nh * hd, hd)], 0, None, 1 / math.sqrt(hd), cap=50.0, mask_mode=1, cnt=cnt_t,
                       prefix=P, cond=C, rows_per_token=nh, mask_row0=(P + C) * nh, key_split=True)
    ops.flash_fwd(a)
    allowed, dead = joint_mask(cnt, P, C, L)
    q = Q.float().view(B, Hc, nh, hd).permute(0, 2, 1, 3)
    ref, _ = ref_attention(q, K.float()[:, None, :L], V.float()[:, None, :L], 1 / math.sqrt(hd), 50.0,
                           allowed[:, P + C:].to(dev), dead[:, P + C:].to(dev))
    close(O.view(B, Hc, nh, hd), ref.permute(0, 2, 1, 3))


def _grads(q, k, v, dO, scale, cap=0.0, allowed=None, dead=None):
    q, k, v = (t.detach().clone().requires_grad_() for t in (q, k, v))
    o, _ = ref_attention(q, k, v, scale, cap, allowed, dead)
    o.backward(dO)
    return q.grad, k.grad, v.grad


@pytest.mark.parametrize("unit,sig,B", [("0", "0", 2), ("1", "0", 2), ("1", "1", 2), ("1", "1", 40)])
def test_flash_bwd_siglip(unit, sig, B, monkeypatch):
    from pizero_native import ops

    monkeypatch.setenv("PZ_FLASH_UNIT", unit)
    monkeypatch.setenv("PZ_FLASH_SIG", sig)

    nh, hd, N = 16, 72, 256
    qkv = (torch.randn(B * N, 3 * nh * hd, device=dev) * 1.5).to(torch.bfloat16)
    O = torch.empty(B * N, nh * hd, device=dev, dtype=torch.bfloat16)
    lse = torch.empty(B * nh, N, device=dev)
    ops.flash_fwd(ops.siglip_flash_args(qkv, O, lse, B, nh, hd, N))
    dO = torch.randn(B * N, nh * hd, device=dev).to(torch.bfloat16)
    delta = torch.empty(B * nh, N, device=dev)
    dqkv = torch.full_like(qkv, float("nan"))
    ops.flash_bwd(ops.siglip_flash_args(qkv, O, lse, B, nh, hd, N, dO=dO, delta=delta, dqkv=dqkv))
    x = qkv.float().view(B, N, 3, nh, hd).permute(2, 0, 3, 1, 4)
    g = dO.float().view(B, N, nh, hd).permute(0, 2, 1, 3)
    dq, dk, dv = _grads(x[0], x[1], x[2], g, hd ** -0.5)
    got = dqkv.float().view(B, N, 3, nh, hd).permute(2, 0, 3, 1, 4)
    for out, ref in ((got[0], dq), (got[1], dk), (got[2], dv)):
        close(out, ref, rtol=3e-2, atol=3e-2 * ref.abs().max().item() / 4)


@pytest.mark.parametrize("cnt", [[276, 276], [276, 9]])
def test_flash_bwd_joint_block_mask(cnt):
    from pizero_native import ops

    B, P, C, Hc, nh, hd = len(cnt), 276, 1, 4, 8, 256
    L = P + C + Hc
    Lp = (L + 7) // 8 * 8
    Q = (torch.randn(B, L * nh, hd, device=dev) * 2).to(torch.bfloat16)
    K = torch.zeros(B, Lp, hd, device=dev, dtype=torch.bfloat16)
    V = torch.zeros(B, Lp, hd, device=dev, dtype=torch.bfloat16)
    K[:, :L] = (torch.randn(B, L, hd, device=dev) * 2).to(torch.bfloat16)
    V[:, :L] = torch.randn(B, L, hd, device=dev).to(torch.bfloat16)
    Ov = torch.empty(B * P, nh * hd, device=dev, dtype=torch.bfloat16)
    Oe = torch.empty(B * (C + Hc), nh * hd, device=dev, dtype=torch.bfloat16)
    dOv = torch.randn(B * P, nh * hd, device=dev).to(torch.bfloat16)
    dOe = torch.randn(B * (C + Hc), nh * hd, device=dev).to(torch.bfloat16)
    cnt_t = torch.tensor(cnt, device=dev, dtype=torch.int32)
    # the pad rows' outputs reach nothing downstream in the model (no row attends to them), so their dO is 0
    allowed, dead = joint_mask(cnt, P, C, L)
    dOv.view(B, P, nh * hd)[dead[:, :P].to(dev)] = 0
    lse = torch.empty(B, L * nh, device=dev)
    delta = torch.empty(B, L * nh, device=dev)
    dQ = torch.full_like(Q, float("nan"))
    dK = torch.zeros_like(K)
    dV = torch.zeros_like(V)
    groups = [(0, Ov, P * nh * hd, hd), (P * nh, Oe, (C + Hc) * nh * hd, hd)]
    a = ops.flash_args(B, 1, L * nh, L, hd, Q, (hd, L * nh * hd, 0), K, (hd, Lp * hd, 0), V, (hd, Lp * hd, 0),
                       groups, 0, lse, 1 / math.sqrt(hd), cap=50.0, mask_mode=1, cnt=cnt_t, prefix=P, cond=C,
                       rows_per_token=nh, dgroups=[dOv, dOe], delta=delta, dq=dQ, dk=dK, dv=dV)
    ops.flash_fwd(a)
    ops.flash_bwd(a)
    q = Q.float().view(B, L, nh, hd).permute(0, 2, 1, 3)
    g = torch.cat([dOv.float().view(B, P, nh, hd), dOe.float().view(B, C + Hc, nh, hd)], 1).permute(0, 2, 1, 3)
    kk = K.float()[:, None, :L].expand(B, nh, L, hd)
    vv = V.float()[:, None, :L].expand(B, nh, L, hd)
    dq, dk, dv = _grads(q, kk, vv, g, 1 / math.sqrt(hd), 50.0, allowed.to(dev), dead.to(dev))
    close(dQ.float().view(B, L, nh, hd).permute(0, 2, 1, 3), dq, atol=3e-2 * dq.abs().max().item() / 4)
    close(dK.float()[:, :L], dk.sum(1), atol=3e-2 * dk.abs().max().item())
    close(dV.float()[:, :L], dv.sum(1), atol=3e-2 * dv.abs().max().item())


@pytest.mark.parametrize("B", [2, 40])
def test_flash_bwd_siglip_poisoned_lds(B, monkeypatch):
    """The persistent SigLIP kernels with every CU's LDS filled with NaN before each launch (pz_debug_poison_lds):
    B = 2 gives 32 units over 32 workgroups, so each workgroup's second LDS buffer is never written -- round 5's dQ
    kernel read row 255 of buffer 0's V image on into it (0 x NaN = NaN).  Outputs must be finite and
    bitwise equal to an unpoisoned run."""
    from pizero_native import _lib, ops

    monkeypatch.setenv("PZ_FLASH_UNIT", "1")
    monkeypatch.setenv("PZ_FLASH_SIG", "1")
    nh, hd, N = 16, 72, 256
    qkv = (torch.randn(B * N, 3 * nh * hd, device=dev) * 1.5).to(torch.bfloat16)
    dO = torch.randn(B * N, nh * hd, device=dev).to(torch.bfloat16)

    def run():
        O = torch.full((B * N, nh * hd), float("nan"), device=dev, dtype=torch.bfloat16)
        lse = torch.full((B * nh, N), float("nan"), device=dev)
        delta = torch.full((B * nh, N), float("nan"), device=dev)
        dqkv = torch.full_like(qkv, float("nan"))
        ops.flash_fwd(ops.siglip_flash_args(qkv, O, lse, B, nh, hd, N))
        ops.flash_bwd(ops.siglip_flash_args(qkv, O, lse, B, nh, hd, N, dO=dO, delta=delta, dqkv=dqkv))
        torch.cuda.synchronize()
        return O, lse, dqkv

    ref = run()
    _lib.set_poison_lds(0xFFFFFFFF)
    try:
        got = run()
    finally:
        _lib.set_poison_lds(None)
    for r, g in zip(ref, got):
        assert bool(torch.isfinite(g.float()).all())
        assert torch.equal(r, g)


def test_flash_siglip_persistent_repeat_bitwise(monkeypatch):
    """The persistent SigLIP kernels take their units from self-resetting per-XCD ticket counters (FsTickets): launches
    of different unit counts back to back (B = 40, 2, 17 -- 17 images leave XCDs with 3 and 2 images, 2 leave six
    XCDs without work) and a hipGraph replay must all reproduce each shape's first result bitwise"""
    from pizero_native import ops

    monkeypatch.setenv("PZ_FLASH_UNIT", "1")
    monkeypatch.setenv("PZ_FLASH_SIG", "1")
    nh, hd, N = 16, 72, 256
    data = {}
    for B in (40, 2, 17):
        qkv = (torch.randn(B * N, 3 * nh * hd, device=dev) * 1.5).to(torch.bfloat16)
        dO = torch.randn(B * N, nh * hd, device=dev).to(torch.bfloat16)
        data[B] = (qkv, dO)

    def run(B):
        qkv, dO = data[B]
        O = torch.empty(B * N, nh * hd, device=dev, dtype=torch.bfloat16)
        lse = torch.empty(B * nh, N, device=dev)
        delta = torch.empty(B * nh, N, device=dev)
        dqkv = torch.empty_like(qkv)
        ops.flash_fwd(ops.siglip_flash_args(qkv, O, lse, B, nh, hd, N))
        ops.flash_bwd(ops.siglip_flash_args(qkv, O, lse, B, nh, hd, N, dO=dO, delta=delta, dqkv=dqkv))
        return O, lse, dqkv

    first = {B: [t.clone() for t in run(B)] for B in (40, 2, 17)}
    for B in (17, 40, 2, 40, 17):
        for r, g in zip(first[B], run(B)):
            assert torch.equal(r, g), B
    # B = 17 itself against the fp32 reference (units of the uneven XCD split all computed, none twice)
    qkv, dO = data[17]
    x = qkv.float().view(17, N, 3, nh, hd).permute(2, 0, 3, 1, 4)
    ref, _ = ref_attention(x[0], x[1], x[2], hd ** -0.5)
    close(first[17][0].view(17, N, nh, hd).permute(0, 2, 1, 3), ref)
    # captured into a hipGraph and replayed twice
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        run(40)
    torch.cuda.current_stream().wait_stream(s)
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        outs = run(40)
    for _ in range(2):
        gr.replay()
        torch.cuda.synchronize()
        for r, g in zip(first[40], outs):
            assert torch.equal(r, g)
