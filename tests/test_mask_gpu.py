"""General additive attention masks on the MI355X path against the fp32 oracle.

The reference adds whatever mask the caller passes to the soft-capped logits (joint_model.py:261-287).
The native PiZero validates each new mask: the Pi0 block pattern goes to the fused kernels (mask
regenerated from per-sample prefix counts), anything else to the GEMM + additive-softmax path
(pz_attn_softmax mask_mode 2).  Here the mask is NOT the block pattern -- the action rows cannot see
the proprio token and some image/text logits carry a finite -1.5 bias -- and loss, every gradient
(probe gate of tests/pizero_gpu_helpers.py) and the action chunk must match the oracle run on the
same mask.  (Parity is pinned through the oracle, itself pinned to the reference fixtures.)
"""

import numpy as np
import pytest
import torch

from tests.oracle_helpers import O, oracle_run
from tests.pizero_gpu_helpers import GRAD_COS, GRAD_REL, build_gpu_model, gpu_inputs, run_infer, run_loss

pytestmark = pytest.mark.gpu


def _edit(d):
    P, C = d["max_seq_len"], d["cond_steps"]

    def f(mask):
        lo = torch.finfo(torch.bfloat16).min  # the reference's bf16 masks (exactly representable in fp32)
        m = torch.where(mask < 0, torch.full_like(mask, lo), mask)
        m[:, :, P + C:, P] = lo  # action rows blind to proprio
        allowed = m[:, :, :P, :8] == 0
        m[:, :, :P, :8] = torch.where(allowed, torch.full_like(m[:, :, :P, :8], -1.5), m[:, :, :P, :8])
        return m
    return f


@pytest.fixture(scope="module")
def setup():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    d = O.TINY_DIMS
    ref, inp = oracle_run(d, 3, ragged=True, mask_fn=_edit(d))
    m = build_gpu_model(d)
    gi = gpu_inputs(m, d, 3)
    gm = ref["mask"].to(torch.bfloat16)
    assert torch.equal(gm.float(), ref["mask"])  # the edit is exact in bf16
    gi["causal_mask"] = gm.to("cuda")
    gi["itp"], gi["amask"] = [x.contiguous().to("cuda") for x in m.split_full_mask_into_submasks(gm)]
    return d, ref, m, gi


def test_general_mask_is_routed_to_general_path(setup):
    from pizero_native.engine import GeneralMask

    d, ref, m, gi = setup
    L = gi["causal_mask"].shape[-1]
    assert isinstance(m._mask_spec([gi["causal_mask"]], [torch.arange(L, device="cuda")]), GeneralMask)


@pytest.mark.parametrize("joint_attn", ["flash", "gemm", "probs"])
def test_general_mask_loss_and_grads(setup, joint_attn):
    from tests.golden.gradprobe import compare, probe

    d, ref, m, gi = setup
    eng = m._engine()
    prev = eng.joint_flash, eng.joint_probs
    # a general mask must take the GEMM path whatever the joint-attention mode
    eng.joint_flash, eng.joint_probs = joint_attn == "flash", joint_attn == "probs"
    try:
        loss = run_loss(m, gi).item()
    finally:
        eng.joint_flash, eng.joint_probs = prev
    assert abs(loss - ref["loss"]) <= 1e-2 * abs(ref["loss"]), (loss, ref["loss"])
    params = dict(m.named_parameters())
    bad = []
    for n, gref in ref["grads"].items():
        p = params.get(n)
        if p is None or gref is None or not p.requires_grad:
            continue
        rn = float(gref.double().norm())
        if rn == 0.0 or n.endswith("self_attn.k_proj.bias") and n.startswith("vision_tower"):
            continue  # SigLIP key bias: the exact gradient is 0 (softmax shift invariance), both are noise
        c = compare(probe(n, p.grad), probe(n, gref))
        if c["rel"] > GRAD_REL or c["cos"] < GRAD_COS:
            bad.append((n, c))
    assert not bad, bad


def test_general_mask_actions(setup):
    d, ref, m, gi = setup
    a = run_infer(m, gi, clip=False).float().cpu().numpy()
    err = np.abs(a - ref["actions"].numpy())
    assert err.mean() <= 5e-3 and err.max() <= 3e-2, (err.mean(), err.max())
    # and the mask really matters: the block-mask chunk differs
    blk = gpu_inputs(m, d, 3)
    b = run_infer(m, blk, clip=False).float().cpu().numpy()
    assert np.abs(b - a).max() > 1e-2
