"""End-to-end parity of the native MI355X PiZero against the reference fixtures.

The fixtures (tests/golden/{tiny,full,b16}.npz, written by tests/golden/make_golden.py, which
imports and runs the REFERENCE) hold its fp32 loss, cached and naive action chunks and, for EVERY
parameter, a gradient summary (tests/golden/gradprobe.py: norm, ~4096 seeded samples incl. the
last row / last column tile tails, 2 whole-tensor Rademacher projections), plus the reference's own
bf16-vs-fp32 deviation for the same inputs.

The HIP path runs in bf16 (fp32 accumulation) and is held to SURVEY 8(c)'s gate against the fp32
reference:
  * loss:    |d| <= max(3x the reference's own bf16 deviation, 1e-2 rel);
  * grads:   per tensor sample rel-L2 <= 8 % and cosine >= 0.995, |norm| rel <= 8 %, projections
             within 5 x 8 % of |g| -- widened to 2x the reference's own bf16 deviation for the few
             tensors where that is larger (pizero_gpu_helpers.grad_tolerance);
  * actions: mean|d| <= max(3x dev, 5e-3), max|d| <= max(3x dev, 3e-2).
Shapes: tiny (B=3), bridge B=2 (full), bridge B=16 (config C2's micro-batch) and the benched
micro-batch 64 (the 16 fixture samples x 4: the batch mean makes its loss and gradients equal to
the B=16 fixture's, so the bench's M = 17664-row GEMM instantiations and split tails are checked
end to end).
"""

import numpy as np
import pytest
import torch

from tests.oracle_helpers import O, load_golden
from tests.pizero_gpu_helpers import build_gpu_model, check_grads_probe, gpu_inputs, run_infer, run_loss

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _check_loss(g, loss):
    ref, rb = float(g["fp32/loss"]), float(g["bf16/loss"])
    tol = max(3 * abs(rb - ref), 1e-2 * abs(ref))
    assert abs(loss - ref) <= tol, (loss, ref, rb)


def _check_grads(g, m, label):
    return check_grads_probe(g, dict(m.named_parameters()), label=label)


def _check_actions(g, a, key, sel=None):
    ref = g[f"fp32/{key}"]
    rb = g[f"bf16/{key}"]
    if sel is not None:  # a sub-batch of the fixture's samples (samples are independent)
        ref, rb = ref[list(sel)], rb[list(sel)]
    a = a.float().cpu().numpy()
    assert a.shape == ref.shape, (a.shape, ref.shape)
    dev = np.abs(rb - ref)
    err = np.abs(a - ref)
    assert err.mean() <= max(3 * dev.mean(), 5e-3), (err.mean(), dev.mean())
    assert err.max() <= max(3 * dev.max(), 3e-2), (err.max(), dev.max())


@pytest.fixture(scope="module")
def tiny():
    d = O.TINY_DIMS
    g = load_golden("tiny")
    m = build_gpu_model(d)
    gi = gpu_inputs(m, d, int(g["bsz"]))
    return d, g, m, gi


def test_tiny_loss_and_grads(tiny):
    d, g, m, gi = tiny
    loss = run_loss(m, gi)
    _check_loss(g, loss.item())
    _check_grads(g, m, "tiny")


def test_tiny_grad_accumulation_and_zero(tiny):
    d, g, m, gi = tiny
    run_loss(m, gi)
    g1 = m.action_decoder.weight.grad.float().clone()
    run_loss(m, gi, accumulate=True)
    g2 = m.action_decoder.weight.grad.float().clone()
    assert torch.allclose(g2, 2 * g1, rtol=2e-2, atol=1e-3)
    m.zero_grad(set_to_none=True)
    assert m.action_decoder.weight.grad is None


def test_tiny_actions(tiny):
    d, g, m, gi = tiny
    a = run_infer(m, gi, clip=False)
    _check_actions(g, a, "actions_unclipped")
    a2 = m.infer_action_naive(input_ids=gi["input_ids"], pixel_values=gi["pixel_values"].float(),
                              causal_mask=gi["causal_mask"], vlm_position_ids=gi["vpos"],
                              proprio_position_ids=gi["ppos"], action_position_ids=gi["apos"],
                              proprios=gi["proprios"], noise=gi["noise"], clip=False)
    _check_actions(g, a2, "actions_naive_unclipped")
    a3 = run_infer(m, gi, clip=True)
    assert a3.abs().max().item() <= 1.0


@pytest.fixture(scope="module")
def full_model():
    return build_gpu_model(O.FULL_DIMS)


@pytest.fixture(scope="module")
def full(full_model):
    d = O.FULL_DIMS
    g = load_golden("full")
    gi = gpu_inputs(full_model, d, int(g["bsz"]))
    return d, g, full_model, gi


def test_full_loss_and_grads(full):
    d, g, m, gi = full
    loss = run_loss(m, gi)
    _check_loss(g, loss.item())
    _check_grads(g, m, "full B=2")


def test_full_actions(full):
    d, g, m, gi = full
    a = run_infer(m, gi, clip=False)
    _check_actions(g, a, "actions_unclipped")
    a3 = run_infer(m, gi, clip=True)
    np.testing.assert_allclose(a3.float().cpu().numpy(), np.clip(a.float().cpu().numpy(), -1, 1), atol=1e-2)


def test_full_actions_hipgraph(full):
    """The hipGraph-captured chunk (pizero_native/graph.py) at bridge size against the reference."""
    from pizero_native.graph import InferenceGraph

    d, g, m, gi = full
    B = int(g["bsz"])
    ig = InferenceGraph(m, B, clip=False)
    ig.load(gi["input_ids"], gi["pixel_values"], m.block_prefix_counts(gi["itp"], gi["amask"]), gi["vpos"], gi["ppos"], gi["apos"],
            gi["proprios"].float(), gi["noise"])
    ig.capture()
    for _ in range(3):  # replays are idempotent (static inputs, KV rewritten by each prefill)
        a = ig.replay()
    torch.cuda.synchronize()
    _check_actions(g, a.clone(), "actions_unclipped")
    eager = run_infer(m, gi, clip=False)
    assert torch.equal(a.float(), eager.float()), float((a.float() - eager.float()).abs().max())


@pytest.mark.parametrize("sample", [0, 1])
def test_full_actions_b1_benched_config(full_model, sample):
    """Config C4 as benched (bench.py: B=1, eager infer_action AND the hipGraph replay it times) against
    the reference: sample ``sample`` of full.npz run alone must reproduce the fixture's actions for that
    sample (pizero.py:416-490 treats samples independently).  B=1 routes the prefill's 256-row SigLIP and
    276-row Gemma GEMMs and the 4-row denoise GEMVs through other kernels / split counts than B=2."""
    from pizero_native.graph import InferenceGraph

    d = O.FULL_DIMS
    g = load_golden("full")
    m = full_model
    gi = gpu_inputs(m, d, int(g["bsz"]), select=[sample])
    assert gi["input_ids"].shape[0] == 1
    a = run_infer(m, gi, clip=False)
    _check_actions(g, a, "actions_unclipped", sel=[sample])
    ig = InferenceGraph(m, 1, clip=False)
    ig.load(gi["input_ids"], gi["pixel_values"], m.block_prefix_counts(gi["itp"], gi["amask"]), gi["vpos"], gi["ppos"],
            gi["apos"], gi["proprios"].float(), gi["noise"])
    ig.capture()
    for _ in range(2):
        ag = ig.replay()
    torch.cuda.synchronize()
    _check_actions(g, ag.clone(), "actions_unclipped", sel=[sample])
    assert torch.equal(ag.float(), a.float()), float((ag.float() - a.float()).abs().max())


def test_fused_denoise_glue_bitwise(full_model, monkeypatch):
    """pz_action_in / pz_action_out (a denoise step's cast + action Linear + time embedding, and final RMSNorm +
    action decoder + Euler update, two launches instead of six) give the same action chunk bit for bit as the
    separate kernels (PZ_FUSED_GLUE=0), at the benched B=1 and at B=2 (the fused path is the default).  The
    fused path also folds the joint model's sqrt(hidden) = 32 input scale into the action encoder's last Linear
    (alpha + a pre-scaled bias) where PZ_FUSED_GLUE=0 scales the rows in a separate launch."""
    d = O.FULL_DIMS
    g = load_golden("full")
    m = full_model
    for sel in ([0], None):
        gi = gpu_inputs(m, d, int(g["bsz"]), select=sel)
        outs = []
        for fused in ("1", "0"):
            monkeypatch.setenv("PZ_FUSED_GLUE", fused)
            outs.append(run_infer(m, gi, clip=False).float().clone())
        torch.cuda.synchronize()
        assert torch.equal(outs[0], outs[1]), float((outs[0] - outs[1]).abs().max())


def test_full_actions_fp8(full):
    """Config C5's fp8 inference (PiZero.use_fp8_inference: e4m3 weights with per-tensor scales; prefill
    GEMMs W8A8 on the fp8 MFMA with per-row activation scales, denoise rows W8A16) at bridge size
    against the reference's fp32 action chunk.  Parity vs an fp8 reference is unpinned (the reference
    has no fp8 path): the gate is the bf16 action tolerance widened 2x (fp8 e4m3 keeps 3 mantissa bits
    against bf16's 7), and the measured deviation is printed."""
    from pizero_native.graph import InferenceGraph

    d, g, m, gi = full
    ref = g["fp32/actions_unclipped"]
    dev = np.abs(g["bf16/actions_unclipped"] - ref)
    a16 = run_infer(m, gi, clip=False).float().cpu().numpy()
    try:
        m.use_fp8_inference(True)
        a8 = run_infer(m, gi, clip=False)
        e8, e16 = np.abs(a8.float().cpu().numpy() - ref), np.abs(a16 - ref)
        print(f"fp8 actions: mean|d| {e8.mean():.4g} max {e8.max():.4g}; bf16 {e16.mean():.4g} / {e16.max():.4g}; "
              f"reference bf16 {dev.mean():.4g} / {dev.max():.4g}")
        assert e8.mean() <= 2 * max(3 * dev.mean(), 5e-3), (e8.mean(), dev.mean())
        assert e8.max() <= 2 * max(3 * dev.max(), 3e-2), (e8.max(), dev.max())
        B = int(g["bsz"])
        ig = InferenceGraph(m, B, clip=False)
        ig.load(gi["input_ids"], gi["pixel_values"], m.block_prefix_counts(gi["itp"], gi["amask"]), gi["vpos"],
                gi["ppos"], gi["apos"], gi["proprios"].float(), gi["noise"])
        ig.capture()
        a = ig.replay()
        torch.cuda.synchronize()
        assert torch.equal(a.float(), a8.float())
    finally:
        m.use_fp8_inference(False)


def test_fp8_codes_follow_weight_changes(full):
    """the fp8 weight copies are re-quantised when the weights change after use_fp8_inference
    (an in-place write through a parameter, e.g. load_state_dict; FusedAdamW.step bumps the same version
    counter after its raw-pointer kernel writes): eager and hipGraph inference then equal a fresh
    prepare on the new weights, never the stale codes.  The action encoder's last bias also changes: the
    graph reads an alpha-scaled copy of it (Engine.derived_refresh), refreshed in place before a replay."""
    from pizero_native.graph import InferenceGraph
    from pizero_native.optim import FusedAdamW

    d, g, m, gi = full
    B = int(g["bsz"])
    name = "joint_model.mixtures.action.layers.0.mlp.down_proj.weight"
    p = m._param(name)  # (tied: named_parameters() may list it under the proprio alias)
    keep = p.detach().clone()
    pb = m._param("action_encoder.linear_3.bias")
    keep_b = pb.detach().clone()
    try:
        m.use_fp8_inference(True)
        a0 = run_infer(m, gi, clip=False)
        ig = InferenceGraph(m, B, clip=False)
        ig.load(gi["input_ids"], gi["pixel_values"], m.block_prefix_counts(gi["itp"], gi["amask"]), gi["vpos"],
                gi["ppos"], gi["apos"], gi["proprios"].float(), gi["noise"])
        ig.capture()
        torch.cuda.synchronize()
        with torch.no_grad():
            p.mul_(-3.0)  # a large change of one fp8-served weight
            pb.add_(0.25)  # and of a bf16 bias read through a derived (scaled) copy
        a1 = run_infer(m, gi, clip=False)
        ag = ig.replay().clone()
        torch.cuda.synchronize()
        m.use_fp8_inference(True)  # fresh codes of the new weights
        a2 = run_infer(m, gi, clip=False)
        assert not torch.equal(a0, a2)
        assert torch.equal(a1, a2), float((a1.float() - a2.float()).abs().max())
        assert torch.equal(ag.float(), a2.float()), float((ag.float() - a2.float()).abs().max())
        # the optimizer's kernel writes bump the arena's weight version
        v0 = m._engine().weights_version()
        opt = FusedAdamW([p], lr=1e-3, state_bits=32)
        p.grad = torch.ones_like(p)
        opt.step()
        p.grad = None
        assert m._engine().weights_version() != v0
    finally:
        with torch.no_grad():
            p.copy_(keep)
            pb.copy_(keep_b)
        m.use_fp8_inference(False)
        m.zero_grad(set_to_none=True)


@pytest.fixture(scope="module")
def b16(full_model):
    d = O.FULL_DIMS
    g = load_golden("b16")
    assert int(g["bsz"]) == 16
    return d, g, full_model


def test_b16_loss_and_grads(b16):
    """config C2's micro-batch (bridge, B=16) against the reference."""
    d, g, m = b16
    gi = gpu_inputs(m, d, 16)
    loss = run_loss(m, gi)
    _check_loss(g, loss.item())
    _check_grads(g, m, "bridge B=16")


def test_microbatch64_batch_invariance(b16):
    """The bench's micro-batch 64 = the 16 fixture samples x 4 in 4 DIFFERENT row orders
    (pizero_gpu_helpers.dealias_orders): same loss / gradients as B=16.  Copy c is a distinct
    permutation, so an error that aliases sample i with sample i + 16c (a batch-stride bug in the
    64-way batched attention GEMMs / kernels) changes the result."""
    from tests.pizero_gpu_helpers import dealias_orders

    d, g, m = b16
    orders = dealias_orders(16, 4)
    assert all(not np.array_equal(orders[a], orders[b]) for a in range(4) for b in range(a))
    assert all((orders[a] != orders[b]).all() for a in range(4) for b in range(a))  # no sample at the same slot
    gi = gpu_inputs(m, d, 16, repeat=4)
    assert gi["input_ids"].shape[0] == 64
    loss = run_loss(m, gi)
    _check_loss(g, loss.item())
    _check_grads(g, m, "micro-batch 64")


@pytest.mark.parametrize("repeat", [8, 16])
def test_microbatch_batch_invariance(b16, repeat):
    """The bench's micro-batches (gbsz 1024 = 256 x 4 on one GPU, 128 x 1 per rank on eight) = the 16 fixture
    samples x ``repeat`` in different row orders, no sample at the same slot in two copies: same loss / gradients
    as B = 16 (35328- / 70656-row GEMMs: whole 256-tile rounds and tails of another shape than at 64)."""
    from tests.pizero_gpu_helpers import dealias_orders

    d, g, m = b16
    orders = dealias_orders(16, repeat)
    assert all((orders[a] != orders[b]).all() for a in range(repeat) for b in range(a))
    if repeat > 8:  # micro-batch 256 needs ~240 GB of activations
        torch.cuda.empty_cache()
        free, _ = torch.cuda.mem_get_info()
        if free < 250e9:
            pytest.skip(f"micro-batch {16 * repeat} needs ~250 GB free, {free / 1e9:.0f} GB free")
    gi = gpu_inputs(m, d, 16, repeat=repeat)
    assert gi["input_ids"].shape[0] == 16 * repeat
    loss = run_loss(m, gi)
    _check_loss(g, loss.item())
    _check_grads(g, m, f"micro-batch {16 * repeat}")
    del gi, loss
    m.zero_grad(set_to_none=True)
    torch.cuda.empty_cache()


@pytest.mark.parametrize("which", ["tiny", "full"])
def test_loss_and_grads_fused_joint_attention(which, request):
    """the fused (flash) joint attention path against the same fixtures"""
    d, g, m, gi = request.getfixturevalue(which)
    eng = m._engine()
    prev = eng.joint_flash, eng.joint_probs
    eng.joint_flash, eng.joint_probs = True, False
    try:
        loss = run_loss(m, gi)
        _check_loss(g, loss.item())
        _check_grads(g, m, f"{which} flash")
    finally:
        eng.joint_flash, eng.joint_probs = prev


@pytest.mark.parametrize("which", ["tiny", "full"])
def test_loss_and_grads_probs_joint_attention(which, request):
    """the fused forward exporting P / tanh(cap) (pz_flash_fwd_probs) + GEMM-path backward"""
    d, g, m, gi = request.getfixturevalue(which)
    eng = m._engine()
    prev = eng.joint_flash, eng.joint_probs
    eng.joint_flash, eng.joint_probs = False, True
    try:
        loss = run_loss(m, gi)
        _check_loss(g, loss.item())
        _check_grads(g, m, f"{which} probs")
    finally:
        eng.joint_flash, eng.joint_probs = prev


@pytest.mark.parametrize("which", ["tiny", "full"])
def test_loss_and_grads_gemm_joint_attention(which, request):
    """the GEMM + softmax joint attention path against the same fixtures"""
    d, g, m, gi = request.getfixturevalue(which)
    eng = m._engine()
    prev = eng.joint_flash, eng.joint_probs
    eng.joint_flash, eng.joint_probs = False, False
    try:
        loss = run_loss(m, gi)
        _check_loss(g, loss.item())
        _check_grads(g, m, f"{which} gemm")
    finally:
        eng.joint_flash, eng.joint_probs = prev


def test_interleaved_forwards_keep_their_saved_state(tiny):
    """two forwards before one backward (autograd semantics): each keeps its own saved K/V, so the
    gradient of loss(A) + loss(B) equals the sum of the separate gradients"""
    d, g, m, gi = tiny
    gj = gpu_inputs(m, d, 3)
    gj["x0"] = -gj["x0"]
    gj["t32"] = 1.0 - gj["t32"]
    run_loss(m, gi)
    ga = m.action_decoder.weight.grad.float().clone()
    run_loss(m, gj)
    gb = m.action_decoder.weight.grad.float().clone()
    m.zero_grad(set_to_none=True)
    la = run_loss(m, gi, backward=False)
    lb = run_loss(m, gj, backward=False)
    (la + lb).backward()
    torch.cuda.synchronize()
    torch.testing.assert_close(m.action_decoder.weight.grad.float(), ga + gb, rtol=2e-2, atol=2e-3)


@pytest.mark.parametrize("which", ["full", "b16"])
def test_expert_stream_backward_bitwise(which, request):
    """The action-expert group's backward on its own HIP stream (Engine.expert_stream, events and
    record_stream at the joint attention) gives the SAME gradient arena bits as the single-stream
    backward (every kernel is deterministic; only the interleaving changes)."""
    if which == "full":
        d, g, m, gi = request.getfixturevalue("full")
    else:
        d, g, m = request.getfixturevalue("b16")
        gi = gpu_inputs(m, d, 16)
    eng = m._engine()
    prev = eng.expert_stream, eng.expert_stream_fwd
    try:
        eng.expert_stream = False
        run_loss(m, gi)
        ref = m._arena.grad.clone()
        for fwd in (False, True):  # backward-only (default) and forward + backward on the second stream
            eng.expert_stream, eng.expert_stream_fwd = True, fwd
            run_loss(m, gi)
            assert torch.equal(m._arena.grad, ref), (fwd, float((m._arena.grad.float() - ref.float()).abs().max()))
    finally:
        eng.expert_stream, eng.expert_stream_fwd = prev
