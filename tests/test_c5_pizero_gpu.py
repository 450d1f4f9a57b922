"""Config C5 at the PiZero level: several images per sample (the Pi0-paper shape: 3 images = 768 image
tokens + text + 1 proprio + an action chunk of 50).

The reference PiZero composes one image per sample (pizero.py:389-413), so a multi-image PiZero is an
extension: SigLIP runs per image and each sample's images' tokens fill its image-token slots in image
order.  Its parity is pinned by composition: (1) a tiny 3-image model against the fp32 oracle running
the same composition (oracle/pizero_oracle.py embed_siglip_and_text), loss + every gradient (probe gate)
+ the action chunk; (2) the JointModel at the full C5 shape against the reference itself
(tests/test_c5_gpu.py); (3) the full-size 3-image / chunk-50 inference chunk that bench.py times (B=1,
hipGraph, bf16 and fp8) against the reference's own infer_action at that shape (tests/golden/c5_infer.npz).
"""

import numpy as np
import pytest
import torch

from tests.oracle_helpers import O, oracle_run
from tests.pizero_gpu_helpers import GRAD_COS, GRAD_REL, build_gpu_model, gpu_inputs, run_infer, run_loss

pytestmark = pytest.mark.gpu

TINY3 = dict(O.TINY_DIMS, num_images=3, num_image_tokens=48, max_seq_len=56, horizon_steps=6)
C5_FULL = dict(O.FULL_DIMS, num_images=3, num_image_tokens=768, max_seq_len=788, horizon_steps=50)


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def test_three_image_pizero_matches_oracle():
    from tests.golden.gradprobe import compare, probe

    d = TINY3
    ref, _ = oracle_run(d, 2, ragged=True)
    m = build_gpu_model(d)
    gi = gpu_inputs(m, d, 2)
    assert gi["pixel_values"].shape == (2, 3, 3, 56, 56)
    loss = run_loss(m, gi).item()
    assert abs(loss - ref["loss"]) <= 1e-2 * abs(ref["loss"]), (loss, ref["loss"])
    params = dict(m.named_parameters())
    bad = []
    for n, gref in ref["grads"].items():
        p = params.get(n)
        if p is None or gref is None or not p.requires_grad or float(gref.norm()) == 0.0:
            continue
        if n.endswith("self_attn.k_proj.bias") and n.startswith("vision_tower"):
            continue  # exact gradient 0 (softmax shift invariance): both sides are rounding noise
        c = compare(probe(n, p.grad), probe(n, gref))
        if c["rel"] > GRAD_REL or c["cos"] < GRAD_COS:
            bad.append((n, c))
    assert not bad, bad
    a = run_infer(m, gi, clip=False).float().cpu().numpy()
    err = np.abs(a - ref["actions"].numpy())
    assert err.mean() <= 5e-3 and err.max() <= 3e-2, (err.mean(), err.max())


def _c5_graph(m, gi):
    """bench.py's C5 object: InferenceGraph at B=1 (prefill + 10 Euler steps in one hipGraph)."""
    from pizero_native.graph import InferenceGraph

    ig = InferenceGraph(m, 1, clip=False)
    ig.load(gi["input_ids"], gi["pixel_values"], m.block_prefix_counts(gi["itp"], gi["amask"]), gi["vpos"],
            gi["ppos"], gi["apos"], gi["proprios"].float(), gi["noise"])
    ig.capture()
    a = ig.replay()
    torch.cuda.synchronize()
    return a.float().clone()


def _c5_gate(g, a, widen=1.0, label=""):
    """Action gate against the reference's fp32 chunk (tests/golden/c5_infer.npz): mean |d| <= max(3 x the
    reference's own bf16 deviation, 5e-3) and max |d| <= max(3 x dev, 3e-2) (the bridge-size gate of
    tests/test_pizero_gpu.py::_check_actions), times ``widen``."""
    ref, dev = g["fp32/actions_unclipped"], np.abs(g["bf16/actions_unclipped"] - g["fp32/actions_unclipped"])
    a = a.float().cpu().numpy()
    assert a.shape == ref.shape == (1, 50, 7), (a.shape, ref.shape)
    err = np.abs(a - ref)
    print(f"C5 {label}: mean|d| {err.mean():.4g} max {err.max():.4g}; reference bf16 {dev.mean():.4g} / "
          f"{dev.max():.4g}; gate x{widen}")
    assert err.mean() <= widen * max(3 * dev.mean(), 5e-3), (err.mean(), dev.mean())
    assert err.max() <= widen * max(3 * dev.max(), 3e-2), (err.max(), dev.max())


@pytest.fixture(scope="module")
def c5_full():
    from tests.oracle_helpers import load_golden

    g = load_golden("c5_infer")
    m = build_gpu_model(C5_FULL)
    m.eval()
    gi = gpu_inputs(m, C5_FULL, 1, ragged=False)
    assert gi["input_ids"].shape == (1, 788) and gi["pixel_values"].shape[1] == 3
    assert np.array_equal(gi["input_ids"].cpu().numpy(), g["in/input_ids"])
    assert np.array_equal(gi["noise"].cpu().numpy(), g["in/noise"])
    return g, m, gi


def test_c5_full_shape_inference_matches_reference(c5_full):
    """The benched C5 chunk (bench.py c5_inference: 3 x 224^2 images = 768 image tokens + 20 text + 1
    proprio, 788-token prefill into the KV cache, 10 Euler steps over a 50-action chunk, B=1, bf16, one
    hipGraph) against the REFERENCE's own infer_action at that shape (tests/golden/make_golden_c5.py
    main_infer: pizero.py:416-490, joint_model.py:143-240), eager and graph; graph == eager bitwise."""
    g, m, gi = c5_full
    eager = run_infer(m, gi, clip=False)
    _c5_gate(g, eager, label="bf16 eager")
    a = _c5_graph(m, gi)
    _c5_gate(g, a, label="bf16 hipGraph")
    assert torch.equal(a, eager.float())


def test_c5_full_shape_fp8_inference_matches_reference(c5_full):
    """C5 as BASELINE.json names it (fp8, PiZero.use_fp8_inference) against the reference's fp32 chunk at
    the C5 shape.  The reference has no fp8 path, so the gate is the bf16 action gate widened 2x (e4m3
    keeps 3 mantissa bits against bf16's 7 -- the same widening as test_pizero_gpu.py::test_full_actions_fp8);
    the hipGraph replay equals eager bitwise."""
    g, m, gi = c5_full
    try:
        m.use_fp8_inference(True)
        eager = run_infer(m, gi, clip=False)
        _c5_gate(g, eager, widen=2.0, label="fp8 eager")
        a = _c5_graph(m, gi)
        assert torch.equal(a, eager.float())
    finally:
        m.use_fp8_inference(False)
