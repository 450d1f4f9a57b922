"""Pin the CPU oracle against fixtures produced by the reference itself.

tests/golden/tiny.npz is written by tests/golden/make_golden.py, which imports
/root/reference (shroglck/open-pi-zero) in the build container and runs
PiZero.forward/backward/infer_action/infer_action_naive in fp32 on
generator-defined weights.  The oracle must reproduce it to fp32 rounding.
"""

import numpy as np
import pytest
import torch

from tests.oracle_helpers import O, load_golden, oracle_run

REL = 2e-5  # fp32 restatement vs fp32 reference (different op order only)


@pytest.fixture(scope="module")
def tiny():
    g = load_golden("tiny")
    out, inp = oracle_run(O.TINY_DIMS, int(g["bsz"]), ragged=True)
    return g, out, inp


def test_inputs_regenerate(tiny):
    g, _, inp = tiny
    np.testing.assert_array_equal(g["in/input_ids"], inp["input_ids"])
    np.testing.assert_array_equal(g["in/attention_mask"], inp["attention_mask"])
    np.testing.assert_array_equal(g["in/t"], inp["t"])
    assert inp["attention_mask"].sum(1).tolist() != [inp["attention_mask"].shape[1]] * inp["attention_mask"].shape[0]


def test_mask_builder_matches_reference(tiny):
    g, _, inp = tiny
    m, *_ = O.build_mask_and_positions(O.TINY_DIMS, torch.from_numpy(inp["attention_mask"]))
    np.testing.assert_array_equal(m[:, 0].numpy(), g["fp32/mask"])


def test_loss(tiny):
    g, out, _ = tiny
    ref = float(g["fp32/loss"])
    assert abs(out["loss"] - ref) <= REL * abs(ref) + 1e-7


def test_grads(tiny):
    """every parameter: the oracle's gradient probe (norm, seeded samples, projections) = the reference's"""
    from tests.golden.gradprobe import compare, probe

    g, out, _ = tiny
    names = [str(n) for n in g["grad_names"]]
    assert len(names) > 30
    for n in names:
        ref_norm = float(g["fp32/gradnorm/" + n])
        mine = out["grads"].get(n)
        if ref_norm < 0:
            assert mine is None, n
            continue
        assert mine is not None, n
        if ref_norm == 0.0:
            assert float(mine.abs().max()) == 0.0, n
            continue
        ref = {"norm": ref_norm, "sample": torch.from_numpy(g["fp32/gsamp/" + n]),
               "proj": torch.from_numpy(g["fp32/gproj/" + n])}
        c = compare(probe(n, mine, int(g["n_sample"])), ref)
        assert c["rel"] <= 1e-4 and c["norm_rel"] <= 1e-4 and c["proj_err"] <= 1e-4, (n, c)


def test_actions_cached_and_naive(tiny):
    g, out, _ = tiny
    np.testing.assert_allclose(out["actions"].numpy(), g["fp32/actions_unclipped"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(out["actions_naive"].numpy(), g["fp32/actions_naive_unclipped"], rtol=1e-4, atol=1e-5)


def test_reference_bf16_deviation_recorded(tiny):
    g, _, _ = tiny
    assert abs(float(g["bf16/loss"]) - float(g["fp32/loss"])) < 0.05 * abs(float(g["fp32/loss"]))


TEXT_DIMS = dict(O.TINY_DIMS, use_lm_head=True, vlm_final_norm=True)


def test_infer_text_matches_reference():
    """infer_text (pizero.py:559-593) with the reference's KV-cache greedy loop (tests/golden/text.npz):
    the oracle's one-pass restatement, teacher-forced with the reference's tokens, gives the same
    prefill logits and per-step logits, and greedy argmax reproduces the reference's tokens"""
    from oracle.synth import synth_inputs

    g = load_golden("text")
    W = O.synth_weights(TEXT_DIMS, seed=0)
    assert W["lm_head.weight"] is W["embed_tokens.weight"]
    inp = synth_inputs(TEXT_DIMS, 2, seed=3, ragged=True)
    np.testing.assert_array_equal(g["in/input_ids"], inp["input_ids"])
    toks = torch.from_numpy(g["fp32/tokens"])
    n = toks.shape[1] - 1
    with torch.no_grad():
        lg = O.pizero_infer_text(W, TEXT_DIMS, torch.from_numpy(inp["input_ids"]),
                                 torch.from_numpy(inp["pixel_values"]), torch.from_numpy(inp["attention_mask"]),
                                 toks[:, :n])
    q = inp["input_ids"].shape[1]
    pre, steps = g["fp32/prefill_logits"], g["fp32/step_logits"]
    scale = np.abs(pre).max()
    np.testing.assert_allclose(lg[:, :q].numpy(), pre, rtol=0, atol=1e-4 * scale)
    np.testing.assert_allclose(lg[:, q:].numpy(), steps, rtol=0, atol=1e-4 * scale)
    assert torch.equal(lg[:, q - 1:].argmax(-1), toks)


def test_adamw8bit_maps_match_between_oracle_and_optimizer():
    """the optimizer's device maps and the oracle's are the same float32 values (bnb's float32 torch
    construction in both)"""
    from oracle import adamw8bit as O8
    from pizero_native.optim import create_dynamic_map

    for s in (True, False):
        a = O8.create_dynamic_map(s)
        b = create_dynamic_map(s).numpy()
        assert a.shape == (256,) and (a == b).all()
        assert (np.diff(a) >= 0).all() and a[-1] == 1.0


def test_adamw8bit_oracle_sign_fix():
    from oracle import adamw8bit as O8

    q1 = O8.create_dynamic_map(True)
    zero = int(np.nonzero(q1 == 0.0)[0][0])
    m = np.array([-1e-12, 1e-12, 0.0, -0.5], np.float32)
    c = O8.quantize(m / np.float32(1.0), q1, True)
    f = O8.sign_fix(c, m, q1)
    assert c[0] == zero and f[0] == zero - 1  # tiny negative: off the +0 entry
    assert f[1] == c[1] == zero and f[2] == zero and f[3] == c[3]
