"""Host-side logic of the native PiZero (CPU only: no kernels are launched)."""

import numpy as np
import pytest
import torch

from tests.golden.make_golden import ref_cfg
from tests.oracle_helpers import O, frozen


@pytest.fixture(scope="module")
def tiny_model():
    from src.model.vla.pizero import PiZero

    m = PiZero(ref_cfg(O.TINY_DIMS))
    m.tie_action_proprio_weights()
    m.freeze_unused_weights()
    return m


def test_state_dict_keys_and_shapes_match_reference(tiny_model):
    sd = tiny_model.state_dict()
    want = O.param_shapes(O.TINY_DIMS)
    assert set(sd) == set(want)
    for k, v in sd.items():
        assert tuple(v.shape) == tuple(want[k]), k


def test_load_state_dict_strict_into_arena(tiny_model):
    W = O.synth_weights(O.TINY_DIMS)
    tiny_model.load_state_dict({k: v for k, v in W.items()}, strict=True)
    sd = tiny_model.state_dict()
    for k in ("joint_model.mixtures.vlm.layers.1.self_attn.k_proj.weight",
              "vision_tower.vision_model.encoder.layers.0.mlp.fc1.bias", "action_decoder.weight"):
        assert torch.equal(sd[k], W[k])
    # tied alias: proprio keys are the action tensors
    a = tiny_model.joint_model.mixtures["action"].layers[0].mlp.up_proj.weight
    p = tiny_model.joint_model.mixtures["proprio"].layers[0].mlp.up_proj.weight
    assert a is p
    # every parameter is a view of the single flat arena
    base = tiny_model._arena.data
    lo, hi = base.data_ptr(), base.data_ptr() + base.numel() * base.element_size()
    for _, prm in tiny_model.named_parameters():
        assert lo <= prm.data_ptr() < hi


def test_fused_spans_are_adjacent(tiny_model):
    ar = tiny_model._arena
    p = "joint_model.mixtures.vlm.layers.0."
    span = ar.span(p + "self_attn.q_proj.weight", p + "self_attn.v_proj.weight")
    cat = torch.cat([ar.view(p + f"self_attn.{k}_proj.weight") for k in "qkv"], 0)
    assert torch.equal(span, cat)
    gu = ar.span(p + "mlp.gate_proj.weight", p + "mlp.up_proj.weight")
    assert torch.equal(gu, torch.cat([ar.view(p + "mlp.gate_proj.weight"), ar.view(p + "mlp.up_proj.weight")], 0))


def test_freezing_matches_reference_rules(tiny_model):
    for n, prm in tiny_model.named_parameters():
        if n.replace("mixtures.proprio.", "mixtures.action.") != n:
            n = n.replace("mixtures.proprio.", "mixtures.action.")
        assert prm.requires_grad == (not frozen(O.TINY_DIMS, n)), n
    nact = sum(p.numel() for p in tiny_model.action_expert_parameters)
    nvlm = sum(p.numel() for p in tiny_model.trainable_vlm_parameters)
    assert nact > 0 and nvlm > 0


def test_mask_builder_matches_reference_semantics(tiny_model):
    am = torch.tensor([[1] * 10 + [0] * 14, [1] * 7 + [0] * 17], dtype=torch.int64)
    m1, v1, p1, a1 = tiny_model.build_causal_mask_and_position_ids(am, torch.bfloat16)
    m2, v2, p2, a2 = O.build_mask_and_positions(O.TINY_DIMS, am, torch.bfloat16)
    assert torch.equal(m1, m2) and torch.equal(v1, v2) and torch.equal(p1, p2) and torch.equal(a1, a2)
    assert tiny_model._prefix_counts(m1).tolist() == [10, 7]
    itp, amask = tiny_model.split_full_mask_into_submasks(m1)
    assert itp.shape[-1] == 24 + 1 and amask.shape[-2] == 4


def test_dtype_conversion_keeps_arena_binding(tiny_model):
    tiny_model.to(torch.bfloat16)
    assert tiny_model._arena.data.dtype == torch.bfloat16
    w = tiny_model.joint_model.mixtures["vlm"].layers[0].self_attn.q_proj.weight
    assert w.dtype == torch.bfloat16
    assert w.data_ptr() == tiny_model._arena.view("joint_model.mixtures.vlm.layers.0.self_attn.q_proj.weight").data_ptr()
    assert not tiny_model.joint_model.mixtures["vlm"].layers[-1].self_attn.v_proj.weight.requires_grad
    tiny_model.to(torch.float32)


def test_cpu_execution_fails_loudly(tiny_model):
    with pytest.raises(RuntimeError, match="MI355X HIP path only"):
        tiny_model._engine()


def test_mask_contract_block_vs_general(tiny_model):
    """the reference builder's mask -> per-sample prefix counts (block kernels); any other
    additive mask -> GeneralMask (GEMM + additive softmax path).  Validated once per tensor."""
    from pizero_native.engine import GeneralMask

    am = torch.tensor([[1] * 10 + [0] * 14, [1] * 7 + [0] * 17], dtype=torch.int64)
    for dt in (torch.bfloat16, torch.float32):
        m, *_ = tiny_model.build_causal_mask_and_position_ids(am, dt)
        L = m.shape[-1]
        spec = tiny_model._mask_spec([m], [torch.arange(L)])
        assert isinstance(spec, torch.Tensor) and spec.tolist() == [10, 7]
        assert tiny_model._mask_spec([m], [torch.arange(L)]) is spec  # cached by identity + version
        itp, amask = tiny_model.split_full_mask_into_submasks(m)
        L1 = itp.shape[-1]
        s2 = tiny_model._mask_spec([itp, amask], [torch.arange(L1), torch.arange(L1, L1 + amask.shape[2])])
        assert isinstance(s2, torch.Tensor) and s2.tolist() == [10, 7]
    m, *_ = tiny_model.build_causal_mask_and_position_ids(am, torch.bfloat16)
    L = m.shape[-1]
    # action rows blind to the proprio token: not the block pattern
    m2 = m.clone()
    m2[:, :, -4:, 24] = torch.finfo(torch.bfloat16).min
    assert isinstance(tiny_model._mask_spec([m2], [torch.arange(L)]), GeneralMask)
    # in-place edit of a validated tensor bumps its version -> re-validated
    spec = tiny_model._mask_spec([m], [torch.arange(L)])
    assert isinstance(spec, torch.Tensor)
    m[:, :, 0, 0] = -2.0
    g = tiny_model._mask_spec([m], [torch.arange(L)])
    assert isinstance(g, GeneralMask) and g.full.dtype == torch.float32 and g.full.shape == (2, L, L)
    # fp16-style "-65504" masking does not absorb the logits like finfo.min: general path
    m3, *_ = tiny_model.build_causal_mask_and_position_ids(am, torch.float32)
    m3 = torch.where(m3 < 0, torch.full_like(m3, -65504.0), m3)
    assert isinstance(tiny_model._mask_spec([m3], [torch.arange(L)]), GeneralMask)
    with pytest.raises(ValueError, match="block mask"):
        itp, amask = tiny_model.split_full_mask_into_submasks(m2)
        tiny_model.block_prefix_counts(itp, amask)
