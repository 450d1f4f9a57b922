"""Build the native PiZero on the GPU with generator-defined weights (fixture twin)."""

from __future__ import annotations

import numpy as np
import torch

from oracle.synth import param_rule, synth_inputs, tensor_seed
from tests.golden.make_golden import ref_cfg


def build_gpu_model(d, dtype=torch.bfloat16):
    from pizero_native import ops
    from src.model.vla.pizero import PiZero

    m = PiZero(ref_cfg(d), device="cuda", dtype=dtype, init="none")
    m.tie_action_proprio_weights()
    m.freeze_unused_weights()
    for name in m._arena.order:
        v = m._arena.view(name)
        off, sc = param_rule(name, tuple(v.shape))
        ops.fill_uniform(v, tensor_seed(name, 0), off, sc)
    torch.cuda.synchronize()
    return m


def gpu_inputs(m, d, bsz, ragged=True):
    inp = synth_inputs(d, bsz, seed=0, ragged=ragged)
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a))  # noqa: E731
    am = T(inp["attention_mask"])
    mask, vpos, ppos, apos = m.build_causal_mask_and_position_ids(am, torch.bfloat16)
    itp, amask = m.split_full_mask_into_submasks(mask)
    dev = "cuda"
    return dict(
        input_ids=T(inp["input_ids"]).to(dev), pixel_values=T(inp["pixel_values"]).to(dev, torch.bfloat16),
        causal_mask=mask.to(dev), itp=itp.to(dev), amask=amask.to(dev), vpos=vpos.to(dev), ppos=ppos.to(dev),
        apos=apos.to(dev), proprios=T(inp["proprios"]).to(dev, torch.bfloat16),
        actions=T(inp["actions"]).to(dev, torch.bfloat16), t=T(inp["t"]).to(dev, torch.bfloat16),
        x0=T(inp["x0"]).to(dev), noise=T(inp["noise"]).to(dev),
        # fp32 copies (the loss compares against fp32 actions/t; bf16 rounding of these inputs is
        # part of the reference's bf16 pipeline)
        actions32=T(inp["actions"]).to(dev), t32=T(inp["t"]).to(dev),
    )


def run_loss(m, g, backward=True, accumulate=False):
    if not accumulate:
        m.zero_grad(set_to_none=True)
    loss = m(input_ids=g["input_ids"], pixel_values=g["pixel_values"], causal_mask=g["causal_mask"],
             vlm_position_ids=g["vpos"], proprio_position_ids=g["ppos"], action_position_ids=g["apos"],
             proprios=g["proprios"], actions=g["actions32"], t=g["t32"], noise=g["x0"])
    if backward:
        loss.backward()
    torch.cuda.synchronize()
    return loss


def run_infer(m, g, clip=False):
    return m.infer_action(input_ids=g["input_ids"], pixel_values=g["pixel_values"].float(), image_text_proprio_mask=g["itp"],
                          action_mask=g["amask"], vlm_position_ids=g["vpos"], proprio_position_ids=g["ppos"],
                          action_position_ids=g["apos"], proprios=g["proprios"], noise=g["noise"], clip=clip)
