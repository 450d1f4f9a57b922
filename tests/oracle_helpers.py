"""Shared helpers: run the CPU oracle on the synthetic fixture inputs."""

from __future__ import annotations

import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from oracle import pizero_oracle as O  # noqa: E402
from oracle.synth import synth_inputs  # noqa: E402

GOLDEN = os.path.join(ROOT, "tests", "golden")


def load_golden(name):
    return dict(np.load(os.path.join(GOLDEN, f"{name}.npz"), allow_pickle=False))


def frozen(d, name):
    """pizero.py:224-256: embed + last-layer vlm post*/mlp/o_proj/v_proj frozen."""
    if name == "embed_tokens.weight":
        return True
    last = d["n_layers"] - 1
    if ".mixtures.vlm." in name:
        for s in (f"{last}.post", f"{last}.mlp", f"{last}.self_attn.o_proj", f"{last}.self_attn.v_proj"):
            if s in name:
                return True
    return False


def oracle_run(d, bsz, ragged, want_grads=True, mask_fn=None):
    """fp32 oracle loss (+ grads) and action chunks on the fixture inputs; ``mask_fn`` edits the
    additive [B,1,L,L] mask before use (general-mask tests)."""
    W = O.synth_weights(d, seed=0)
    leaves = {}
    for k, v in W.items():
        if id(v) not in leaves:
            leaves[id(v)] = v.requires_grad_(not frozen(d, k))
    inp = synth_inputs(d, bsz, seed=0, ragged=ragged)
    ids = torch.from_numpy(inp["input_ids"])
    mask, vpos, ppos, apos = O.build_mask_and_positions(d, torch.from_numpy(inp["attention_mask"]))
    if mask_fn is not None:
        mask = mask_fn(mask)
    out_mask = mask
    T = lambda a: torch.from_numpy(a)  # noqa: E731
    loss = O.pizero_loss(W, d, ids, T(inp["pixel_values"]), mask, vpos, ppos, apos,
                         T(inp["proprios"]), T(inp["actions"]), T(inp["t"]), T(inp["x0"]))
    out = {"loss": loss.item(), "mask": out_mask}
    if want_grads:
        loss.backward()
        out["grads"] = {k: (None if v.grad is None else v.grad.detach().clone()) for k, v in W.items()}
    with torch.no_grad():
        itp, amask = O.split_mask(d, mask)
        out["actions"] = O.pizero_infer(W, d, ids, T(inp["pixel_values"]), itp, amask, vpos, ppos,
                                        apos, T(inp["proprios"]), T(inp["noise"]), clip=False)
        out["actions_naive"] = O.pizero_infer_naive(W, d, ids, T(inp["pixel_values"]), mask, vpos,
                                                    ppos, apos, T(inp["proprios"]), T(inp["noise"]),
                                                    clip=False)
    return out, inp
