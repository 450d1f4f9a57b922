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


def dealias_orders(bsz, repeat):
    """``repeat`` different row orders of the ``bsz`` fixture samples: copy c is a distinct permutation
    (identity, reversed, rotated by 6, reversed + rotated by 6), so for an even bsz (16) no slot holds the
    same sample in two copies (even rotations: 2i = odd has no solution mod an even bsz) -- a batch-stride
    error that aliases rows of different copies changes the loss / gradients."""
    base = np.arange(bsz)
    out = []
    for c in range(repeat):
        o = base[::-1] if c % 2 else base
        out.append(np.roll(o, (c // 2) * 6))
    return out


def gpu_inputs(m, d, bsz, ragged=True, repeat=1, select=None):
    """Fixture inputs of batch ``bsz`` on the device.  ``repeat`` tiles the batch with a different row
    order per copy (dealias_orders; the loss is a mean over samples, so the r-fold batch has the same
    loss and gradients -- batch invariance); ``select`` keeps only those fixture samples (e.g. [0]:
    one sample of the fixture at B=1 -- samples are independent, so its outputs are that sample's)."""
    inp = synth_inputs(d, bsz, seed=0, ragged=ragged)
    if repeat > 1:
        orders = dealias_orders(bsz, repeat)
        inp = {k: np.concatenate([v[o] for o in orders], axis=0) for k, v in inp.items()}
    if select is not None:
        inp = {k: v[list(select)] for k, v in inp.items()}
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


# ---------------------------------------------------------------- gradient gate --
# per-tensor gradient rel-L2 <= 8 % and cosine >= 0.995 against the fp32 reference,
# widened only where the reference's OWN bf16 run deviates more (tolerance = 2x that deviation).
GRAD_REL = 0.08
GRAD_COS = 0.995
PROJ_SIGMA = 5.0  # projection error bound in units of tol * |g_ref| (an error e moves it ~N(0, |e|^2))


def grad_tolerance(g, n):
    brel = float(g.get(f"bf16/grel/{n}", 0.0))
    tol = max(GRAD_REL, 2.0 * brel)
    return tol, min(GRAD_COS, 1.0 - 0.5 * tol * tol)


def check_grads_probe(g, params, name_map=None, label="", skip_frozen=False):
    """Every tensor of the fixture: sample rel-L2 / cosine, norm, whole-tensor projections.

    ``params``: name -> nn.Parameter of the native model; ``name_map`` maps a fixture name to it.
    ``skip_frozen``: ignore tensors the native model freezes (JointModel-level fixtures, where the
    reference module applies no PiZero freezing rules).
    Returns the worst margins (also printed, so the GPU log records them)."""
    from tests.golden.gradprobe import compare, probe

    names = [str(n) for n in g["grad_names"]]
    ns = int(g.get("n_sample", 4096))
    bad, worst = [], {"rel": 0.0, "cos": 1.0, "norm_rel": 0.0, "proj_err": 0.0, "n": 0}
    for n in names:
        p = params[name_map(n) if name_map else n]
        if skip_frozen and not p.requires_grad:
            continue
        ref_norm = float(g[f"fp32/gradnorm/{n}"])
        if ref_norm < 0:  # frozen in the reference (no grad)
            if not (p.grad is None or not p.requires_grad):
                bad.append((n, "reference has no gradient, native has one"))
            continue
        if p.grad is None:
            bad.append((n, "missing gradient"))
            continue
        if ref_norm == 0.0:  # e.g. last-layer vlm q_proj (pizero.py:224-256): exactly zero
            if float(p.grad.float().abs().max()) != 0.0:
                bad.append((n, "reference gradient is exactly 0"))
            continue
        if float(g.get(f"bf16/grel/{n}", 0.0)) > 1.0:
            # noise-only gradient: the exact value is 0 (e.g. SigLIP k_proj.bias -- softmax is invariant to
            # a per-query constant, so d/d(key bias) = 0) and the reference's own bf16 run differs from its
            # fp32 run by > 100 %: require the native norm to stay at that rounding-noise level
            noise = max(ref_norm, float(g[f"bf16/gradnorm/{n}"]))
            mine = float(p.grad.double().norm())
            if mine > 10.0 * noise:
                bad.append((n, f"noise-level gradient {mine:.3e} > 10 x {noise:.3e}"))
            worst["noise"] = worst.get("noise", 0) + 1
            continue
        ref = {"norm": ref_norm, "sample": torch.from_numpy(g[f"fp32/gsamp/{n}"]),
               "proj": torch.from_numpy(g[f"fp32/gproj/{n}"])}
        c = compare(probe(n, p.grad, ns), ref)
        tol, cmin = grad_tolerance(g, n)
        ok = c["rel"] <= tol and c["cos"] >= cmin and c["norm_rel"] <= tol and c["proj_err"] <= PROJ_SIGMA * tol
        if not ok:
            bad.append((n, {k: round(v, 5) for k, v in c.items()}, round(tol, 4), round(cmin, 5)))
        worst["rel"] = max(worst["rel"], c["rel"])
        worst["cos"] = min(worst["cos"], c["cos"])
        worst["norm_rel"] = max(worst["norm_rel"], c["norm_rel"])
        worst["proj_err"] = max(worst["proj_err"], c["proj_err"])
        worst["n"] += 1
    print(f"[grad gate {label}] tensors {worst['n']}: max rel-L2 {worst['rel']:.4f}, min cos {worst['cos']:.5f}, "
          f"max norm rel {worst['norm_rel']:.4f}, max proj err {worst['proj_err']:.4f} |g|; "
          f"{worst.get('noise', 0)} noise-only (exact gradient 0)")
    assert not bad, "\n".join(map(str, bad))
    return worst
