"""Golden fixture for config C5 (BASELINE.json configs[4], the Pi0-paper shape) from the REFERENCE.

Run from the repo root (build container only):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_c5.py

The reference PiZero has one image per sample (pizero.py:389-413), so C5 -- 3 images (768 image
tokens) + 20 text + 1 proprio + an action chunk of 50, L = 839 -- is composed at the JointModel
level: the reference's own ``JointModel`` (joint_model.py:307-383, built from the
bridge.yaml joint config at full Gemma-2B / action-expert dims, proprio mixture tied to action
weights as pizero.py:262-264 does) runs forward + backward on generator-defined embeddings,
with the reference's own block mask / positions (pizero.py:271-324, 8 pad text tokens).  Loss =
sum(action_hidden * R) for a generator-defined R.  Stored: the action hidden states and, for the
input-embedding gradients and EVERY JointModel parameter gradient, the tests/golden/gradprobe.py
summary (norm, seeded samples incl. tile tails, whole-tensor projections) in fp32, plus the
reference's own bf16-vs-fp32 deviation (sets the GPU tolerance).
Inputs are regenerated from seeds on both sides (oracle/synth.py; pz_fill_uniform on device).
Nothing under /root/reference is copied; this script only imports it.
"""

from __future__ import annotations

import os
import sys
import time
import types

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"

from gradprobe import probe  # noqa: E402
from make_golden import install_stubs, ref_cfg  # noqa: E402
from oracle.pizero_oracle import FULL_DIMS, synth_weights  # noqa: E402
from oracle.synth import synth_tensor  # noqa: E402

C5_DIMS = dict(FULL_DIMS, max_seq_len=788, horizon_steps=50)
C5_CNT = 780  # image/text tokens actually present (8 pad text tokens exercise the pad rows)
C5_INPUTS = {  # name -> (shape, scale) of the generator-defined inputs (offset 0)
    "c5/embeds.vlm": ((1, 788, 2048), 1.0),
    "c5/embeds.proprio": ((1, 1, 1024), 1.0),
    "c5/embeds.action": ((1, 50, 1024), 1.0),
    "c5/R": ((1, 50, 1024), 1.0),
}


def c5_grad_names(joint):
    """Every JointModel parameter (after the tie the shared expert tensors appear once, as proprio)."""
    return [n for n, _ in joint.named_parameters()]


def run(dtype):
    from hydra.utils import instantiate
    from src.model.vla import pizero as pz

    d = C5_DIMS
    cfg = ref_cfg(d)
    torch.manual_seed(0)
    joint = instantiate(cfg.joint)
    W = synth_weights(d)
    sd = joint.state_dict()
    joint.load_state_dict({k: torch.as_tensor(W["joint_model." + k]) for k in sd}, strict=True)
    # tie proprio <- action (pizero.py:262-264)
    joint.mixtures["proprio"] = joint.mixtures["action"]
    joint.to(dtype)
    ns = types.SimpleNamespace(max_image_text_tokens=788, num_proprio_tokens=1, num_action_tokens=50,
                               total_num_tokens=839)
    am = torch.zeros(1, 788, dtype=torch.int64)
    am[:, :C5_CNT] = 1
    mask, vpos, ppos, apos = pz.PiZero.build_causal_mask_and_position_ids(ns, am, dtype)
    inp = {k: torch.from_numpy(synth_tensor(k, s, 0.0, sc)) for k, (s, sc) in C5_INPUTS.items()}
    leaves = {n: inp[f"c5/embeds.{n}"].to(dtype).requires_grad_() for n in ("vlm", "proprio", "action")}
    embeds = {n: leaves[n] * 1 for n in ("vlm", "proprio", "action")}  # JointModel scales in place
    out = joint(attention_mask=mask, position_ids_all={"vlm": vpos, "proprio": ppos, "action": apos},
                embeds_all=embeds)
    ya = out["action"]
    loss = (ya.float() * inp["c5/R"]).sum()
    loss.backward()
    res = {"action_hidden": ya.detach().float().numpy()}
    for n, lf in leaves.items():
        pr = probe("dembeds." + n, lf.grad)
        res[f"gradnorm/dembeds.{n}"] = np.float64(pr["norm"])
        res[f"gsamp/dembeds.{n}"] = pr["sample"].numpy()
        res[f"gproj/dembeds.{n}"] = pr["proj"].numpy()
    names = c5_grad_names(joint)
    named = dict(joint.named_parameters())
    for n in names:
        p = named[n]
        if p.grad is None:
            res[f"gradnorm/{n}"] = np.float64(-1.0)
            continue
        pr = probe(n, p.grad)
        res[f"gradnorm/{n}"] = np.float64(pr["norm"])
        res[f"gsamp/{n}"] = pr["sample"].numpy()
        res[f"gproj/{n}"] = pr["proj"].numpy()
    res["_names"] = names
    return res


C5_INFER_DIMS = dict(FULL_DIMS, num_images=3, num_image_tokens=768, max_seq_len=788, horizon_steps=50)


def run_infer(dtype, W, inp):
    """The reference's own ``PiZero.infer_action`` (pizero.py:416-490) at the C5 shape, B=1: the full model
    (SigLIP + projector + Gemma-2B + action expert, tied + frozen as train.py:99-102), prefill of vlm +
    proprio into the reference KVCache, 10 Euler steps with ``cache_mode="append_non_active"``
    (joint_model.py:143-240).  The reference takes one image per sample (pizero.py:389), so its
    ``vision_tower`` is called once per image and the 3 x 256 token features are concatenated in image
    order -- the composition the native multi-image embedding implements; everything after that
    (projector, /sqrt(2048), the image-row scatter, the joint model, the loop) is the reference's code
    unchanged.  ``torch.randn`` is patched to return a clone of the supplied noise (pizero.py:454), the
    final clip is off (the chunk stays informative).  Returns the chunk and each step's velocity."""
    from src.model.vla import pizero as pz

    d = C5_INFER_DIMS
    torch.manual_seed(0)
    model = pz.PiZero(ref_cfg(d))
    model.tie_action_proprio_weights()
    model.freeze_unused_weights()
    sd = model.state_dict()
    model.load_state_dict({k: torch.as_tensor(W[k]) for k in sd}, strict=True)
    model.to(dtype).eval()
    vt = model.vision_tower
    one_image = vt.forward
    vt.forward = lambda pv: torch.cat([one_image(pv[:, i]) for i in range(pv.shape[1])], dim=1)
    vel = []
    model.action_decoder.register_forward_hook(lambda m, a, o: vel.append(o.detach().float().clone()))
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dtype)  # noqa: E731
    am = torch.from_numpy(inp["attention_mask"])
    mask, vpos, ppos, apos = model.build_causal_mask_and_position_ids(am, dtype)
    itp, amask = model.split_full_mask_into_submasks(mask)
    noise = T(inp["noise"])
    orig = torch.randn
    try:
        torch.randn = lambda *a, **k: noise.clone()
        model.final_action_clip_value = None
        with torch.inference_mode():
            a = model.infer_action(input_ids=torch.from_numpy(inp["input_ids"]), pixel_values=T(inp["pixel_values"]),
                                   image_text_proprio_mask=itp, action_mask=amask, vlm_position_ids=vpos,
                                   proprio_position_ids=ppos, action_position_ids=apos, proprios=T(inp["proprios"]))
    finally:
        torch.randn = orig
    assert len(vel) == d["num_inference_steps"], len(vel)
    return a.float().numpy(), torch.stack(vel, 0).numpy()


def main_infer():
    """tests/golden/c5_infer.npz: the benched C5 chunk (B=1, 3 images, full prefix, chunk 50) from the
    reference, fp32 (canonical) and bf16 (the reference's own bf16 deviation sets the GPU tolerance)."""
    from oracle.synth import synth_inputs

    install_stubs()
    sys.path.insert(0, REF)
    torch.set_num_threads(os.cpu_count() or 8)
    d = C5_INFER_DIMS
    W = synth_weights(d)
    inp = synth_inputs(d, 1, seed=0, ragged=False)
    assert inp["pixel_values"].shape == (1, 3, 3, 224, 224) and inp["input_ids"].shape == (1, 788)
    out = {"in/input_ids": inp["input_ids"], "in/noise": inp["noise"]}
    for tag, dt in (("fp32", torch.float32), ("bf16", torch.bfloat16)):
        t0 = time.time()
        a, v = run_infer(dt, W, inp)
        print(f"c5 infer {tag}: {time.time() - t0:.1f}s  chunk |a| mean {np.abs(a).mean():.4f}", flush=True)
        out[f"{tag}/actions_unclipped"] = a
        out[f"{tag}/velocities"] = v
    dev = np.abs(out["bf16/actions_unclipped"] - out["fp32/actions_unclipped"])
    print(f"reference bf16 vs fp32: mean |d| {dev.mean():.3e} max {dev.max():.3e}")
    path = os.path.join(ROOT, "tests", "golden", "c5_infer.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path), "bytes")


def main():
    install_stubs()
    sys.path.insert(0, REF)
    torch.set_num_threads(os.cpu_count() or 8)
    out = {"cnt": np.int64(C5_CNT)}
    for tag, dt in (("fp32", torch.float32), ("bf16", torch.bfloat16)):
        t0 = time.time()
        r = run(dt)
        print(f"{tag}: {time.time() - t0:.1f}s", flush=True)
        names = r.pop("_names")
        out["grad_names"] = np.array(["dembeds." + n for n in ("vlm", "proprio", "action")] + names)
        for k, v in r.items():
            out[f"{tag}/{k}"] = v
    for n in [str(x) for x in out["grad_names"]]:  # the reference's own bf16-vs-fp32 deviation
        a, b = out.get(f"bf16/gsamp/{n}"), out.get(f"fp32/gsamp/{n}")
        if a is None or b is None:
            continue
        a64, b64 = a.astype(np.float64), b.astype(np.float64)
        nb = np.linalg.norm(b64)
        out[f"bf16/grel/{n}"] = np.float64(np.linalg.norm(a64 - b64) / max(nb, 1e-30))
        del out[f"bf16/gsamp/{n}"]
    out["n_sample"] = np.int64(4096)
    path = os.path.join(ROOT, "tests", "golden", "c5.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "infer":
        main_infer()
    else:
        main()
