"""Generate golden fixtures by running the REFERENCE itself (build container only).

Run from the repo root:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py [tiny|full|all]

What it does
  * imports shroglck/open-pi-zero from /root/reference with three stub modules
    for absent third-party packages (omegaconf.OmegaConf.merge,
    hydra.utils.instantiate, bitsandbytes placeholder classes) -- SURVEY 8(c);
  * builds ``PiZero(cfg)`` + ``tie_action_proprio_weights()`` +
    ``freeze_unused_weights()`` exactly as train.py:94-102 does;
  * loads generator-defined weights (oracle/synth.py) with strict=True;
  * runs ``forward`` (noise patched to the supplied x0), ``.backward()``,
    ``infer_action`` and ``infer_action_naive`` (noise patched) in fp32, and
    the same in bf16 (weights + inputs cast, CPU) to record the reference's
    own bf16-vs-fp32 deviation, which sets the GPU tolerances;
  * writes tests/golden/<name>.npz (inputs are regenerated from seeds, only
    outputs and small input tensors are stored).

Nothing under /root/reference is copied; this script only imports it.
"""

from __future__ import annotations

import os
import sys
import types

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
REF = "/root/reference"

from oracle.pizero_oracle import FULL_DIMS, TINY_DIMS, param_shapes, synth_weights  # noqa: E402
from oracle.synth import synth_inputs  # noqa: E402


class AttrDict(dict):
    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = v


def to_attr(x):
    if isinstance(x, dict):
        return AttrDict({k: to_attr(v) for k, v in x.items()})
    return x


def deep_merge(a, b):
    out = AttrDict(a)
    for k, v in b.items():
        if k in out and isinstance(out[k], dict) and isinstance(v, dict):
            out[k] = deep_merge(out[k], v)
        else:
            out[k] = v
    return out


def install_stubs():
    om = types.ModuleType("omegaconf")

    class OmegaConf:
        @staticmethod
        def merge(a, b):
            return deep_merge(a, b)

    om.OmegaConf = OmegaConf
    sys.modules["omegaconf"] = om

    hy = types.ModuleType("hydra")
    hu = types.ModuleType("hydra.utils")

    def instantiate(c):
        import importlib

        mod, cls = c["_target_"].rsplit(".", 1)
        kw = {k: v for k, v in c.items() if k != "_target_"}
        return getattr(importlib.import_module(mod), cls)(**kw)

    hu.instantiate = instantiate
    hy.utils = hu
    sys.modules["hydra"] = hy
    sys.modules["hydra.utils"] = hu

    bnb = types.ModuleType("bitsandbytes")
    bnn = types.ModuleType("bitsandbytes.nn")

    class Params4bit(torch.nn.Parameter):
        pass

    class Linear4bit(torch.nn.Linear):
        pass

    bnn.Params4bit = Params4bit
    bnn.Linear4bit = Linear4bit
    bnb.nn = bnn
    sys.modules["bitsandbytes"] = bnb
    sys.modules["bitsandbytes.nn"] = bnn


def ref_cfg(d):
    """bridge.yaml-shaped config (config/train/bridge.yaml:68-181) from dims."""
    mix = {
        "vlm": dict(hidden_size=d["vlm_hidden"], intermediate_size=d["vlm_inter"],
                    use_final_norm=False, cache=True, use_quantize=False, use_lora=False,
                    adaptive_mode=None, rope_theta=d["vlm_theta"]),
        "proprio": dict(hidden_size=d["act_hidden"], intermediate_size=d["act_inter"],
                        use_final_norm=True, cache=True, use_quantize=False, use_lora=False,
                        adaptive_mode=None, rope_theta=d["act_theta"]),
        "action": dict(hidden_size=d["act_hidden"], intermediate_size=d["act_inter"],
                       use_final_norm=True, cache=False, use_quantize=False, use_lora=False,
                       adaptive_mode=None, rope_theta=d["act_theta"]),
    }
    c = dict(
        vocab_size=d["vocab_size"], pad_token_id=d["pad_token_id"],
        image_token_index=d["image_token_index"], use_lm_head=False,
        max_seq_len=d["max_seq_len"], max_image_text_tokens=d["max_seq_len"],
        cond_steps=d["cond_steps"], horizon_steps=d["horizon_steps"],
        action_dim=d["action_dim"], proprio_dim=d["proprio_dim"],
        num_inference_steps=d["num_inference_steps"],
        final_action_clip_value=d["final_action_clip_value"],
        flow_sig_min=d["flow_sig_min"], action_expert_adaptive_mode=None,
        time_hidden_size=256, time_max_period=d["time_max_period"],
        action_expert_rope_theta=d["act_theta"], mixture=mix,
        vision=dict(_target_="src.model.paligemma.siglip.SiglipVisionModel",
                    config=dict(hidden_size=d["vis_hidden"], intermediate_size=d["vis_inter"],
                                num_hidden_layers=d["vis_layers"], num_attention_heads=d["vis_heads"],
                                num_channels=3, image_size=d["image_size"], patch_size=d["patch_size"],
                                layer_norm_eps=d["ln_eps"], attention_dropout=0.0,
                                num_image_tokens=d["num_image_tokens"], lora=dict(r=32, dropout=0.0)),
                    use_quantize=False, use_lora=False),
        vision_projector=dict(_target_="src.model.paligemma.siglip.PaliGemmaMultiModalProjector",
                              config=dict(vision_config=dict(hidden_size=d["vis_hidden"],
                                                             projection_dim=d["proj_dim"]),
                                          lora=dict(r=32, dropout=0.0)),
                              use_quantize=False, use_lora=False),
        joint=dict(_target_="src.model.vla.joint_model.JointModel",
                   config=dict(action_expert_adaptive_mode=None, time_hidden_size=256, mixture=mix,
                               lora=dict(r=32, dropout=0.0), num_hidden_layers=d["n_layers"],
                               num_attention_heads=d["n_heads"], num_key_value_heads=d["n_kv"],
                               head_dim=d["head_dim"], rms_norm_eps=d["rms_eps"],
                               attention_bias=False, attention_dropout=0.0,
                               pad_token_id=d["pad_token_id"])),
    )
    return to_attr(c)


def run_reference(d, bsz, ragged, dtype, W, inp, grad_names):
    from src.model.vla import pizero as pz

    cfg = ref_cfg(d)
    torch.manual_seed(0)
    model = pz.PiZero(cfg)
    model.tie_action_proprio_weights()
    model.freeze_unused_weights()
    sd = model.state_dict()
    assert set(sd) == set(param_shapes(d)), set(sd) ^ set(param_shapes(d))
    for k, v in sd.items():
        assert tuple(v.shape) == tuple(param_shapes(d)[k]), k
    model.load_state_dict({k: W[k] for k in sd}, strict=True)
    model.to(dtype)
    t = lambda a: torch.from_numpy(a).to(dtype)  # noqa: E731
    ids = torch.from_numpy(inp["input_ids"])
    am = torch.from_numpy(inp["attention_mask"])
    mask, vpos, ppos, apos = model.build_causal_mask_and_position_ids(am, dtype)
    itp, amask = model.split_full_mask_into_submasks(mask)
    x0 = t(inp["x0"])
    noise = t(inp["noise"])
    orig_randn_like, orig_randn = torch.randn_like, torch.randn
    out = {}
    try:
        torch.randn_like = lambda *a, **k: x0.clone()
        loss = model(input_ids=ids, pixel_values=t(inp["pixel_values"]), causal_mask=mask,
                     vlm_position_ids=vpos, proprio_position_ids=ppos, action_position_ids=apos,
                     proprios=t(inp["proprios"]), actions=t(inp["actions"]), t=t(inp["t"]))
        loss.backward()
        out["loss"] = np.float64(loss.detach().float().item())
        named = dict(model.named_parameters())
        for n in grad_names:
            p = named[n]
            g = p.grad
            if g is None:
                out["gradnorm/" + n] = np.float64(-1.0)
                continue
            gf = g.detach().double()
            out["gradnorm/" + n] = np.float64(gf.norm().item())
            out["gradhead/" + n] = gf.flatten()[:64].numpy().astype(np.float64)
        model.zero_grad(set_to_none=True)
        model.eval()
        with torch.inference_mode():
            torch.randn = lambda *a, **k: noise.clone()
            cv = model.final_action_clip_value
            model.final_action_clip_value = None
            a1 = model.infer_action(input_ids=ids, pixel_values=t(inp["pixel_values"]),
                                    image_text_proprio_mask=itp, action_mask=amask,
                                    vlm_position_ids=vpos, proprio_position_ids=ppos,
                                    action_position_ids=apos, proprios=t(inp["proprios"]))
            a2 = model.infer_action_naive(input_ids=ids, pixel_values=t(inp["pixel_values"]),
                                          causal_mask=mask, vlm_position_ids=vpos,
                                          proprio_position_ids=ppos, action_position_ids=apos,
                                          proprios=t(inp["proprios"]))
            model.final_action_clip_value = cv
            a3 = model.infer_action(input_ids=ids, pixel_values=t(inp["pixel_values"]),
                                    image_text_proprio_mask=itp, action_mask=amask,
                                    vlm_position_ids=vpos, proprio_position_ids=ppos,
                                    action_position_ids=apos, proprios=t(inp["proprios"]))
        out["actions_unclipped"] = a1.float().numpy()
        out["actions_naive_unclipped"] = a2.float().numpy()
        out["actions_clipped"] = a3.float().numpy()
        out["mask"] = mask[:, 0].float().numpy() if d is TINY_DIMS else np.zeros(1)
    finally:
        torch.randn_like, torch.randn = orig_randn_like, orig_randn
    return out


def grad_name_subset(d):
    """A representative set of trained parameters (every kind, first/last layers)."""
    names = []
    vt = "vision_tower.vision_model."
    Lv, Lj = d["vis_layers"] - 1, d["n_layers"] - 1
    names += [vt + "embeddings.patch_embedding.weight", vt + "embeddings.patch_embedding.bias",
              vt + "embeddings.position_embedding.weight", vt + "post_layernorm.weight"]
    for i in sorted({0, Lv}):
        p = f"{vt}encoder.layers.{i}."
        names += [p + "self_attn.q_proj.weight", p + "self_attn.k_proj.weight",
                  p + "self_attn.v_proj.weight", p + "self_attn.out_proj.weight",
                  p + "self_attn.q_proj.bias", p + "layer_norm1.weight", p + "layer_norm2.bias",
                  p + "mlp.fc1.weight", p + "mlp.fc1.bias", p + "mlp.fc2.weight"]
    names += ["multi_modal_projector.linear.weight", "multi_modal_projector.linear.bias"]
    for mix in ("vlm", "action"):
        for i in sorted({0, Lj // 2, Lj}):
            p = f"joint_model.mixtures.{mix}.layers.{i}."
            names += [p + "self_attn.q_proj.weight", p + "self_attn.k_proj.weight",
                      p + "self_attn.o_proj.weight", p + "mlp.gate_proj.weight",
                      p + "mlp.up_proj.weight", p + "mlp.down_proj.weight",
                      p + "input_layernorm.weight", p + "post_attention_layernorm.weight"]
            if not (mix == "vlm" and i == Lj):
                names += [p + "self_attn.v_proj.weight"]
    names += ["joint_model.mixtures.action.norm.weight"]
    names += ["action_encoder.linear_1.weight", "action_encoder.linear_2.weight",
              "action_encoder.linear_3.bias", "proprio_encoder.weight", "proprio_encoder.bias",
              "action_decoder.weight", "action_decoder.bias"]
    # mixtures.proprio.* alias mixtures.action.* after the tie; named_parameters
    # reports the shared tensor once, under the first registered name (proprio)
    return [n.replace(".mixtures.action.layers", ".mixtures.proprio.layers")
            .replace(".mixtures.action.norm", ".mixtures.proprio.norm") for n in names]


def make(name, d, bsz, ragged):
    install_stubs()
    if REF not in sys.path:
        sys.path.insert(0, REF)
    torch.set_num_threads(os.cpu_count() or 8)
    W = synth_weights(d, seed=0)
    inp = synth_inputs(d, bsz, seed=0, ragged=ragged)
    gnames = grad_name_subset(d)
    res = {}
    for tag, dt in (("fp32", torch.float32), ("bf16", torch.bfloat16)):
        print(f"[{name}] reference run {tag} ...", flush=True)
        o = run_reference(d, bsz, ragged, dt, W, inp, gnames)
        for k, v in o.items():
            res[f"{tag}/{k}"] = v
    for k in ("input_ids", "attention_mask", "t"):
        res["in/" + k] = inp[k]
    res["grad_names"] = np.array(gnames)
    res["bsz"] = np.int64(bsz)
    path = os.path.join(ROOT, "tests", "golden", f"{name}.npz")
    np.savez_compressed(path, **res)
    print("wrote", path, "loss fp32", res["fp32/loss"], "bf16", res["bf16/loss"])


if __name__ == "__main__":
    which = sys.argv[1] if len(sys.argv) > 1 else "all"
    if which in ("tiny", "all"):
        make("tiny", TINY_DIMS, 3, ragged=True)
    if which in ("full", "all"):
        make("full", FULL_DIMS, 2, ragged=True)


def make_lr():
    """lr trace of the reference CosineAnnealingWarmupRestarts (utils/optim.py:31-159)."""
    if REF not in sys.path:
        sys.path.insert(0, REF)
    from src.utils.optim import CosineAnnealingWarmupRestarts

    out = {}
    for name, (first, mult, mx, mn, warm, gamma) in {
        "bridge": (10000000, 1.0, 5e-5, 1e-8, 200, 1.0),
        "restarts": (50, 1.0, 1e-3, 1e-6, 10, 0.5),
        "mult": (40, 2.0, 1e-3, 1e-6, 5, 0.8),
    }.items():
        p = [torch.nn.Parameter(torch.zeros(1))]
        opt = torch.optim.SGD(p, lr=1.0)
        s = CosineAnnealingWarmupRestarts(opt, first_cycle_steps=first, cycle_mult=mult, max_lr=mx, min_lr=mn,
                                          warmup_steps=warm, gamma=gamma)
        lrs = [opt.param_groups[0]["lr"]]
        for _ in range(300):
            s.step()
            lrs.append(opt.param_groups[0]["lr"])
        out[name] = np.array(lrs, dtype=np.float64)
        out[name + "_args"] = np.array([first, mult, mx, mn, warm, gamma], dtype=np.float64)
    np.savez_compressed(os.path.join(ROOT, "tests", "golden", "lr_schedule.npz"), **out)
    print("wrote lr_schedule.npz")


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "lr":
    make_lr()
