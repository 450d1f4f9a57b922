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
  * summarises EVERY parameter gradient with tests/golden/gradprobe.py (norm, ~4096
    seeded samples incl. tile tails, 2 whole-tensor Rademacher projections) and
    writes tests/golden/<name>.npz (inputs are regenerated from seeds, only
    outputs and small input tensors are stored).

Fixtures: tiny (2+2 layers at full widths... see oracle TINY_DIMS, B=3), full (bridge
dims, B=2, + actions), b16 (bridge dims, B=16 = config C2's micro-batch, chunked).

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
from tests.golden.gradprobe import N_SAMPLE, probe  # noqa: E402


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
    """bridge.yaml-shaped config (config/train/bridge.yaml:68-181) from dims (text generation:
    use_lm_head + the vlm final norm, as pizero.py:712-714 sets them)."""
    mix = {
        "vlm": dict(hidden_size=d["vlm_hidden"], intermediate_size=d["vlm_inter"],
                    use_final_norm=bool(d.get("vlm_final_norm", False)), cache=True, use_quantize=False, use_lora=False,
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
        image_token_index=d["image_token_index"], use_lm_head=bool(d.get("use_lm_head", False)),
        max_seq_len=d["max_seq_len"], max_image_text_tokens=d["max_seq_len"],
        cond_steps=d["cond_steps"], horizon_steps=d["horizon_steps"],
        action_dim=d["action_dim"], proprio_dim=d["proprio_dim"],
        num_inference_steps=d["num_inference_steps"],
        final_action_clip_value=d["final_action_clip_value"],
        flow_sig_min=d["flow_sig_min"], action_expert_adaptive_mode=None, num_images=d.get("num_images", 1),
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


def run_reference(d, bsz, ragged, dtype, W, inp, grad_names, chunk=None, infer=True, n_sample=N_SAMPLE):
    """Reference forward/backward (+ infer_action) at batch ``bsz``.

    ``chunk``: run the training pass over sub-batches of that size and accumulate
    ``loss_c * (b_c / bsz)`` -- the batch loss is a mean over samples and nothing in the
    forward crosses samples, so this is the same gradient (train.py:350-368 accumulates
    micro-batches the same way); it keeps a B=16 full-size fp32 run inside host memory.
    """
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
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dtype)  # noqa: E731
    ids_all = torch.from_numpy(inp["input_ids"])
    am = torch.from_numpy(inp["attention_mask"])
    mask_all, vpos_all, ppos_all, apos_all = model.build_causal_mask_and_position_ids(am, dtype)
    orig_randn_like, orig_randn = torch.randn_like, torch.randn
    out = {}
    chunk = chunk or bsz
    try:
        total = 0.0
        for s0 in range(0, bsz, chunk):
            sl = slice(s0, min(bsz, s0 + chunk))
            bc = sl.stop - sl.start
            x0 = t(inp["x0"][sl])
            torch.randn_like = lambda *a, **k: x0.clone()
            loss = model(input_ids=ids_all[sl], pixel_values=t(inp["pixel_values"][sl]), causal_mask=mask_all[sl],
                         vlm_position_ids=vpos_all[sl], proprio_position_ids=ppos_all[sl],
                         action_position_ids=apos_all[sl], proprios=t(inp["proprios"][sl]),
                         actions=t(inp["actions"][sl]), t=t(inp["t"][sl]))
            (loss * (bc / bsz)).backward()
            total += loss.detach().double().item() * bc / bsz
            print(f"  chunk {sl.start}:{sl.stop} loss {loss.item():.6f}", flush=True)
        out["loss"] = np.float64(total)
        named = dict(model.named_parameters())
        for n in grad_names:
            p = named[n]
            g = p.grad
            if g is None:
                out["gradnorm/" + n] = np.float64(-1.0)
                continue
            pr = probe(n, g, n_sample)
            out["gradnorm/" + n] = np.float64(pr["norm"])
            out["gsamp/" + n] = pr["sample"].numpy()
            out["gproj/" + n] = pr["proj"].numpy()
        model.zero_grad(set_to_none=True)
        if infer:
            ids, itp_amask = ids_all, model.split_full_mask_into_submasks(mask_all)
            itp, amask = itp_amask
            vpos, ppos, apos, mask = vpos_all, ppos_all, apos_all, mask_all
            noise = t(inp["noise"])
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
        out["mask"] = mask_all[:, 0].float().numpy() if d is TINY_DIMS else np.zeros(1)
    finally:
        torch.randn_like, torch.randn = orig_randn_like, orig_randn
    return out


def all_grad_names(d):
    """Every parameter name the reference's named_parameters() reports (after the tie the
    shared expert tensors appear once, under mixtures.proprio.*, registered first)."""
    from src.model.vla import pizero as pz

    with torch.device("meta"):
        model = pz.PiZero(ref_cfg(d))
    model.tie_action_proprio_weights()
    model.freeze_unused_weights()
    return [n for n, _ in model.named_parameters()]


def make(name, d, bsz, ragged, chunk=None, infer=True, n_sample=N_SAMPLE, tags=("fp32", "bf16")):
    install_stubs()
    if REF not in sys.path:
        sys.path.insert(0, REF)
    torch.set_num_threads(os.cpu_count() or 8)
    W = synth_weights(d, seed=0)
    inp = synth_inputs(d, bsz, seed=0, ragged=ragged)
    gnames = all_grad_names(d)
    res = {}
    for tag in tags:
        dt = {"fp32": torch.float32, "bf16": torch.bfloat16}[tag]
        print(f"[{name}] reference run {tag} ...", flush=True)
        o = run_reference(d, bsz, ragged, dt, W, inp, gnames, chunk=chunk, infer=infer, n_sample=n_sample)
        for k, v in o.items():
            res[f"{tag}/{k}"] = v
        del o
    if "bf16" in tags:
        # the reference's own bf16-vs-fp32 deviation per tensor (sets the GPU tolerances)
        for n in gnames:
            a, b = res.get(f"bf16/gsamp/{n}"), res.get(f"fp32/gsamp/{n}")
            if a is None or b is None:
                continue
            a64, b64 = a.astype(np.float64), b.astype(np.float64)
            nb = np.linalg.norm(b64)
            res[f"bf16/grel/{n}"] = np.float64(np.linalg.norm(a64 - b64) / max(nb, 1e-30))
            res[f"bf16/gcos/{n}"] = np.float64(a64 @ b64 / max(np.linalg.norm(a64) * nb, 1e-30))
            del res[f"bf16/gsamp/{n}"]
    for k in ("input_ids", "attention_mask", "t"):
        res["in/" + k] = inp[k]
    res["grad_names"] = np.array(gnames)
    res["bsz"] = np.int64(bsz)
    res["n_sample"] = np.int64(n_sample)
    path = os.path.join(ROOT, "tests", "golden", f"{name}.npz")
    np.savez_compressed(path, **res)
    print("wrote", path, "loss fp32", res.get("fp32/loss"), "bf16", res.get("bf16/loss"))


if __name__ == "__main__":
    which = sys.argv[1] if len(sys.argv) > 1 else "all"
    if which in ("tiny", "all"):
        make("tiny", TINY_DIMS, 3, ragged=True)
    if which in ("full", "all"):
        make("full", FULL_DIMS, 2, ragged=True)
    if which in ("b16", "all"):
        # config C2's micro-batch (bridge, B=16), fp32 + bf16, accumulated over chunks of 2
        make("b16", FULL_DIMS, 16, ragged=True, chunk=2, infer=False, n_sample=2048)


def make_lr():
    """lr trace of the reference CosineAnnealingWarmupRestarts (utils/optim.py:31-159)."""
    if REF not in sys.path:
        sys.path.insert(0, REF)
    from src.utils.optim import CosineAnnealingWarmupRestarts

    out, states = {}, {}
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
        for i in range(300):
            s.step()
            lrs.append(opt.param_groups[0]["lr"])
            if i + 1 == 137:  # the reference's own state_dict mid-schedule (resume format, optim.py:56-60)
                states[name] = {k: v for k, v in s.state_dict().items()}
        out[name] = np.array(lrs, dtype=np.float64)
        out[name + "_args"] = np.array([first, mult, mx, mn, warm, gamma], dtype=np.float64)
    np.savez_compressed(os.path.join(ROOT, "tests", "golden", "lr_schedule.npz"), **out)
    import json

    with open(os.path.join(ROOT, "tests", "golden", "lr_state.json"), "w") as f:
        json.dump(states, f, indent=1, sort_keys=True)
    print("wrote lr_schedule.npz")


def make_fm_time():
    """Seeded draws of the reference's TrainAgent.sample_fm_time (train.py:216-247), beta and uniform."""
    import types as _t

    if REF not in sys.path:
        sys.path.insert(0, REF)
    import importlib.util

    spec = importlib.util.spec_from_file_location("_ref_train", os.path.join(REF, "src", "agent", "train.py"))
    src_txt = open(spec.origin).read()
    # compile only the sample_fm_time method (the module imports tensorflow/wandb, absent here)
    import ast

    tree = ast.parse(src_txt)
    fn = next(n for c in tree.body if isinstance(c, ast.ClassDef) for n in c.body
              if isinstance(n, ast.FunctionDef) and n.name == "sample_fm_time")
    mod = ast.Module(body=[fn], type_ignores=[])
    ns = {"torch": torch}
    exec(compile(mod, "reference:train.py:sample_fm_time", "exec"), ns)
    out = {}
    for mode in ("beta", "uniform"):
        obj = _t.SimpleNamespace(flow_sampling=mode, flow_t_max=1 - 0.001,
                                 flow_beta_dist=torch.distributions.Beta(1.5, 1))
        torch.manual_seed(1234)
        out[mode] = np.concatenate([ns["sample_fm_time"](obj, b).numpy() for b in (16, 7, 64)])
    np.savez_compressed(os.path.join(ROOT, "tests", "golden", "fm_time.npz"), **out)
    print("wrote fm_time.npz")


def make_time_embed():
    """The reference SinusoidalPosEmb (vla/modules.py:9-22) in fp32 and in bf16 (t in bf16 as in bf16
    training, train.py:311: arange and every op in bf16) for the bridge width / both max periods."""
    if REF not in sys.path:
        sys.path.insert(0, REF)
    from src.model.vla.modules import SinusoidalPosEmb

    t = torch.linspace(0.0, 0.999, 37)
    out = {"t": t.numpy()}
    for P in (100.0, 10000.0):
        m = SinusoidalPosEmb(1024, P)
        out[f"fp32_{int(P)}"] = m(t).numpy()
        out[f"bf16_{int(P)}"] = m(t.to(torch.bfloat16)).float().numpy()
        out[f"t_bf16_{int(P)}"] = t.to(torch.bfloat16).float().numpy()
    np.savez_compressed(os.path.join(ROOT, "tests", "golden", "time_embed.npz"), **out)
    print("wrote time_embed.npz")


TEXT_NEW = 6  # tokens generated after the prefill


def make_text():
    """Greedy text generation through the reference's infer_text with its KV cache (the loop of
    pizero.py:763-790, batched: B=2 ragged prompts, no stop token), TINY_DIMS + lm_head + vlm final
    norm, fp32 and bf16.  Stores the prefill logits, every step's logits and the generated tokens.
    The reference's build_causal_mask_and_position_ids_for_text reads a module-global ``bsz``
    (pizero.py:349, set by its __main__ block); it is set here the same way."""
    install_stubs()
    if REF not in sys.path:
        sys.path.insert(0, REF)
    from src.model.vla import pizero as pz

    d = dict(TINY_DIMS, use_lm_head=True, vlm_final_norm=True)
    torch.set_num_threads(os.cpu_count() or 8)
    W = synth_weights(d, seed=0)
    B = 2
    inp = synth_inputs(d, B, seed=3, ragged=True)
    res = {}
    for tag, dt in (("fp32", torch.float32), ("bf16", torch.bfloat16)):
        torch.manual_seed(0)
        model = pz.PiZero(ref_cfg(d))
        model.tie_action_proprio_weights()
        sd = model.state_dict()
        assert set(sd) == set(param_shapes(d)) | {"lm_head.weight"}, set(sd) ^ set(param_shapes(d))
        model.load_state_dict({k: W[k] for k in sd}, strict=True)
        assert model.lm_head.weight is model.embed_tokens.weight
        model.to(dt).eval()
        pz.bsz = B
        ids = torch.from_numpy(inp["input_ids"])
        am = torch.from_numpy(inp["attention_mask"])
        pix = torch.from_numpy(inp["pixel_values"]).to(dt)
        cache = model.build_text_cache()
        steps, toks = [], []
        with torch.inference_mode():
            for k in range(TEXT_NEW + 1):
                o = model.infer_text(input_ids=ids, pixel_values=pix, attention_mask=am, kv_cache=cache)
                lg = o["logits"].float()
                if k == 0:
                    res[f"{tag}/prefill_logits"] = lg.numpy()
                else:
                    steps.append(lg[:, -1].numpy())
                nxt = lg[:, -1].argmax(-1, keepdim=True)
                toks.append(nxt.numpy())
                ids = nxt
                am = torch.cat([am, torch.ones(B, 1, dtype=am.dtype)], dim=-1)
        res[f"{tag}/step_logits"] = np.stack(steps, 1)
        res[f"{tag}/tokens"] = np.concatenate(toks, 1)
        print(f"[text] {tag} tokens", res[f"{tag}/tokens"].tolist(), flush=True)
    res["in/input_ids"] = inp["input_ids"]
    res["in/attention_mask"] = inp["attention_mask"]
    np.savez_compressed(os.path.join(ROOT, "tests", "golden", "text.npz"), **res)
    print("wrote text.npz")


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "text":
    make_text()

if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "lr":
    make_lr()
    make_fm_time()
    make_time_embed()
