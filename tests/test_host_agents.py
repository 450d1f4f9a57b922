"""Host-side agent logic on CPU: LR schedule vs the reference's own trace, config loader, launcher args."""

import os

import numpy as np
import torch

from tests.conftest import PKG, ROOT
from tests.oracle_helpers import load_golden


def test_lr_schedule_matches_reference_trace():
    from src.utils.optim import CosineAnnealingWarmupRestarts

    g = load_golden("lr_schedule")
    for name in ("bridge", "restarts", "mult"):
        first, mult, mx, mn, warm, gamma = g[name + "_args"]
        p = [torch.nn.Parameter(torch.zeros(1))]
        opt = torch.optim.SGD(p, lr=1.0)
        s = CosineAnnealingWarmupRestarts(opt, first_cycle_steps=int(first), cycle_mult=mult, max_lr=mx, min_lr=mn,
                                          warmup_steps=int(warm), gamma=gamma)
        lrs = [opt.param_groups[0]["lr"]]
        for _ in range(len(g[name]) - 1):
            s.step()
            lrs.append(opt.param_groups[0]["lr"])
        np.testing.assert_allclose(np.array(lrs), g[name], rtol=1e-9, atol=1e-15, err_msg=name)


def test_bridge_config_resolves_hot_path_keys():
    from src.utils.config import load_config

    c = load_config(os.path.join(PKG, "config", "train", "bridge.yaml"))
    assert c.max_image_text_tokens == 276 and c.horizon_steps == 4
    assert c.joint.config.mixture.action.rope_theta == 100.0
    assert c.joint.config.mixture.vlm.use_quantize is False
    assert isinstance(c.vision.config.layer_norm_eps, float) and c.action_lr == 5e-5


def test_param_counts_match_reference_survey():
    """3.2381 B unique params, 0.3146 B action expert, 2.2913 B trained VLM."""
    from src.model.vla.pizero import PiZero
    from src.utils.config import load_config

    c = load_config(os.path.join(PKG, "config", "train", "bridge.yaml"))
    m = PiZero(c, device="meta", init="none") if False else None  # noqa: F841
    m = PiZero(c, init="none")
    m.tie_action_proprio_weights()
    m.freeze_unused_weights()
    assert abs(sum(p.numel() for p in m.parameters()) / 1e9 - 3.2381) < 1e-3
    assert abs(sum(p.numel() for p in m.action_expert_parameters) / 1e9 - 0.3146) < 1e-3
    assert abs(sum(p.numel() for p in m.trainable_vlm_parameters) / 1e9 - 2.2913) < 1e-3


def test_launcher_parses_overrides():
    import importlib.util

    spec = importlib.util.spec_from_file_location("pz_run", os.path.join(PKG, "scripts", "run.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    assert mod._parse_value("16") == 16 and mod._parse_value("5e-5") == 5e-5 and mod._parse_value("true") is True
    assert os.path.exists(os.path.join(ROOT, "include", "pz_abi.h"))


def test_lr_scheduler_state_dict_matches_reference_and_resumes():
    """state_dict keys/values = the reference's own (tests/golden/lr_state.json, written by the reference
    class after 137 steps); loading that state continues the reference lr trace exactly."""
    import json

    from src.utils.optim import CosineAnnealingWarmupRestarts

    g = load_golden("lr_schedule")
    with open(os.path.join(ROOT, "tests", "golden", "lr_state.json")) as f:
        ref_states = json.load(f)
    for name, ref in ref_states.items():
        first, mult, mx, mn, warm, gamma = g[name + "_args"]
        mk = lambda: CosineAnnealingWarmupRestarts(  # noqa: E731
            torch.optim.SGD([torch.nn.Parameter(torch.zeros(1))], lr=1.0), first_cycle_steps=int(first),
            cycle_mult=mult, max_lr=mx, min_lr=mn, warmup_steps=int(warm), gamma=gamma)
        s = mk()
        for _ in range(137):
            s.step()
        mine = s.state_dict()
        assert set(mine) == set(ref), (name, set(mine) ^ set(ref))
        for k, v in ref.items():
            np.testing.assert_allclose(np.array(mine[k], dtype=np.float64), np.array(v, dtype=np.float64),
                                       rtol=1e-12, err_msg=f"{name}.{k}")
        r = mk()
        r.load_state_dict(ref)
        lrs = [r.optimizer.param_groups[0]["lr"]]
        for _ in range(len(g[name]) - 138):
            r.step()
            lrs.append(r.optimizer.param_groups[0]["lr"])
        np.testing.assert_allclose(np.array(lrs), g[name][137:], rtol=1e-9, atol=1e-15, err_msg=name)


def test_sample_fm_time_matches_reference_seeded():
    """train.py:239-247 draws, seeded, against the reference method's own output (tests/golden/fm_time.npz)."""
    from src.agent.train import sample_fm_time

    g = load_golden("fm_time")
    torch.manual_seed(1234)
    beta = torch.distributions.Beta(1.5, 1)
    mine = np.concatenate([sample_fm_time(b, "beta", beta, 1 - 0.001).numpy() for b in (16, 7, 64)])
    np.testing.assert_array_equal(mine, g["beta"])
    torch.manual_seed(1234)
    mine = np.concatenate([sample_fm_time(b, "uniform").numpy() for b in (16, 7, 64)])
    np.testing.assert_array_equal(mine, g["uniform"])
    assert (g["beta"] > 0).all() and (g["beta"] <= 0.999).all()
