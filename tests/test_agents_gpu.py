"""Agents on the MI355X: TrainAgent updates (tiny model), EvalAgent chunk via hipGraph == eager."""

import pytest
import torch

from tests.golden.make_golden import ref_cfg
from tests.oracle_helpers import O

pytestmark = pytest.mark.gpu


def _cfg():
    c = ref_cfg(O.TINY_DIMS)
    c.update(dict(global_batch_size=8, per_device_batch_size=4, action_lr=1e-3, vlm_lr=1e-3,
                  action_weight_decay=0.0, vlm_weight_decay=0.0, max_grad_norm=1.0, n_updates=3, log_freq=1,
                  train_vlm=True, use_bf16=True, flow_sampling="beta", load_pretrained_weights=False,
                  action_lr_scheduler=dict(first_cycle_steps=100, min_lr=1e-8, warmup_steps=2),
                  vlm_lr_scheduler=dict(first_cycle_steps=100, min_lr=1e-8, warmup_steps=2)))
    return c


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def test_train_agent_updates_weights():
    from src.agent.train import TrainAgent

    a = TrainAgent(_cfg())
    w0 = a.model.action_decoder.weight.detach().float().clone()
    v0 = a.model.vision_tower.vision_model.encoder.layers[0].mlp.fc1.weight.detach().float().clone()
    a.run()
    assert a.cnt_update == 3 and a.cnt_batch == 6
    assert not torch.equal(w0, a.model.action_decoder.weight.detach().float())
    assert not torch.equal(v0, a.model.vision_tower.vision_model.encoder.layers[0].mlp.fc1.weight.detach().float())
    # the frozen last-layer vlm v_proj never moves (pizero.py:231)
    assert not a.model.joint_model.mixtures["vlm"].layers[-1].self_attn.v_proj.weight.requires_grad
    assert a.action_optimizer.param_groups[0]["lr"] > 1e-8


def test_eval_agent_graph_matches_eager():
    from src.agent.eval import EvalAgent
    from src.agent.train import SyntheticBridgeDataset

    ag = EvalAgent(_cfg(), use_graph=True)
    b = next(iter(SyntheticBridgeDataset(_cfg(), 2, seed=3)))
    pix = (b["pixel_values"].float() / 255 - 0.5) / 0.5
    noise = torch.randn(2, 4, 7, device="cuda")
    a_graph = ag.infer_chunk(b["input_ids"], b["attention_mask"], pix, b["proprio"], noise=noise)
    ag.use_graph = False
    a_eager = ag.infer_chunk(b["input_ids"], b["attention_mask"], pix, b["proprio"], noise=noise)
    assert a_graph.shape == (2, 4, 7)
    assert torch.allclose(a_graph.float(), a_eager.float(), atol=1e-2)
