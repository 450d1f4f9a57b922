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


def _one_update(agent, batch, seed):
    from pizero_native.optim import clip_grad_norm_

    torch.manual_seed(seed)
    inputs = agent.preprocess_batch(batch)
    loss = agent.model(**inputs, noise=torch.zeros(inputs["actions"].shape, device="cuda"))
    loss.backward()
    clip_grad_norm_(agent.optimizers, agent.max_grad_norm)
    for o in agent.optimizers:
        o.step()
        o.zero_grad(set_to_none=True)
    agent.action_lr_scheduler.step()
    agent.vlm_lr_scheduler.step()


def test_save_resume_roundtrip(tmp_path):
    """train.py:497-560: save_training -> TrainAgent(resume_checkpoint_path) restores weights, counters,
    both optimizers' moments/steps and both schedulers; the next update is bitwise identical."""
    from src.agent.train import SyntheticBridgeDataset, TrainAgent

    c = _cfg()
    c.update(dict(log_dir=str(tmp_path), n_updates=2, save_model_freq=2))
    a = TrainAgent(c).run()
    path = tmp_path / "checkpoint" / "step2.pt"
    assert path.exists()
    c2 = _cfg()
    c2.update(dict(resume_checkpoint_path=str(path)))
    b = TrainAgent(c2)
    assert (b.cnt_update, b.cnt_batch) == (2, a.cnt_batch - 1)
    sa, sb = a.model.state_dict(), b.model.state_dict()
    assert all(torch.equal(sa[k], sb[k]) for k in sa)
    for oa, ob in ((a.action_optimizer, b.action_optimizer), (a.vlm_optimizer, b.vlm_optimizer)):
        da, db = oa.state_dict(), ob.state_dict()
        assert da["param_groups"][0]["step"] == db["param_groups"][0]["step"] == 2
        assert da["param_groups"][0]["lr"] == db["param_groups"][0]["lr"]
        assert set(da["state"]) == set(db["state"]) and da["state"]
        for i in da["state"]:  # 8-bit state by default: codes, absmax, qmaps (fp32 for small tensors)
            for k, v in da["state"][i].items():
                if isinstance(v, torch.Tensor):
                    assert torch.equal(v, db["state"][i][k]), (i, k)
    assert a.action_lr_scheduler.last_epoch == b.action_lr_scheduler.last_epoch == 1  # 2 steps from -1
    batch = next(iter(SyntheticBridgeDataset(c, 4, seed=9)))
    _one_update(a, batch, 5)
    _one_update(b, batch, 5)
    sa, sb = a.model.state_dict(), b.model.state_dict()
    assert all(torch.equal(sa[k], sb[k]) for k in sa)
