"""FusedAdamW + the folded clip against torch (train.py:371-379: clip_grad_norm_ then AdamW.step).

Parameters and gradients are views of one flat bf16 arena (the layout FusedAdamW runs over); the
torch reference runs torch.nn.utils.clip_grad_norm_ + torch.optim.AdamW on fp32 copies of the same
parameters and gradients.  Also: the clip is bitwise deterministic (no atomics), and state_dict()
round-trips through torch.optim.AdamW's layout.
"""

import pytest
import torch

pytestmark = pytest.mark.gpu

SHAPES = [(64, 96), (257,), (33, 7), (1024,), (128, 130)]


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _arena(seed, scale):
    g = torch.Generator(device="cpu").manual_seed(seed)
    n = sum(int(torch.tensor(s).prod()) for s in SHAPES)
    pad = [(-int(torch.tensor(s).prod())) % 8 for s in SHAPES]  # keep every tensor 16-B aligned
    tot = n + sum(pad)
    w = (torch.rand(tot, generator=g) * 2 - 1).to("cuda", torch.bfloat16)
    gr = ((torch.rand(tot, generator=g) * 2 - 1) * scale).to("cuda", torch.bfloat16)
    ps, o = [], 0
    for s, pd in zip(SHAPES, pad):
        k = int(torch.tensor(s).prod())
        p = torch.nn.Parameter(w[o:o + k].view(s))
        p.grad = gr[o:o + k].view(s)
        ps.append(p)
        o += k + pd
    return ps


@pytest.mark.parametrize("scale", [10.0, 1e-3])  # clip active / inactive
def test_clip_and_adamw_match_torch(scale):
    from pizero_native.optim import FusedAdamW, clip_grad_norm_

    ps = _arena(0, scale)
    a, b = ps[:2], ps[2:]
    ref = [torch.nn.Parameter(p.detach().float().clone()) for p in ps]
    oa = FusedAdamW(a, lr=1e-2, weight_decay=0.01)
    ob = FusedAdamW(b, lr=5e-3, weight_decay=0.0)
    ra = torch.optim.AdamW(ref[:2], lr=1e-2, weight_decay=0.01)
    rb = torch.optim.AdamW(ref[2:], lr=5e-3, weight_decay=0.0)
    for _ in range(3):
        for p, r in zip(ps, ref):
            r.grad = p.grad.detach().float().clone()
        n_ref = torch.nn.utils.clip_grad_norm_(ref, 1.0)
        n_mine = clip_grad_norm_([oa, ob], 1.0)
        assert abs(n_mine.item() - n_ref.item()) <= 1e-4 * n_ref.item()
        ra.step()
        rb.step()
        oa.step()
        ob.step()
    for p, r in zip(ps, ref):
        torch.testing.assert_close(p.detach().float(), r.detach(), atol=1.5e-2, rtol=0)  # bf16 weights
    assert oa.param_groups[0]["step"] == 3


def test_clip_norm_is_deterministic():
    from pizero_native.optim import FusedAdamW, clip_grad_norm_

    ps = _arena(1, 3.0)
    o = FusedAdamW(ps, lr=1e-3)
    n1 = clip_grad_norm_([o], 1.0).clone()
    c1 = o._gscale.clone()
    for _ in range(5):
        n2 = clip_grad_norm_([o], 1.0)
        assert torch.equal(n1, n2) and torch.equal(c1, o._gscale)


def test_state_dict_roundtrip_via_torch_adamw():
    from pizero_native.optim import FusedAdamW

    ps = _arena(2, 1.0)
    o = FusedAdamW(ps, lr=1e-3)
    for _ in range(2):
        o.step()
    sd = o.state_dict()
    assert set(sd["state"][0]) == {"step", "exp_avg", "exp_avg_sq"} and sd["param_groups"][0]["step"] == 2
    ref = [torch.nn.Parameter(p.detach().float().clone()) for p in ps]
    t = torch.optim.AdamW(ref, lr=1e-3)
    t.load_state_dict(sd)
    for i, r in enumerate(ref):
        torch.testing.assert_close(t.state[r]["exp_avg"], sd["state"][i]["exp_avg"].float())
    # and back: torch's state into a fresh FusedAdamW
    ps2 = _arena(2, 1.0)
    o2 = FusedAdamW(ps2, lr=1e-3)
    o2.load_state_dict(t.state_dict())
    sd2 = o2.state_dict()
    assert sd2["param_groups"][0]["step"] == 2
    for i in sd["state"]:
        assert torch.equal(sd2["state"][i]["exp_avg"], sd["state"][i]["exp_avg"])
        assert torch.equal(sd2["state"][i]["exp_avg_sq"], sd["state"][i]["exp_avg_sq"])
