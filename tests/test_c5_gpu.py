"""Config C5 (BASELINE.json configs[4]: the Pi0-paper shape, 3 images = 768 image tokens + 20 text
+ 1 proprio + an action chunk of 50, L = 839) against the REFERENCE's own JointModel.

The reference PiZero takes one image per sample (pizero.py:389-413), so C5 is composed at the
JointModel level; tests/golden/make_golden_c5.py ran the reference JointModel at
full Gemma-2B / action-expert dims (proprio tied to action) on generator-defined embeddings with
the reference block mask (8 pad text tokens) and loss = sum(action_hidden * R), in fp32 and bf16.
Here the native engine runs the same JointModel forward + backward (``Engine.joint_train``) on the
same embeddings (pz_fill_uniform reproduces oracle/synth.py bit-exactly) in bf16 on the GPU.
Tolerance = max(3x the reference's own bf16-vs-fp32 deviation, a floor): action hidden rel-L2
<= 3e-2; gradient norms rel <= max(3*dev, 0.05), gradient-head cosine >= 0.97.
Precision: bf16 (the fp8 variant of C5 is not built).  Both joint-attention kernels are checked.
"""

import numpy as np
import pytest
import torch

from tests.oracle_helpers import O, load_golden
from tests.pizero_gpu_helpers import build_gpu_model

pytestmark = pytest.mark.gpu

C5_DIMS = dict(O.FULL_DIMS, max_seq_len=788, horizon_steps=50)
C5_INPUTS = {"c5/embeds.vlm": (1, 788, 2048), "c5/embeds.proprio": (1, 1, 1024), "c5/embeds.action": (1, 50, 1024),
             "c5/R": (1, 50, 1024)}


@pytest.fixture(scope="module")
def c5():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from oracle.synth import tensor_seed
    from pizero_native import ops

    g = load_golden("c5")
    m = build_gpu_model(C5_DIMS)
    inp = {}
    for k, shp in C5_INPUTS.items():
        t = torch.empty(shp, device="cuda", dtype=torch.float32)
        ops.fill_uniform(t, tensor_seed(k, 0), 0.0, 1.0)
        inp[k] = t
    am = torch.zeros(1, 788, dtype=torch.int64)
    am[:, : int(g["cnt"])] = 1
    mask, vpos, ppos, apos = m.build_causal_mask_and_position_ids(am, torch.bfloat16)
    pos = {"vlm": vpos.to("cuda"), "expert": m._cat_pos(ppos, apos)}
    cnt = m._prefix_counts(mask.to("cuda"))
    assert int(cnt[0]) == int(g["cnt"])
    return g, m, inp, pos, cnt


def _rel(a, b):
    return float(np.linalg.norm(a - b) / (np.linalg.norm(b) + 1e-30))


@pytest.mark.parametrize("joint_attn", ["gemm", "flash"])
def test_c5_joint_model_forward_backward(c5, joint_attn):
    g, m, inp, pos, cnt = c5
    eng = m._engine()
    eng.joint_flash = joint_attn == "flash"
    try:
        m.zero_grad(set_to_none=True)
        emb = {n: inp[f"c5/embeds.{n}"].to(torch.bfloat16) for n in ("vlm", "proprio", "action")}
        R = inp["c5/R"]
        m._arena.ensure_grad()
        out, demb = eng.joint_train(emb, pos, cnt, R)
        m._attach_grads()
        torch.cuda.synchronize()
    finally:
        eng.joint_flash = False
    ref, refb = g["fp32/action_hidden"], g["bf16/action_hidden"]
    mine = out.float().cpu().numpy()
    tol = max(3 * _rel(refb, ref), 3e-2)
    assert _rel(mine, ref) <= tol, (_rel(mine, ref), _rel(refb, ref))
    bad = []
    for n in ("vlm", "proprio", "action"):
        gd = demb[n].double()
        r, rb = float(g[f"fp32/dembeds/{n}/norm"]), float(g[f"bf16/dembeds/{n}/norm"])
        t = max(3 * abs(rb - r) / r, 0.05)
        head = gd.flatten()[:64].cpu().numpy()
        rh = g[f"fp32/dembeds/{n}/head"]
        cos = float(np.dot(head, rh) / (np.linalg.norm(head) * np.linalg.norm(rh) + 1e-30))
        if abs(gd.norm().item() - r) > t * r or cos < 0.97:
            bad.append(("dembeds/" + n, gd.norm().item(), r, rb, cos))
    params = dict(m.named_parameters())
    for n in [str(x) for x in g["grad_names"]]:
        r = float(g[f"fp32/gradnorm/{n}"])
        full = "joint_model." + n
        p = params.get(full)
        if p is None:
            p = params.get(full.replace("mixtures.action.", "mixtures.proprio."))
        if r < 0:
            assert p is None or p.grad is None or not p.requires_grad, n
            continue
        if r == 0 and (p is None or p.grad is None or not p.requires_grad):
            continue  # reachable but gradient exactly 0 in the reference (frozen/unused here)
        if p is None or p.grad is None:
            bad.append((n, None, r))
            continue
        gg = p.grad.double()
        mine_n = gg.norm().item()
        rb = float(g[f"bf16/gradnorm/{n}"])
        t = max(3 * abs(rb - r) / max(r, 1e-30), 0.05)
        head = gg.flatten()[:64].cpu().numpy()
        rh = g[f"fp32/gradhead/{n}"]
        cos = float(np.dot(head, rh) / (np.linalg.norm(head) * np.linalg.norm(rh) + 1e-30))
        ok = (r == 0 and mine_n == 0) or (abs(mine_n - r) <= t * r and
                                         (np.linalg.norm(rh) < 1e-12 * r or cos >= 0.97))
        if not ok:
            bad.append((n, mine_n, r, rb, cos))
    assert not bad, "\n".join(map(str, bad))
