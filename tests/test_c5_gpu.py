"""Config C5 (BASELINE.json configs[4]: the Pi0-paper shape, 3 images = 768 image tokens + 20 text
+ 1 proprio + an action chunk of 50, L = 839) against the REFERENCE's own JointModel.

The reference PiZero takes one image per sample (pizero.py:389-413), so C5 is composed at the
JointModel level; tests/golden/make_golden_c5.py ran the reference JointModel at
full Gemma-2B / action-expert dims (proprio tied to action) on generator-defined embeddings with
the reference block mask (8 pad text tokens) and loss = sum(action_hidden * R), in fp32 and bf16.
Here the native engine runs the same JointModel forward + backward (``Engine.joint_train``) on the
same embeddings (pz_fill_uniform reproduces oracle/synth.py bit-exactly) in bf16 on the GPU.
Tolerance: action hidden rel-L2 <= max(3x the reference's own bf16-vs-fp32 deviation, 3e-2); the
input-embedding gradients and EVERY JointModel parameter gradient pass the probe gate of
tests/pizero_gpu_helpers.py (sample rel-L2 <= 8 %, cosine >= 0.995, whole-tensor projections).
Precision: bf16 training-shape JointModel (C5's fp8 path is an inference path: its full-shape chunk is
checked in tests/test_c5_pizero_gpu.py and its bridge-size reference gate in
tests/test_pizero_gpu.py::test_full_actions_fp8).  Both joint-attention kernels are checked.
"""

import types

import numpy as np
import pytest
import torch

from tests.oracle_helpers import O, load_golden
from tests.pizero_gpu_helpers import build_gpu_model, check_grads_probe

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


@pytest.mark.parametrize("joint_attn", ["gemm", "flash", "probs"])
def test_c5_joint_model_forward_backward(c5, joint_attn):
    g, m, inp, pos, cnt = c5
    eng = m._engine()
    prev = eng.joint_flash, eng.joint_probs
    eng.joint_flash, eng.joint_probs = joint_attn == "flash", joint_attn == "probs"
    try:
        m.zero_grad(set_to_none=True)
        emb = {n: inp[f"c5/embeds.{n}"].to(torch.bfloat16) for n in ("vlm", "proprio", "action")}
        R = inp["c5/R"]
        m._arena.ensure_grad()
        out, demb = eng.joint_train(emb, pos, cnt, R)
        m._attach_grads()
        torch.cuda.synchronize()
    finally:
        eng.joint_flash, eng.joint_probs = prev
    ref, refb = g["fp32/action_hidden"], g["bf16/action_hidden"]
    mine = out.float().cpu().numpy()
    tol = max(3 * _rel(refb, ref), 3e-2)
    assert _rel(mine, ref) <= tol, (_rel(mine, ref), _rel(refb, ref))
    params = {n: p for n, p in m.named_parameters()}
    for n in ("vlm", "proprio", "action"):
        params["dembeds." + n] = types.SimpleNamespace(grad=demb[n], requires_grad=True)

    def name_map(n):
        return n if n.startswith("dembeds.") else "joint_model." + n

    # (the last vlm layer's v_proj is frozen by freeze_unused_weights, pizero.py:224-256: skipped)
    check_grads_probe(g, params, name_map=name_map, label=f"C5 {joint_attn}", skip_frozen=True)
