"""Text generation (PiZero.infer_text, pizero.py:559-593) on the GPU against the reference's own greedy
KV-cache loop (tests/golden/text.npz, written by tests/golden/make_golden.py text).

The native path: prefill = the vlm mixture over the prompt (SigLIP image tokens merged), flash attention
with no mask (the all-zeros text mask, pizero.py:336-365), then the vlm final norm and the lm_head tied to
embed_tokens; each decode step = ONE token per sample through the few-row kernels (fused q|k|v + RoPE
GEMV writing the static cache, pz_decode_attn without a mask, GEMV o / gate|up / down).  Steps are
teacher-forced with the reference's tokens, so every step compares the same computation.

Tolerance: the reference's own bf16-vs-fp32 logit deviation on the same inputs (rel-L2 per step),
times 2, floored at 2% -- the same rule as the gradient gates."""

import numpy as np
import pytest
import torch

from tests.oracle_helpers import O, load_golden
from tests.pizero_gpu_helpers import build_gpu_model

pytestmark = pytest.mark.gpu

TEXT_DIMS = dict(O.TINY_DIMS, use_lm_head=True, vlm_final_norm=True)


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.fixture(scope="module")
def setup():
    from oracle.synth import synth_inputs

    g = load_golden("text")
    m = build_gpu_model(TEXT_DIMS)
    m.eval()
    assert m.lm_head.weight is m.embed_tokens.weight
    inp = synth_inputs(TEXT_DIMS, 2, seed=3, ragged=True)
    np.testing.assert_array_equal(g["in/input_ids"], inp["input_ids"])
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a))  # noqa: E731
    gi = dict(ids=T(inp["input_ids"]).cuda(), pix=T(inp["pixel_values"]).cuda().to(torch.bfloat16),
              am=T(inp["attention_mask"]).cuda())
    return g, m, gi


def _rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / np.linalg.norm(b))


def _tol(g, key, sl=slice(None)):
    return max(0.02, 2 * _rel(g["bf16/" + key][sl], g["fp32/" + key][sl]))


def _generate(m, gi, toks, kv_cache):
    """prefill + teacher-forced decode steps (the reference loop, pizero.py:763-790)"""
    am = gi["am"]
    out = m.infer_text(gi["ids"], gi["pix"], am, kv_cache=kv_cache)
    pre = out["logits"].float().cpu().numpy()
    steps = []
    for k in range(toks.shape[1] - 1):
        am = torch.cat([am, torch.ones(am.shape[0], 1, dtype=am.dtype, device=am.device)], dim=-1)
        o = m.infer_text(toks[:, k:k + 1].cuda(), gi["pix"], am, kv_cache=kv_cache)
        assert o["logits"].shape[:2] == (am.shape[0], 1)
        steps.append(o["logits"][:, -1].float().cpu().numpy())
    return pre, np.stack(steps, 1)


def test_text_generation_matches_reference(setup):
    g, m, gi = setup
    toks = torch.from_numpy(g["fp32/tokens"])
    cache = m.build_text_cache()
    pre, steps = _generate(m, gi, toks, cache)
    assert cache.num_items() == gi["ids"].shape[1] + toks.shape[1] - 1
    assert np.isfinite(pre).all() and np.isfinite(steps).all()
    r_pre = _rel(pre, g["fp32/prefill_logits"])
    assert r_pre <= _tol(g, "prefill_logits"), (r_pre, _tol(g, "prefill_logits"))
    for k in range(steps.shape[1]):
        r = _rel(steps[:, k], g["fp32/step_logits"][:, k])
        tol = _tol(g, "step_logits", (slice(None), k))
        assert r <= tol, (k, r, tol)
    # greedy tokens where the reference's top-2 margin is clear of bf16 noise
    ref_all = np.concatenate([g["fp32/prefill_logits"][:, -1:], g["fp32/step_logits"]], 1)
    mine_all = np.concatenate([pre[:, -1:], steps], 1)
    top2 = np.sort(ref_all, -1)[..., -2:]
    clear = (top2[..., 1] - top2[..., 0]) > 0.05 * np.abs(ref_all).max()
    assert clear.any()
    np.testing.assert_array_equal(mine_all.argmax(-1)[clear], g["fp32/tokens"][clear])


def test_text_prefill_without_cache_equals_cached(setup):
    """kv_cache=None (a standalone prefill, like the reference) gives the cached prefill's logits"""
    _, m, gi = setup
    a = m.infer_text(gi["ids"], gi["pix"], gi["am"])["logits"]
    b = m.infer_text(gi["ids"], gi["pix"], gi["am"], kv_cache=m.build_text_cache())["logits"]
    assert "kv_cache" not in m.infer_text(gi["ids"], gi["pix"], gi["am"])
    assert torch.equal(a, b)


def test_text_decode_kernels_match_unfused(setup, monkeypatch):
    """the few-row decode path (GEMV + pz_decode_attn, no mask) against the general path (GEMM + flash
    with key split) on the same cache: bf16 rounding differences only"""
    g, m, gi = setup
    toks = torch.from_numpy(g["fp32/tokens"])
    _, fast = _generate(m, gi, toks, m.build_text_cache())
    monkeypatch.setenv("PZ_GEMV", "0")
    _, slow = _generate(m, gi, toks, m.build_text_cache())
    assert _rel(fast, slow) <= 0.01, _rel(fast, slow)


def test_text_cache_grows(setup):
    """a cache filled past its capacity is regrown with the cached rows kept"""
    g, m, gi = setup
    toks = torch.from_numpy(g["fp32/tokens"])
    cache = m.build_text_cache()
    m.infer_text(gi["ids"], gi["pix"], gi["am"], kv_cache=cache)
    cap = cache.k.shape[2]
    k0 = cache.k[:, :, :cache.num_items()].clone()
    am = gi["am"]
    n_before = cache.num_items()
    for _ in range(cap - n_before + 3):
        am = torch.cat([am, torch.ones(am.shape[0], 1, dtype=am.dtype, device=am.device)], dim=-1)
        m.infer_text(toks[:, :1].cuda(), gi["pix"], am, kv_cache=cache)
    assert cache.k.shape[2] > cap and cache.num_items() == cap + 3
    assert torch.equal(cache.k[:, :, :n_before], k0)


def test_text_generation_fp8(setup):
    """infer_text under PiZero.use_fp8_inference (C5's fp8 weights: prefill W8A8 where the widths allow,
    decode rows W8A16): logits stay close to the bf16 path's (fp8 e4m3 keeps 3 mantissa bits; parity vs
    an fp8 reference is unpinned -- the reference has no fp8 path)"""
    g, m, gi = setup
    toks = torch.from_numpy(g["fp32/tokens"])
    pre16, steps16 = _generate(m, gi, toks, m.build_text_cache())
    try:
        m.use_fp8_inference(True)
        pre8, steps8 = _generate(m, gi, toks, m.build_text_cache())
    finally:
        m.use_fp8_inference(False)
    r_pre, r_steps = _rel(pre8, pre16), _rel(steps8, steps16)
    print(f"fp8 vs bf16 text logits rel-L2: prefill {r_pre:.4g}, decode {r_steps:.4g}")
    assert np.isfinite(pre8).all() and np.isfinite(steps8).all()
    assert r_pre < 0.1 and r_steps < 0.1, (r_pre, r_steps)
