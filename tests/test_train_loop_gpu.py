"""Several optimizer steps of the benched training loop with uninitialised memory poisoned.

Round 5's driver bench ended with a NaN loss while every builder box gave the same finite loss: the step read
memory it had not written -- the SigLIP dQ kernel's 32-wide k step ran past row 255 of one buffer's V image into
the other buffer's K image, LDS that a previous kernel left there or that an LDS-DMA was still filling, and met
it with zeroed dO columns (0 x NaN = NaN).  The single-step parity tests could not see that: a fresh process's
LDS and allocator pool happened to hold finite bytes.  Here the same loop (micro-batch 64 x accumulation 2,
full Pi0, gradient clip + 8-bit AdamW on both parameter groups, the action expert's backward on its side
stream) runs twice from the same weights:

  * clean: as the bench runs it;
  * poisoned: every block of the caching allocator's pool (large and small) and every engine / GEMM workspace
    filled with 0xff bytes (NaN in bf16 and fp32) before the run, and every CU's LDS filled with NaN before EVERY
    kernel launch (``_lib.set_poison_lds``: pz_debug_poison_lds on the launch's stream).

Both must give finite losses and gradient norms at every step and be BITWISE equal (the path is deterministic:
no atomics, fixed-order reductions) -- a kernel that reads an unwritten byte, or races, breaks one or the other.
Reference: train.py:316-410 (the accumulation loop, clip, two AdamW8bit groups).
"""

import math

import pytest
import torch

from tests.oracle_helpers import O
from tests.pizero_gpu_helpers import build_gpu_model, gpu_inputs

pytestmark = pytest.mark.gpu

STEPS, ACCUM, REPEAT = 3, 2, 4  # 3 optimizer steps of 2 micro-batches of 16 x 4 = 64 samples


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def poison_allocator():
    """Fill (nearly) all free device memory with 0xff through the caching allocator and free it again: later
    torch.empty blocks -- large (> 1 MB) and small pool alike -- come back holding NaN bytes."""
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    free, _ = torch.cuda.mem_get_info()
    big = []
    for _ in range(int(free * 0.85) // (1 << 30)):
        big.append(torch.empty(1 << 30, dtype=torch.uint8, device="cuda").fill_(0xFF))
    small = [torch.empty(512 << 10, dtype=torch.uint8, device="cuda").fill_(0xFF) for _ in range(2048)]
    torch.cuda.synchronize()
    n = len(big)
    del big, small
    return n


def reset_workspaces(m):
    """drop the engine's and the GEMM front-end's lazily allocated scratch, so it is re-allocated (from the
    poisoned pool) by the next step; zero-initialised buffers (joint K/V pads, padded weights) are re-created as
    zeros by the engine itself"""
    from pizero_native import ops

    ops._WS.clear()
    e = m._engine()
    e._ws.clear()
    e._tables.clear()
    e._jkv_holder = None


def train(m, batches, poison):
    from pizero_native import _lib
    from pizero_native.optim import FusedAdamW, clip_grad_norm_

    opt_a = FusedAdamW(m.action_expert_parameters, lr=1e-4, weight_decay=0.0, state_bits=8)
    opt_v = FusedAdamW(m.trainable_vlm_parameters, lr=5e-5, weight_decay=0.0, state_bits=8)
    reset_workspaces(m)
    if poison:
        print(f"[poison] {poison_allocator()} GiB of the allocator pool filled with 0xff; LDS poisoned per launch")
        _lib.set_poison_lds(0xFFFFFFFF)
    losses, norms = [], []
    try:
        for _ in range(STEPS):
            for i in range(ACCUM):
                b = batches[i]
                loss = m(input_ids=b["input_ids"], pixel_values=b["pixel_values"], causal_mask=b["causal_mask"],
                         vlm_position_ids=b["vpos"], proprio_position_ids=b["ppos"], action_position_ids=b["apos"],
                         proprios=b["proprios"], actions=b["actions32"], t=b["t32"], noise=b["x0"])
                (loss / ACCUM).backward()
                losses.append(loss.item())  # the reference logs every micro-batch's loss (train.py:399-410)
            norms.append(clip_grad_norm_([opt_a, opt_v], 1.0).item())
            opt_a.step()
            opt_v.step()
            opt_a.zero_grad(set_to_none=True)
            opt_v.zero_grad(set_to_none=True)
        torch.cuda.synchronize()
    finally:
        _lib.set_poison_lds(None)
    return losses, norms, m._arena.data.clone()


def test_multistep_training_poisoned_memory_bitwise():
    d = O.FULL_DIMS
    m = build_gpu_model(d)
    g0 = gpu_inputs(m, d, 16, repeat=REPEAT)
    # the second micro-batch: the same 64 samples in another row order (distinct GEMM rows per sample)
    perm = torch.roll(torch.arange(16 * REPEAT), 7)
    g1 = {k: (v[perm.to(v.device)] if v.shape[0] == 16 * REPEAT else v) for k, v in g0.items()}
    w0 = m._arena.data.clone()
    clean = train(m, [g0, g1], poison=False)
    with torch.no_grad():
        m._arena.data.copy_(w0)
    dirty = train(m, [g0, g1], poison=True)
    print(f"[train loop] clean losses {clean[0]} norms {clean[1]}")
    print(f"[train loop] poisoned losses {dirty[0]} norms {dirty[1]}")
    for name, (lc, nc, _) in (("clean", clean), ("poisoned", dirty)):
        assert all(math.isfinite(v) for v in lc + nc), (name, lc, nc)
    assert clean[0] == dirty[0], "micro-batch losses differ between the clean and the poisoned run"
    assert clean[1] == dirty[1], "gradient norms differ between the clean and the poisoned run"
    assert torch.equal(clean[2], dirty[2]), "weights after 3 optimizer steps differ (clean vs poisoned)"
    # the weights moved (the optimizer ran) and stayed finite
    assert not torch.equal(clean[2], w0)
    assert bool(torch.isfinite(clean[2].float()).all())


def test_check_finite_names_first_bad_stage():
    """PZ_CHECK_FINITE (engine._chk): a NaN planted in SigLIP layer 1's fc1 weight is reported at the first stage
    whose outputs it reaches -- 'siglip fwd layer 1', tensor g1 -- with the native launches since the last check"""
    from tests.pizero_gpu_helpers import run_loss

    d = O.TINY_DIMS
    m = build_gpu_model(d)
    gi = gpu_inputs(m, d, 2)
    e = m._engine()
    e.check_finite = True
    from pizero_native import _lib

    prev = _lib._RECENT[0]
    _lib._RECENT[0] = []
    try:
        run_loss(m, gi)  # clean: no error
        w = m._arena.view("vision_tower.vision_model.encoder.layers.1.mlp.fc1.weight")
        with torch.no_grad():
            w.view(-1)[0] = float("nan")
        with pytest.raises(FloatingPointError, match=r"siglip fwd layer 1: g1 .*pz_gemm"):
            run_loss(m, gi)
    finally:
        e.check_finite = False
        _lib._RECENT[0] = prev
