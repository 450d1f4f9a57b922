"""CPU restatement of bitsandbytes' blockwise 8-bit AdamW (TEST INFRASTRUCTURE: the oracle).

Only tests/ may import this module; it is the checker for pz_adamw8bit (csrc/pz_optim.hip), never
the thing that runs in training.

The reference trains with ``bnb.optim.AdamW8bit`` (src/agent/train.py:171-175, 194-198; pinned
``bitsandbytes==0.45.0`` in pyproject.toml:14).  bitsandbytes is a third-party CUDA library that is
NOT installed here and not vendored in /root/reference, so its kernels cannot be run: this file
restates its published algorithm (Dettmers et al., "8-bit Optimizers via Block-wise Quantization",
ICLR 2022; bitsandbytes ``functional.create_dynamic_map`` and the 2-state blockwise optimizer
kernel) and the GPU kernel is pinned to THIS restatement.  Parity with bitsandbytes itself is
therefore UNPINNED (no golden vector of bnb exists in the reference or here).

Algorithm (per parameter tensor with >= 4096 elements -- smaller tensors keep fp32 state, bnb's
``min_8bit_size``):
  * state1 (m) and state2 (v) are uint8 codes into two 256-entry "dynamic tree" maps
    (signed for m, unsigned for v), with one fp32 absmax per block of 256 consecutive elements;
  * step t: g *= gscale; m = qmap1[c1]*absmax1, v = qmap2[c2]*absmax2 (dequantise);
    m = b1*m + (1-b1)*g; v = b2*v + (1-b2)*g*g;
    p += -lr*sqrt(1-b2^t)/(1-b1^t) * m / (sqrt(v) + eps*sqrt(1-b2^t));  then p *= 1 - lr*wd;
    absmax = max |.| over the block of the NEW m / v; codes = quantise(m/absmax), quantise(v/absmax)
    by the 7-step binary search over the sorted map with midpoint rounding; the m code then keeps
    m's sign (bnb's sign fix: a code whose map entry has the other sign bit moves one step toward m).
All arithmetic is float32 (the kernel's), including the map values (built by bnb's float32 torch
arithmetic).  Still unpinned against bnb itself: its exact kernel launch shape (the block-local
order of the absmax reduction does not change a max) and its handling of non-finite gradients.
"""

from __future__ import annotations

import numpy as np

BLOCK = 256
MIN_8BIT_SIZE = 4096


def create_dynamic_map(signed: bool = True, max_exponent_bits: int = 7, total_bits: int = 8) -> np.ndarray:
    """The 256 sorted float32 values of the dynamic (tree) quantisation map, in bnb's own float32 torch
    arithmetic (functional.create_dynamic_map: torch.linspace(0.1, 1, n) in float32, float32 means, the
    python-float scale multiplied in float32), so each entry equals bnb's saved qmap entry to the bit."""
    import torch

    data = []
    non_sign_bits = total_bits - 1
    additional_items = 2 ** (non_sign_bits - max_exponent_bits) - 1
    for i in range(max_exponent_bits):
        n = int(2 ** (i + non_sign_bits - max_exponent_bits) + 1 if signed
                else 2 ** (i + non_sign_bits - max_exponent_bits + 1) + 1)
        b = torch.linspace(0.1, 1, n)
        means = (b[:-1] + b[1:]) / 2.0
        scale = 10 ** (-(max_exponent_bits - 1) + i)
        data += (scale * means).tolist()
        if signed:
            data += (-scale * means).tolist()
    if additional_items > 0:
        b = torch.linspace(0.1, 1, additional_items + 1)
        means = (b[:-1] + b[1:]) / 2.0
        scale = 10 ** (-(max_exponent_bits - 1) + max_exponent_bits - 1)
        data += (scale * means).tolist()
        if signed:
            data += (-scale * means).tolist()
    data.append(0.0)
    data.append(1.0)
    data += [0.0] * (2 ** total_bits - len(data))
    data.sort()
    return np.asarray(data, dtype=np.float32)


def quantize(x: np.ndarray, qmap: np.ndarray, signed: bool) -> np.ndarray:
    """uint8 codes of float32 x (already divided by the block absmax): the 7-step binary search of
    the bnb kernels from pivot 127 with midpoint rounding between the bracketing entries."""
    x = np.asarray(x, dtype=np.float32)
    pivot = np.full(x.shape, 127, dtype=np.int64)
    upper_p = np.full(x.shape, 255, dtype=np.int64)
    lower_p = np.zeros(x.shape, dtype=np.int64)
    lower = np.full(x.shape, -1.0 if signed else 0.0, dtype=np.float32)
    upper = np.ones(x.shape, dtype=np.float32)
    val = qmap[pivot]
    i = 64
    while i > 0:
        gt = x > val
        lower_p = np.where(gt, pivot, lower_p)
        lower = np.where(gt, val, lower)
        upper_p = np.where(gt, upper_p, pivot)
        upper = np.where(gt, upper, val)
        pivot = np.where(gt, pivot + i, pivot - i)
        val = qmap[pivot]
        i >>= 1
    gt = x > val
    mid_up = (upper + val) * np.float32(0.5)
    mid_lo = (lower + val) * np.float32(0.5)
    code = np.where(gt, np.where(x > mid_up, upper_p, pivot), np.where(x < mid_lo, lower_p, pivot))
    return code.astype(np.uint8)


def bf16_round(x: np.ndarray) -> np.ndarray:
    """float32 -> nearest-even bfloat16 -> float32."""
    u = np.asarray(x, dtype=np.float32).view(np.uint32).astype(np.uint64)
    u = (u + 0x7FFF + ((u >> 16) & 1)) & 0xFFFF0000
    return u.astype(np.uint32).view(np.float32)


def step_8bit(p, g, c1, c2, absmax1, absmax2, qmap1, qmap2, lr, b1, b2, eps, wd, t, gscale=1.0):
    """One AdamW8bit step on one tensor (flat float32 p/g, uint8 codes, fp32 absmax per block).
    Returns (p_bf16_as_f32, c1, c2, absmax1, absmax2)."""
    f = np.float32
    n = p.size
    nb = (n + BLOCK - 1) // BLOCK
    blk = np.arange(n) // BLOCK
    g = g.astype(f) * f(gscale)
    m = qmap1[c1].astype(f) * absmax1[blk].astype(f)
    v = qmap2[c2].astype(f) * absmax2[blk].astype(f)
    m = f(b1) * m + f(1.0 - b1) * g
    v = f(b2) * v + f(1.0 - b2) * (g * g)
    c1f = f(1.0 - b1 ** t)
    c2f = f(np.sqrt(1.0 - b2 ** t))
    step = f(-lr) * c2f / c1f
    pn = p.astype(f) + step * (m / (np.sqrt(v) + f(eps) * c2f))
    if wd > 0:
        pn = pn * f(1.0 - lr * wd)
    pad = nb * BLOCK - n
    am1 = np.abs(np.concatenate([m, np.zeros(pad, f)])).reshape(nb, BLOCK).max(1).astype(f)
    am2 = np.abs(np.concatenate([v, np.zeros(pad, f)])).reshape(nb, BLOCK).max(1).astype(f)
    d1 = np.where(am1[blk] > 0, m / np.where(am1[blk] > 0, am1[blk], 1), 0).astype(f)
    d2 = np.where(am2[blk] > 0, v / np.where(am2[blk] > 0, am2[blk], 1), 0).astype(f)
    return bf16_round(pn), sign_fix(quantize(d1, qmap1, True), m, qmap1), quantize(d2, qmap2, False), am1, am2


def sign_fix(c1: np.ndarray, m: np.ndarray, qmap1: np.ndarray) -> np.ndarray:
    """bnb's blockwise 2-state kernel keeps the sign of the first moment through quantisation: when the
    chosen map entry's sign bit differs from m's (a tiny negative m rounded to the +0 entry), the code
    moves one step toward m's sign (+1 if m > 0, else -1)."""
    c = c1.astype(np.int64)
    flip = np.signbit(qmap1[c]) != np.signbit(np.asarray(m, dtype=np.float32))
    c = np.where(flip, np.where(m > 0, c + 1, c - 1), c)
    return c.astype(np.uint8)


def step_32bit(p, g, m, v, lr, b1, b2, eps, wd, t, gscale=1.0):
    """bnb's 32-bit-state Adam step (tensors below MIN_8BIT_SIZE), same formula."""
    f = np.float32
    g = g.astype(f) * f(gscale)
    m = f(b1) * m + f(1.0 - b1) * g
    v = f(b2) * v + f(1.0 - b2) * (g * g)
    c1f = f(1.0 - b1 ** t)
    c2f = f(np.sqrt(1.0 - b2 ** t))
    pn = p.astype(f) + (f(-lr) * c2f / c1f) * (m / (np.sqrt(v) + f(eps) * c2f))
    if wd > 0:
        pn = pn * f(1.0 - lr * wd)
    return bf16_round(pn), m, v
