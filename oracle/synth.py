"""Portable counter-based synthetic data for parity tests (TEST INFRASTRUCTURE).

This module is part of the oracle: only ``tests/``, ``__graft_entry__.smoke()``
and ``bench.py``'s ``cpu_baseline`` leg may import it.  It defines the weights
and inputs every parity fixture is computed on, so that the reference (run in
the build container by ``tests/golden/make_golden.py``), the CPU oracle and the
HIP path all see bit-identical fp32 values without shipping multi-GB tensors.

Generator: splitmix64 over ``seed(name) + index`` -> top 24 bits -> U[-1, 1)
(exact in fp32) -> ``offset + scale * u`` (one fp32 multiply-add, IEEE).
The same arithmetic is implemented on the device by ``pz_fill_uniform`` in
``open-pi-zero_amd/csrc/pz_misc.hip``; a GPU test checks the two agree
bit-for-bit.
"""

from __future__ import annotations

import math

import numpy as np

_GOLDEN = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def fnv1a64(text: str) -> int:
    h = 0xCBF29CE484222325
    for ch in text.encode("utf-8"):
        h ^= ch
        h = (h * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return h


def tensor_seed(name: str, seed: int = 0) -> int:
    return (fnv1a64(name) ^ (seed * 0x9E3779B97F4A7C15)) & 0xFFFFFFFFFFFFFFFF


def uniform_pm1(seed: int, n: int, chunk: int = 1 << 24) -> np.ndarray:
    """n float32 values in [-1, 1): splitmix64(seed + i) >> 40, * 2^-23 - 1."""
    out = np.empty(n, dtype=np.float32)
    s = np.uint64(seed)
    with np.errstate(over="ignore"):
        for start in range(0, n, chunk):
            stop = min(n, start + chunk)
            z = np.arange(start, stop, dtype=np.uint64) + s
            z = z + _GOLDEN
            z = (z ^ (z >> np.uint64(30))) * _M1
            z = (z ^ (z >> np.uint64(27))) * _M2
            z = z ^ (z >> np.uint64(31))
            u24 = (z >> np.uint64(40)).astype(np.float32)
            out[start:stop] = u24 * np.float32(2.0**-23) - np.float32(1.0)
    return out


def synth_tensor(name: str, shape, offset: float, scale: float, seed: int = 0) -> np.ndarray:
    n = int(np.prod(shape)) if len(shape) else 1
    u = uniform_pm1(tensor_seed(name, seed), n)
    v = np.float32(offset) + np.float32(scale) * u
    return v.astype(np.float32).reshape(shape)


def param_rule(name: str, shape) -> tuple[float, float]:
    """(offset, scale) of the synthetic value of one reference parameter.

    Linear weights ~ U(-1/sqrt(fan_in), 1/sqrt(fan_in)); biases +-0.02;
    Gemma RMSNorm weights (used as 1 + w, modules.py:20) +-0.1; LayerNorm
    weights 1 +- 0.1 and biases +-0.02; embeddings +-0.05; position embedding
    +-0.02.  Non-zero norm weights exercise the (1 + w) path.
    """
    if name.endswith("position_embedding.weight"):
        return 0.0, 0.02
    if "embed_tokens" in name:
        return 0.0, 0.05
    if "layer_norm" in name or "post_layernorm" in name:
        return (1.0, 0.1) if name.endswith(".weight") else (0.0, 0.02)
    if "layernorm" in name or name.endswith("norm.weight"):
        return 0.0, 0.1  # Gemma RMSNorm, zero-centred (1 + w)
    if name.endswith(".bias"):
        return 0.0, 0.02
    fan_in = int(np.prod(shape[1:])) if len(shape) > 1 else int(shape[0])
    return 0.0, 1.0 / math.sqrt(fan_in)


def synth_state_dict(shapes: dict, seed: int = 0) -> dict:
    """name -> float32 ndarray for every (name, shape) in ``shapes``."""
    out = {}
    for name, shape in shapes.items():
        off, sc = param_rule(name, shape)
        out[name] = synth_tensor(name, tuple(shape), off, sc, seed)
    return out


def synth_inputs(cfg: dict, bsz: int, seed: int = 0, ragged: bool = False) -> dict:
    """Synthetic batch in the reference's input format.

    input_ids: image tokens, BOS(2), text ids, "\\n"(108), pad(0) up to
    max_seq_len.  ``ragged`` gives sample i a text length that differs per
    sample (exercises the block-mask prefix count).
    """
    P = cfg["max_seq_len"]
    n_img = cfg["num_image_tokens"]
    n_text_max = P - n_img
    vocab = cfg["vocab_size"]
    img_tok = cfg["image_token_index"]
    ids = np.zeros((bsz, P), dtype=np.int64)
    u = uniform_pm1(tensor_seed("input_ids", seed), bsz * P).reshape(bsz, P)
    for b in range(bsz):
        n_text = n_text_max if not ragged else max(3, n_text_max - 2 - 3 * b)
        ids[b, :n_img] = img_tok
        ids[b, n_img] = 2
        body = ((u[b] + 1.0) * 0.5 * (min(vocab, img_tok) - 4)).astype(np.int64) + 3
        ids[b, n_img + 1 : n_img + n_text - 1] = body[: n_text - 2]
        ids[b, n_img + n_text - 1] = 108 if vocab > 108 else 3
    attn = (ids != 0).astype(np.int64)
    H = cfg["image_size"]
    n_images = cfg.get("num_images", 1)
    pix = synth_tensor("pixel_values", (bsz, 3, H, H) if n_images == 1 else (bsz, n_images, 3, H, H), 0.0, 1.0, seed)
    prop = synth_tensor("proprios", (bsz, cfg["cond_steps"], cfg["proprio_dim"]), 0.0, 1.0, seed)
    act = synth_tensor("actions", (bsz, cfg["horizon_steps"], cfg["action_dim"]), 0.0, 1.0, seed)
    # x0 ~ approx N(0,1): sum of 4 uniforms scaled (deterministic, portable)
    shp = (bsz, cfg["horizon_steps"], cfg["action_dim"])
    g = sum(synth_tensor(f"x0_{k}", shp, 0.0, 1.0, seed) for k in range(4))
    x0 = (g * np.float32(math.sqrt(3.0 / 4.0))).astype(np.float32)
    g = sum(synth_tensor(f"noise_{k}", shp, 0.0, 1.0, seed) for k in range(4))
    noise = (g * np.float32(math.sqrt(3.0 / 4.0))).astype(np.float32)
    tu = synth_tensor("t", (bsz,), 0.5, 0.5, seed)  # U[0,1)
    # Beta(1.5,1) inverse CDF: z = u^(1/1.5); t = 0.999 (1 - z)   (train.py:239-247)
    t = (np.float32(0.999) * (1.0 - np.power(tu, 1.0 / 1.5))).astype(np.float32)
    return dict(
        input_ids=ids,
        attention_mask=attn,
        pixel_values=pix,
        proprios=prop,
        actions=act,
        x0=x0,
        noise=noise,
        t=t,
    )
