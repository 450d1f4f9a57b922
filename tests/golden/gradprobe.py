"""Whole-tensor gradient probes shared by the fixture generator and the parity tests.

TEST INFRASTRUCTURE (like oracle/): only tests/ and tests/golden/make_golden*.py use it.

A full-size gradient arena is 2.6 B values, too big to store as a fixture.  Each trained
tensor is summarised instead by
  * its L2 norm (float64);
  * ``sample``: ~4096 values at seeded pseudo-random flat indices plus the tile tails
    (the last row and the last column of a 2-D weight, the last elements of a vector),
    so a wrong output tile anywhere in a [16384, 2048] weight shows up in the sample with
    high probability and the tails of partial tiles are always covered;
  * ``proj``: projections onto 2 seeded Rademacher (+-1) vectors over the WHOLE tensor,
    summed in float64: an error e anywhere moves a projection by ~N(0, |e|^2), so it
    catches wrong values the sample misses.

The index and sign streams are a 32-bit integer hash evaluated with int64 torch ops, so
the CPU reference run and the GPU test regenerate the same streams on either device.
"""

from __future__ import annotations

import zlib

import torch

N_SAMPLE = 4096
N_TAIL = 256
N_PROJ = 2
_MASK = 0xFFFFFFFF


def _hash32(x: torch.Tensor) -> torch.Tensor:
    """x int64 in [0, 2^32) -> int64 in [0, 2^32) (a well-mixed 32-bit hash)."""
    x = ((x ^ (x >> 16)) * 0x45D9F3B) & _MASK
    x = ((x ^ (x >> 16)) * 0x45D9F3B) & _MASK
    return x ^ (x >> 16)


def name_seed(name: str, k: int = 0) -> int:
    return (zlib.crc32(name.encode()) + 0x9E3779B1 * (k + 1)) & _MASK


def _spread(n: int, device) -> torch.Tensor:
    """min(n, N_TAIL) integer positions spread evenly over [0, n) (first and last included)."""
    k = min(n, N_TAIL)
    if k <= 1:
        return torch.zeros(k, device=device, dtype=torch.int64)
    return torch.arange(k, device=device, dtype=torch.int64) * (n - 1) // (k - 1)


def sample_index(name: str, shape, n: int = N_SAMPLE, device="cpu") -> torch.Tensor:
    """Flat int64 indices: n - tails pseudo-random ones, then the tails."""
    numel = 1
    for s in shape:
        numel *= int(s)
    tails = []
    if len(shape) >= 2:
        R, C = int(shape[0]), numel // int(shape[0])
        tails.append((R - 1) * C + _spread(C, device))
        tails.append(_spread(R, device) * C + (C - 1))
    else:
        tails.append(torch.arange(max(0, numel - N_TAIL), numel, device=device))
    tail = torch.cat(tails)
    nr = max(0, n - tail.numel())
    j = torch.arange(nr, device=device, dtype=torch.int64)
    h = _hash32((j * 2654435761 + name_seed(name)) & _MASK)
    h2 = _hash32((h + 0x68E31DA4) & _MASK)
    rnd = (((h >> 2) << 31) | (h2 >> 1)) % numel
    return torch.cat([rnd, tail])


def rademacher(numel: int, seed: int, device, start: int = 0) -> torch.Tensor:
    i = torch.arange(start, start + numel, device=device, dtype=torch.int64)
    h = _hash32((i * 2654435761 + seed) & _MASK)
    return (1 - 2 * ((h >> 7) & 1)).to(torch.float64)


def probe(name: str, g: torch.Tensor, n: int = N_SAMPLE, chunk: int = 1 << 24) -> dict:
    """{norm, sample [n] fp32, proj [N_PROJ] fp64} of a gradient tensor (any device)."""
    flat = g.detach().reshape(-1)
    dev = flat.device
    idx = sample_index(name, tuple(g.shape), n, device=dev)
    sample = flat[idx].double()
    norm = 0.0
    proj = [0.0] * N_PROJ
    for s in range(0, flat.numel(), chunk):
        part = flat[s:s + chunk].double()
        norm += float((part * part).sum())
        for k in range(N_PROJ):
            proj[k] += float((part * rademacher(part.numel(), name_seed(name, k + 1), dev, start=s)).sum())
    return {"norm": norm ** 0.5, "sample": sample.float().cpu(), "proj": torch.tensor(proj, dtype=torch.float64)}


def compare(mine: dict, ref: dict) -> dict:
    """rel-L2 / cosine of the samples, relative norm error, projection errors in units of |g_ref|."""
    a = mine["sample"].double()
    b = ref["sample"].double()
    nb = float(b.norm())
    rel = float((a - b).norm()) / max(nb, 1e-30)
    cos = float((a * b).sum()) / max(float(a.norm()) * nb, 1e-30)
    rn = ref["norm"]
    nrel = abs(mine["norm"] - rn) / max(rn, 1e-30)
    pe = float((mine["proj"] - ref["proj"]).abs().max()) / max(rn, 1e-30)
    return {"rel": rel, "cos": cos, "norm_rel": nrel, "proj_err": pe}
