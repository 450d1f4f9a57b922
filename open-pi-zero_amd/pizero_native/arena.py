"""Flat parameter / gradient arenas for the Pi0 model.

All weights live in ONE contiguous buffer (per dtype/device), laid out in
*backward-completion order*: the action expert region first (decoder, final
norm, joint layers 17..0, encoders), then the VLM region (Gemma layers 17..0,
projector, SigLIP 26..0, patch embed), then frozen tensors (token embedding).
Consequences, all MI355X-first:
  * fused operands are free views: q|k|v rows and gate|up rows are adjacent,
    so one GEMM computes the fused projection and one wgrad GEMM its gradient;
  * the gradient arena mirrors the layout, so DDP buckets are contiguous
    slices that become ready layer by layer during backward (RCCL all-reduce
    overlapped with backward, no bucket copies) and AdamW / grad-norm run as a
    handful of flat launches instead of one per tensor;
  * every parameter starts on a 16-byte boundary (vector loads).
nn.Parameters of the module tree are rebound to views of the arena, so
state_dict()/load_state_dict()/named_parameters() keep the reference keys.
"""

from __future__ import annotations

from dataclasses import dataclass

import torch
from torch import nn

ALIGN = 8  # elements (16 bytes of bf16)


@dataclass
class Slot:
    name: str
    shape: tuple
    offset: int
    numel: int
    region: str


def _round(n, a=ALIGN):
    return (n + a - 1) // a * a


class Arena:
    """Owns the flat buffers; maps reference parameter names to views."""

    def __init__(self, entries, device, dtype):
        # entries: list of (name, shape, region, param-or-None) in layout order
        self.slots: dict[str, Slot] = {}
        self.order: list[str] = []
        self.region_range: dict[str, list[int]] = {}
        off = 0
        for name, shape, region, _ in entries:
            n = 1
            for s in shape:
                n *= int(s)
            self.slots[name] = Slot(name, tuple(int(s) for s in shape), off, n, region)
            self.order.append(name)
            r = self.region_range.setdefault(region, [off, off])
            r[1] = off + n
            off += _round(n)
        self.total = _round(off, 64)
        self.data = torch.zeros(self.total, device=device, dtype=dtype)
        self.grad = None
        for name, _, _, p in entries:
            if p is not None and p.device.type != "meta":
                self.view(name).copy_(p.detach())

    # ------------------------------------------------------------------ views
    def view(self, name, buf=None):
        s = self.slots[name]
        b = self.data if buf is None else buf
        return b[s.offset : s.offset + s.numel].view(s.shape)

    def span(self, first, last, buf=None, rows=None):
        """2-D view over adjacent slots first..last (same trailing dim)."""
        a, z = self.slots[first], self.slots[last]
        b = self.data if buf is None else buf
        cols = a.shape[-1] if len(a.shape) > 1 else 1
        n = z.offset + z.numel - a.offset
        assert n % cols == 0
        for nm in self.order[self.order.index(first) : self.order.index(last)]:
            s = self.slots[nm]
            assert s.numel % cols == 0 and s.numel == _round(s.numel), f"{nm} breaks the span"
        v = b[a.offset : a.offset + n]
        return v.view(n // cols, cols) if len(a.shape) > 1 else v

    def grad_view(self, name):
        return self.view(name, self.ensure_grad())

    def grad_span(self, first, last):
        return self.span(first, last, self.ensure_grad())

    def ensure_grad(self):
        if self.grad is None or self.grad.device != self.data.device or self.grad.dtype != self.data.dtype:
            self.grad = torch.zeros_like(self.data)
        return self.grad

    def region_slice(self, region, buf=None):
        a, z = self.region_range[region]
        b = self.data if buf is None else buf
        return b[a : _round(z)]

    # --------------------------------------------------------------- binding
    def bind(self, params: dict):
        """Rebind nn.Parameters (name -> (module, attr, requires_grad)) to arena views."""
        for name, (mod, attr, rg) in params.items():
            if name not in self.slots:
                continue
            mod._parameters[attr] = nn.Parameter(self.view(name), requires_grad=rg)

    def apply(self, fn):
        self.data = fn(self.data)
        if self.grad is not None:
            self.grad = fn(self.grad)
