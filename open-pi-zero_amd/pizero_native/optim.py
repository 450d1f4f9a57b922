"""Fused flat AdamW + gradient-norm clipping over the parameter arena.

Replaces the reference's two bitsandbytes AdamW8bit optimizers and
``torch.nn.utils.clip_grad_norm_`` (train.py:171-198, 371-379).  Parameters
are views of one flat arena, so a param group collapses to a few contiguous
runs: one ``pz_adamw`` launch per run instead of one kernel chain per tensor.
Update rule = torch.optim.AdamW (decoupled weight decay, bias correction);
moments are fp32 (the reference's 8-bit blockwise states are not reproduced:
bitsandbytes is absent here, parity for the optimizer is pinned against
torch.optim.AdamW instead -- SURVEY 8(c)).
"""

from __future__ import annotations

import torch

from . import ops


def contiguous_runs(params):
    """Merge parameters whose storage is adjacent (gaps < 16 B of arena padding)."""
    ps = sorted([p for p in params], key=lambda p: p.data_ptr())
    runs = []
    for p in ps:
        if runs:
            last = runs[-1]
            end = last["ptr"] + last["n"] * p.element_size()
            gap = p.data_ptr() - end
            if 0 <= gap < 16 and p.untyped_storage().data_ptr() == last["base"].untyped_storage().data_ptr():
                last["n"] = (p.data_ptr() - last["ptr"]) // p.element_size() + p.numel()
                last["params"].append(p)
                continue
        runs.append({"ptr": p.data_ptr(), "n": p.numel(), "params": [p], "base": p})
    out = []
    for r in runs:
        b = r["base"]
        st = b.untyped_storage()
        full = torch.empty(0, dtype=b.dtype, device=b.device).set_(st)
        off = (r["ptr"] - st.data_ptr()) // b.element_size()
        out.append((full[off : off + r["n"]], r["params"], off))
    return out


class FusedAdamW(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self._runs = None
        self._gscale = None

    def _prepare(self):
        if self._runs is not None:
            return
        self._runs = []
        for group in self.param_groups:
            runs = []
            for flat, plist, off in contiguous_runs(group["params"]):
                m = torch.zeros(flat.numel(), device=flat.device, dtype=torch.float32)
                v = torch.zeros_like(m)
                runs.append(dict(flat=flat, params=plist, m=m, v=v))
            self._runs.append(runs)

    def _flat_grad(self, run):
        """Gradient run as a flat view (grads are arena views laid out like the params)."""
        p0 = run["params"][0]
        g0 = p0.grad
        if g0 is None:
            return None
        st = g0.untyped_storage()
        full = torch.empty(0, dtype=g0.dtype, device=g0.device).set_(st)
        off = (g0.data_ptr() - st.data_ptr()) // g0.element_size()
        flat = full[off : off + run["flat"].numel()]
        # verify the layout assumption once per run (cheap pointer arithmetic)
        base_p, base_g = run["flat"].data_ptr(), flat.data_ptr()
        for p in run["params"]:
            if p.grad is None or p.grad.data_ptr() - base_g != p.data_ptr() - base_p:
                raise RuntimeError("FusedAdamW: gradients are not arena views; use the native PiZero backward")
        return flat

    def clip_grad_norm_(self, max_norm):
        """clip_grad_norm_ over every param of this optimizer; coefficient applied inside step().
        Returns the total norm as a device tensor (no host sync)."""
        self._prepare()
        dev = self._runs[0][0]["flat"].device
        acc = torch.zeros(1, device=dev, dtype=torch.float32)
        for runs in self._runs:
            for r in runs:
                g = self._flat_grad(r)
                if g is not None:
                    ops.sumsq(g, acc)
        self._gscale = torch.empty(1, device=dev, dtype=torch.float32)
        norm = torch.empty(1, device=dev, dtype=torch.float32)
        ops.clip_coef(acc, self._gscale, norm, max_norm)
        return norm

    def set_grad_scale(self, coef):
        self._gscale = coef

    @torch.no_grad()
    def step(self, closure=None):
        self._prepare()
        for group, runs in zip(self.param_groups, self._runs):
            b1, b2 = group["betas"]
            group["step"] = group.get("step", 0) + 1
            t = group["step"]
            for r in runs:
                g = self._flat_grad(r)
                if g is None:
                    continue
                ops.adamw(r["flat"], g, r["m"], r["v"], group["lr"], b1, b2, group["eps"], group["weight_decay"],
                          1 - b1 ** t, 1 - b2 ** t, self._gscale)
        self._gscale = None

    def zero_grad(self, set_to_none: bool = True):
        for group in self.param_groups:
            for p in group["params"]:
                if set_to_none:
                    p.grad = None
                elif p.grad is not None:
                    p.grad.zero_()


def clip_grad_norm_(optimizers, max_norm):
    """Joint clip over several FusedAdamW optimizers (train.py:371-374 clips the union)."""
    opts = list(optimizers)
    dev = opts[0]._runs[0][0]["flat"].device if opts[0]._runs else None
    acc = None
    for o in opts:
        o._prepare()
        dev = o._runs[0][0]["flat"].device
        if acc is None:
            acc = torch.zeros(1, device=dev, dtype=torch.float32)
        for runs in o._runs:
            for r in runs:
                g = o._flat_grad(r)
                if g is not None:
                    ops.sumsq(g, acc)
    coef = torch.empty(1, device=dev, dtype=torch.float32)
    norm = torch.empty(1, device=dev, dtype=torch.float32)
    ops.clip_coef(acc, coef, norm, max_norm)
    for o in opts:
        o.set_grad_scale(coef)
    return norm
