"""Learning-rate schedule (utils/optim.py:31-159 semantics) and optimizer helpers.

``CosineAnnealingWarmupRestarts``: per cycle, linear warm-up from ``min_lr`` to
the cycle's max over ``warmup_steps`` updates, then half-cosine decay back to
``min_lr`` over the rest of the cycle; cycle c lasts
``warmup + (first_cycle_steps - warmup) * cycle_mult**c`` updates and peaks at
``max_lr * gamma**c``.  The lr is written into every param group of the
wrapped optimizer (pizero_native.optim.FusedAdamW or any torch optimizer);
constructing the scheduler sets ``min_lr`` like the reference (step -1).
"""

from __future__ import annotations

import math

import torch


class CosineAnnealingWarmupRestarts:
    def __init__(self, optimizer, first_cycle_steps: int, cycle_mult: float = 1.0, max_lr: float = 0.1,
                 min_lr: float = 0.001, warmup_steps: int = 0, gamma: float = 1.0, last_epoch: int = -1):
        if warmup_steps >= first_cycle_steps:
            raise ValueError("warmup_steps must be smaller than first_cycle_steps")
        self.optimizer = optimizer
        self.first_cycle_steps = int(first_cycle_steps)
        self.cycle_mult = float(cycle_mult)
        self.base_max_lr = float(max_lr)
        self.min_lr = float(min_lr)
        self.warmup_steps = int(warmup_steps)
        self.gamma = float(gamma)
        self.last_epoch = last_epoch
        self._set(self.lr_at(last_epoch))

    # ------------------------------------------------------------ schedule --
    def _cycle_of(self, step):
        """(cycle index, step within cycle, cycle length) for global update index ``step``."""
        w, L = self.warmup_steps, self.first_cycle_steps
        if step < L:
            return 0, step, L
        if self.cycle_mult == 1.0:
            return step // L, step % L, L
        c, start, length = 0, 0, L
        while step >= start + length:
            start += length
            c += 1
            length = int((length - w) * self.cycle_mult) + w
        return c, step - start, length

    def lr_at(self, step):
        if step < 0:
            return self.min_lr
        c, s, length = self._cycle_of(step)
        peak = self.base_max_lr * self.gamma ** c
        if s < self.warmup_steps:
            return self.min_lr + (peak - self.min_lr) * s / self.warmup_steps
        frac = (s - self.warmup_steps) / max(1, length - self.warmup_steps)
        return self.min_lr + (peak - self.min_lr) * (1 + math.cos(math.pi * frac)) / 2

    def _set(self, lr):
        for g in self.optimizer.param_groups:
            if isinstance(g["lr"], torch.Tensor):
                g["lr"].fill_(lr)
            else:
                g["lr"] = lr

    def step(self, epoch=None):
        self.last_epoch = self.last_epoch + 1 if epoch is None else int(math.floor(epoch))
        self._set(self.lr_at(self.last_epoch))

    def get_last_lr(self):
        return [g["lr"] for g in self.optimizer.param_groups]

    def state_dict(self):
        """The reference's keys (utils/optim.py:56-60 dumps its __dict__ minus the optimizer):
        first_cycle_steps, cycle_mult, base_max_lr, max_lr, min_lr, warmup_steps, gamma,
        cur_cycle_steps, cycle, step_in_cycle, last_epoch, base_lrs."""
        c, s, length = self._cycle_of(self.last_epoch) if self.last_epoch >= 0 else (0, -1, self.first_cycle_steps)
        return {
            "first_cycle_steps": self.first_cycle_steps, "cycle_mult": self.cycle_mult,
            "base_max_lr": self.base_max_lr, "max_lr": self.base_max_lr * self.gamma ** c, "min_lr": self.min_lr,
            "warmup_steps": self.warmup_steps, "gamma": self.gamma, "cur_cycle_steps": length, "cycle": c,
            "step_in_cycle": s, "last_epoch": self.last_epoch,
            "base_lrs": [self.min_lr] * len(self.optimizer.param_groups),
        }

    def load_state_dict(self, state):
        """Restores from this class's or the reference's state_dict (the closed-form schedule needs the
        constants and last_epoch only) and writes the lr of that step into the optimizer."""
        for k in ("first_cycle_steps", "warmup_steps", "last_epoch"):
            if k in state:
                setattr(self, k, int(state[k]))
        for k in ("cycle_mult", "base_max_lr", "min_lr", "gamma"):
            if k in state:
                setattr(self, k, float(state[k]))
        self._set(self.lr_at(self.last_epoch))


def get_num_params_in_billions(optimizer):
    return sum(p.numel() for g in optimizer.param_groups for p in g["params"]) / 1e9


def optimizer_to(optimizer, device):
    for st in optimizer.state.values():
        for k, v in st.items():
            if isinstance(v, torch.Tensor):
                st[k] = v.to(device)
