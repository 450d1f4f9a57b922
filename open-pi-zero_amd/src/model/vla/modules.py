"""Action/time encoders (vla/modules.py:9-53) as parameter containers.

SinusoidalPosEmb -> pz_time_embed (fp32 t, fp32 frequencies; the reference's
bf16 ``arange`` rounding above 256 is not reproduced: parity is stated
against the fp32 oracle).  ActionEncoder -> pz_gemm_small (K=7) +
pz_concat_time + MFMA GEMM with SiLU epilogue + MFMA GEMM.
"""

from __future__ import annotations

from torch import nn


class SinusoidalPosEmb(nn.Module):
    def __init__(self, dim: int, max_period: float = 10000.0):
        super().__init__()
        self.half_dim = dim // 2
        self.max_period = float(max_period)


class ActionEncoder(nn.Module):
    def __init__(self, action_dim: int, width: int, time_cond: bool = False):
        super().__init__()
        if not time_cond:
            raise NotImplementedError("time_cond=False (adaLN action expert) is out of scope (SURVEY 2.1)")
        self.linear_1 = nn.Linear(action_dim, width)
        self.linear_2 = nn.Linear(2 * width, width)
        self.nonlinearity = nn.SiLU()
        self.linear_3 = nn.Linear(width, width)
        self.time_cond = time_cond
