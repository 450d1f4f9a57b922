"""Action/time encoders (vla/modules.py:9-53) as parameter containers.

SinusoidalPosEmb -> pz_time_embed.  Default (mode 0): fp32 t and fp32 frequencies
= the reference module in fp32 (the fp32 oracle's semantics).  The reference in a
bf16 model computes it in bf16 (t cast to bf16 at train.py:311, ``arange`` in t.dtype
so odd indices above 256 round, every op rounded): that arithmetic is mode 1, selected
with the config key ``time_embed_bf16_reference: true``.  Measured size of the
difference (reference fp32 vs reference bf16, 1024 wide, tests/golden/time_embed.npz):
max |d| 5.3e-3, mean 2.3-4.6e-4; tests/test_kernels_gpu.py pins both modes.  ActionEncoder -> pz_gemm_small (K=7) +
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
