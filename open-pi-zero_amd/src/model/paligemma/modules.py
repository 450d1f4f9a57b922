"""Gemma building blocks as parameter containers (paligemma/modules.py:7-95).

RMSNorm ``x*rsqrt(mean(x^2)+eps)*(1+w)`` (fp32 inside), rotary embedding
(fp32 cos/sin, half-split) and the GeGLU-tanh MLP are executed by HIP
kernels: pz_rmsnorm_fwd/bwd, pz_rope_table + pz_qkv_rope_split, and the
pz_gemm PZ_EPI_GEGLU epilogue (gate|up fused in one MFMA GEMM).
"""

from __future__ import annotations

import torch
from torch import nn

from src.utils.config import cfg_get


class GemmaRMSNorm(nn.Module):
    def __init__(self, dim: int, eps: float = 1e-6):
        super().__init__()
        self.eps = float(eps)
        self.weight = nn.Parameter(torch.zeros(dim))


class GemmaRotaryEmbedding(nn.Module):
    """No parameters; the native engine builds fp32 cos/sin tables per theta."""

    def __init__(self, dim, base=10000):
        super().__init__()
        self.dim = dim
        self.base = float(base)


class GemmaMLP(nn.Module):
    def __init__(self, config, use_quantize=False, use_lora=False):
        super().__init__()
        if use_quantize or use_lora:
            raise NotImplementedError("QLoRA/LoRA are out of scope (SURVEY 2.1)")
        self.config = config
        self.hidden_size = cfg_get(config, "hidden_size")
        self.intermediate_size = cfg_get(config, "intermediate_size")
        self.gate_proj = nn.Linear(self.hidden_size, self.intermediate_size, bias=False)
        self.up_proj = nn.Linear(self.hidden_size, self.intermediate_size, bias=False)
        self.down_proj = nn.Linear(self.intermediate_size, self.hidden_size, bias=False)
