"""Per-expert Gemma-layout decoder layers (mixture.py:23-242): parameter containers.

``Mixture`` / ``MixtureDecoderLayer`` / ``MixtureAttention`` keep the
reference attribute names (q/k/v/o_proj, mlp.{gate,up,down}_proj,
input_layernorm, post_attention_layernorm, norm) so state_dict keys match.
The arena lays q|k|v and gate|up out adjacently; the native engine runs each
layer as: RMSNorm -> fused QKV MFMA GEMM -> RoPE/split into the joint token
buffers -> joint attention -> o_proj GEMM (+residual epilogue) -> RMSNorm ->
fused gate|up GEMM with GeGLU epilogue -> down GEMM (+residual epilogue).
adaLN(-Zero) modes are out of scope (adaptive_mode null).
"""

from __future__ import annotations

from torch import nn

from src.model.paligemma.modules import GemmaMLP, GemmaRMSNorm, GemmaRotaryEmbedding
from src.utils.config import cfg_get


class Mixture(nn.Module):
    def __init__(self, config):
        super().__init__()
        if cfg_get(config, "adaptive_mode", None):
            raise NotImplementedError("adaLN / adaLN-Zero action expert is out of scope (SURVEY 2.1)")
        self.layers = nn.ModuleList([MixtureDecoderLayer(config) for _ in range(cfg_get(config, "num_hidden_layers"))])
        self.adaptive_mode = None
        if cfg_get(config, "use_final_norm", False):
            self.norm = GemmaRMSNorm(cfg_get(config, "hidden_size"), eps=float(cfg_get(config, "rms_norm_eps", 1e-6)))

    @property
    def head_dim(self) -> int:
        return self.layers[0].self_attn.head_dim


class MixtureDecoderLayer(nn.Module):
    def __init__(self, config):
        super().__init__()
        self.self_attn = MixtureAttention(config)
        self.mlp = GemmaMLP(config, use_quantize=cfg_get(config, "use_quantize", False),
                            use_lora=cfg_get(config, "use_lora", False))
        self.adaptive_mode = None
        eps = float(cfg_get(config, "rms_norm_eps", 1e-6))
        self.input_layernorm = GemmaRMSNorm(cfg_get(config, "hidden_size"), eps=eps)
        self.post_attention_layernorm = GemmaRMSNorm(cfg_get(config, "hidden_size"), eps=eps)


class MixtureAttention(nn.Module):
    def __init__(self, config):
        super().__init__()
        self.config = config
        self.num_heads = cfg_get(config, "num_attention_heads")
        self.head_dim = cfg_get(config, "head_dim")
        self.num_key_value_heads = cfg_get(config, "num_key_value_heads")
        self.num_key_value_groups = self.num_heads // self.num_key_value_heads
        hid = cfg_get(config, "hidden_size")
        bias = bool(cfg_get(config, "attention_bias", False))
        if bias:
            raise NotImplementedError("attention_bias=True is not used by Pi0 (bridge.yaml:179)")
        self.q_proj = nn.Linear(hid, self.num_heads * self.head_dim, bias=False)
        self.k_proj = nn.Linear(hid, self.num_key_value_heads * self.head_dim, bias=False)
        self.v_proj = nn.Linear(hid, self.num_key_value_heads * self.head_dim, bias=False)
        self.o_proj = nn.Linear(self.num_heads * self.head_dim, hid, bias=False)
        self.rotary_emb = GemmaRotaryEmbedding(self.head_dim, base=cfg_get(config, "rope_theta", 10000.0))
