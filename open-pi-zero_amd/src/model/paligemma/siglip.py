"""SigLIP-So400m/14 vision tower + PaliGemma projector: parameter containers.

Same class names, constructor signatures and parameter names as the
reference (src/model/paligemma/siglip.py:9-320) so hydra-style ``_target_``
configs resolve and checkpoints load with strict=True.  The computation is
not done by these modules: the owning ``PiZero`` packs every weight into its
flat arena and runs the tower with HIP kernels (pizero_native.engine:
patchify + MFMA patch GEMM, 27x [LayerNorm, fused QKV GEMM, fused head_dim-72
attention (flash_fwd_res_kernel<72>: LDS-resident keys, no [B, 16, 256, 256] tensor),
out-proj+residual GEMM, LayerNorm, fc1+GELU GEMM, fc2+residual GEMM], post-LN,
projector GEMM).  Modules are created on the meta
device and materialised by the arena.
"""

from __future__ import annotations

from torch import nn

from src.utils.config import cfg_get


def _native_only(name):
    raise RuntimeError(
        f"{name}.forward is executed by the native Pi0 engine; call PiZero.forward / "
        "PiZero.infer_action instead")


class PaliGemmaMultiModalProjector(nn.Module):
    """siglip.py:9-31: Linear(vision hidden -> projection_dim) with bias."""

    def __init__(self, config, use_quantize: bool = False, use_lora: bool = False):
        super().__init__()
        if use_quantize or use_lora:
            raise NotImplementedError("QLoRA/LoRA are out of scope (SURVEY 2.1: lora/quantize False)")
        self.linear = nn.Linear(cfg_get(config, "vision_config.hidden_size"),
                                cfg_get(config, "vision_config.projection_dim"), bias=True)

    def forward(self, image_features):
        _native_only("PaliGemmaMultiModalProjector")


class SiglipVisionEmbeddings(nn.Module):
    """siglip.py:34-78: Conv2d(3, H, k=s=patch) + learned position embedding."""

    def __init__(self, config):
        super().__init__()
        self.config = config
        self.embed_dim = cfg_get(config, "hidden_size")
        self.image_size = cfg_get(config, "image_size")
        self.patch_size = cfg_get(config, "patch_size")
        self.patch_embedding = nn.Conv2d(cfg_get(config, "num_channels", 3), self.embed_dim,
                                         kernel_size=self.patch_size, stride=self.patch_size, padding="valid")
        self.num_patches = (self.image_size // self.patch_size) ** 2
        self.num_positions = self.num_patches
        self.position_embedding = nn.Embedding(self.num_positions, self.embed_dim)

    def forward(self, pixel_values):
        _native_only("SiglipVisionEmbeddings")


class SiglipAttention(nn.Module):
    """siglip.py:81-166: 16 heads x 72, q/k/v/out Linear with bias, no mask."""

    def __init__(self, config, use_quantize: bool = False, use_lora: bool = False):
        super().__init__()
        self.config = config
        self.embed_dim = cfg_get(config, "hidden_size")
        self.num_heads = cfg_get(config, "num_attention_heads")
        self.head_dim = self.embed_dim // self.num_heads
        self.scale = self.head_dim ** -0.5
        self.dropout = cfg_get(config, "attention_dropout", 0.0)
        # registration order of the reference (k, v, q, out) keeps state_dict order identical
        self.k_proj = nn.Linear(self.embed_dim, self.embed_dim)
        self.v_proj = nn.Linear(self.embed_dim, self.embed_dim)
        self.q_proj = nn.Linear(self.embed_dim, self.embed_dim)
        self.out_proj = nn.Linear(self.embed_dim, self.embed_dim)

    def forward(self, hidden_states):
        _native_only("SiglipAttention")


class SiglipMLP(nn.Module):
    """siglip.py:169-194: fc1 -> gelu(tanh) -> fc2."""

    def __init__(self, config, use_quantize: bool = False, use_lora: bool = False):
        super().__init__()
        self.config = config
        self.fc1 = nn.Linear(cfg_get(config, "hidden_size"), cfg_get(config, "intermediate_size"))
        self.fc2 = nn.Linear(cfg_get(config, "intermediate_size"), cfg_get(config, "hidden_size"))

    def forward(self, hidden_states):
        _native_only("SiglipMLP")


class SiglipEncoderLayer(nn.Module):
    """siglip.py:197-238: pre-LN residual block."""

    def __init__(self, config, use_quantize: bool = False, use_lora: bool = False):
        super().__init__()
        self.embed_dim = cfg_get(config, "hidden_size")
        eps = float(cfg_get(config, "layer_norm_eps", 1e-6))
        self.self_attn = SiglipAttention(config)
        self.layer_norm1 = nn.LayerNorm(self.embed_dim, eps=eps)
        self.mlp = SiglipMLP(config)
        self.layer_norm2 = nn.LayerNorm(self.embed_dim, eps=eps)

    def forward(self, hidden_states):
        _native_only("SiglipEncoderLayer")


class SiglipEncoder(nn.Module):
    def __init__(self, config, use_quantize: bool = False, use_lora: bool = False):
        super().__init__()
        self.config = config
        self.layers = nn.ModuleList([SiglipEncoderLayer(config) for _ in range(cfg_get(config, "num_hidden_layers"))])

    def forward(self, inputs_embeds):
        _native_only("SiglipEncoder")


class SiglipVisionTransformer(nn.Module):
    def __init__(self, config, use_quantize: bool = False, use_lora: bool = False):
        super().__init__()
        self.config = config
        self.embeddings = SiglipVisionEmbeddings(config)
        self.encoder = SiglipEncoder(config)
        self.post_layernorm = nn.LayerNorm(cfg_get(config, "hidden_size"),
                                           eps=float(cfg_get(config, "layer_norm_eps", 1e-6)))

    def forward(self, pixel_values):
        _native_only("SiglipVisionTransformer")


class SiglipVisionModel(nn.Module):
    """siglip.py:303-320."""

    def __init__(self, config, use_quantize: bool = False, use_lora: bool = False):
        super().__init__()
        if use_quantize or use_lora:
            raise NotImplementedError("QLoRA/LoRA are out of scope (SURVEY 2.1: lora/quantize False)")
        self.config = config
        self.vision_model = SiglipVisionTransformer(config)

    def forward(self, pixel_values):
        _native_only("SiglipVisionModel")
