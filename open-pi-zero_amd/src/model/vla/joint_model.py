"""Mixture-of-transformers joint model (joint_model.py:308-383): parameter container.

``JointModel.mixtures`` is an ``nn.ModuleDict`` {vlm, proprio, action} as in
the reference; ``build_mixture_caches`` returns native static KV caches.  The
18-layer loop with the block-causal joint attention is executed by
``pizero_native.engine`` (see that module for the kernel sequence).
"""

from __future__ import annotations

from torch import nn

from src.model.kv_cache import KVCache
from src.model.vla.mixture import Mixture
from src.utils.config import AttrDict, cfg_get


def _merge(base, over):
    out = AttrDict({k: v for k, v in dict(base).items() if k != "mixture"})
    for k, v in dict(over).items():
        out[k] = v
    return out


class JointModel(nn.Module):
    def __init__(self, config):
        super().__init__()
        self.config = config
        self.num_hidden_layers = cfg_get(config, "num_hidden_layers")
        mix = cfg_get(config, "mixture")
        self.num_mixture = len(mix)
        self.cache_names = [n for n in mix if cfg_get(mix[n], "cache", False)]
        self.mixtures = nn.ModuleDict()
        for name in mix:
            self.mixtures[name] = Mixture(_merge(config, mix[name]))
        self.mixture_names = list(mix.keys())

    def build_mixture_caches(self):
        return {name: KVCache() for name in self.cache_names}

    def forward(self, *args, **kwargs):
        raise RuntimeError("JointModel is executed by the native Pi0 engine through PiZero.forward / infer_action")
