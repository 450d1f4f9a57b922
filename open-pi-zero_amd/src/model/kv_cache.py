"""KV cache (kv_cache.py:6-46), MI355X layout.

The reference keeps Python lists of per-layer tensors and ``torch.cat``s on
every append, which allocates and blocks graph capture.  Here a cache is one
static device buffer per layer pair, ``[layers, B, L_pad, kv_heads*head_dim]``
for K and V, holding post-RoPE keys; the vlm + proprio prefix is written once
by the prefill and the action rows [P+C, P+C+H) are rewritten in place by
every denoise step ("append_non_active" mode, joint_model.py:6-11).  The
list-style API of the reference is kept for inspection.
"""

from __future__ import annotations

from typing import Optional

import torch


class KVCache:
    def __init__(self) -> None:
        self.k: Optional[torch.Tensor] = None  # [layers, B, Lp, D]
        self.v: Optional[torch.Tensor] = None
        self.length = 0  # valid tokens

    def allocate(self, layers, bsz, lpad, width, device, dtype=torch.bfloat16):
        shp = (layers, bsz, lpad, width)
        if self.k is None or tuple(self.k.shape) != shp or self.k.device != torch.device(device):
            self.k = torch.zeros(shp, device=device, dtype=dtype)
            self.v = torch.zeros(shp, device=device, dtype=dtype)
        self.length = 0
        return self

    def has_item(self, layer_idx) -> bool:
        return self.k is not None and self.length > 0 and layer_idx < self.k.shape[0]

    def num_items(self) -> int:
        return self.length

    def get(self, layer_idx):
        """[B, kv_heads=1, length, head_dim] views like the reference layout."""
        return (self.k[layer_idx, :, None, : self.length], self.v[layer_idx, :, None, : self.length])
