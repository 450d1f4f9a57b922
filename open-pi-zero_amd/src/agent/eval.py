"""EvalAgent: the reference's inference call site (eval.py:21-189) on the native path.

Construction mirrors the reference: ``PiZeroInference(cfg)``, checkpoint load
(``_orig_mod.`` stripped, strict=True), ``freeze_all_weights``, dtype/device
moves.  The action chunk for one observation is ``infer_chunk`` (mask/position
building + ``model(**inputs)`` = PiZeroInference.forward, eval.py:99-125); with
``use_graph`` the whole chunk replays as one hipGraph (pizero_native/graph.py).
The SimplerEnv rollout loop and env adapters are out of scope:
``run()`` needs ``simpler_env`` and raises without it.
"""

from __future__ import annotations

import torch

from src.utils.config import cfg_get


class EvalAgent:
    def __init__(self, cfg, use_graph: bool = True):
        from src.model.vla.pizero import PiZeroInference

        self.cfg = cfg
        self.device = torch.device(f"cuda:{cfg_get(cfg, 'gpu_id', 0)}")
        self.dtype = torch.bfloat16 if cfg_get(cfg, "use_bf16", True) else torch.float32
        self.model = PiZeroInference(cfg, use_ddp=False, device=self.device, dtype=torch.bfloat16, init="none")
        if cfg_get(cfg, "checkpoint_path"):
            self.load_checkpoint(cfg_get(cfg, "checkpoint_path"))
        self.model.tie_action_proprio_weights()
        self.model.freeze_all_weights()
        self.model.eval()
        self.use_graph = use_graph
        self._graphs = {}
        self.act_steps = cfg_get(cfg, "act_steps", cfg_get(cfg, "horizon_steps"))

    def load_checkpoint(self, path):
        data = torch.load(path, weights_only=True, map_location="cpu")
        sd = {k.replace("_orig_mod.", ""): v for k, v in data["model"].items()}
        self.model.load_state_dict(sd, strict=True)

    @torch.no_grad()
    def infer_chunk(self, input_ids, attention_mask, pixel_values, proprios, noise=None):
        """Tokenized observation -> [B, horizon, action_dim] normalised actions (eval.py:99-125)."""
        m = self.model
        dev = self.device
        # masks are built on the device once per call: the block pattern built from the attention mask is
        # known (its prefix counts are remembered), so no per-call validation or host sync follows
        mask, vpos, ppos, apos = m.build_causal_mask_and_position_ids(attention_mask.to(dev), self.dtype)
        itp, amask = m.split_full_mask_into_submasks(mask)
        B = input_ids.shape[0]
        if noise is None:
            noise = torch.randn(B, m.horizon_steps, m.action_dim, device=dev)
        if not self.use_graph:
            return m(input_ids.to(dev), pixel_values.to(dev, self.dtype), itp, amask, vpos, ppos, apos,
                     proprios.to(dev, self.dtype), noise=noise)
        from pizero_native.graph import InferenceGraph

        cnt = m.block_prefix_counts(itp, amask)
        args = (input_ids.to(dev), pixel_values.to(dev, torch.bfloat16), cnt, vpos, ppos, apos,
                proprios.to(dev, torch.float32), noise)
        g = self._graphs.get(B)
        if g is None:
            g = self._graphs[B] = InferenceGraph(m, B)
            g.load(*args)
            g.capture()
        g.load(*args)
        return g.replay().to(self.dtype)

    def run(self):
        try:
            import simpler_env  # noqa: F401
        except ImportError as e:
            raise RuntimeError("SimplerEnv rollouts need simpler_env (not installed; out of scope, SURVEY 2.1)") from e
        raise NotImplementedError("SimplerEnv adapters are out of scope this round (SURVEY 2.1)")
