"""PiZero (Pi0 VLA) with the reference's nn.Module surface, executed natively on MI355X.

Drop-in for src/model/vla/pizero.py of shroglck/open-pi-zero:
  * same constructor ``PiZero(cfg, use_ddp=False)`` and ``PiZeroInference``;
  * same kwargs for ``forward`` (flow-matching loss, pizero.py:607-661),
    ``infer_action`` (KV-cached prefill + Euler denoising, pizero.py:416-490),
    ``infer_action_naive`` (pizero.py:492-557), mask/position builders
    (pizero.py:271-336), parameter groups / freezing / tying
    (pizero.py:114-264), ``load_pretrained_weights`` (pizero.py:160-222);
  * same state_dict keys (checkpoints load with strict=True).
Differences (all documented in DESIGN.md):
  * all weights live in one flat arena (pizero_native/arena.py) and every
    kernel of the path is a HIP kernel from libpizero_hip.so, launched by
    pizero_native/engine.py; ``loss.backward()`` runs the native backward and
    writes .grad views of the flat gradient arena;
  * RNG: ``noise=`` may be passed explicitly (parity tests); otherwise noise
    is drawn with torch.randn on the device like the reference;
  * ``torch.compile`` is unnecessary: wrapping is harmless but the native
    path is what runs.
"""

from __future__ import annotations

import logging
import math
from typing import Optional, Tuple

import torch
from torch import nn

from src.model.kv_cache import KVCache
from src.model.vla.modules import ActionEncoder, SinusoidalPosEmb
from src.utils.config import cfg_get, instantiate
from src.utils.decorator import NoSyncBase

log = logging.getLogger(__name__)


def _resolve(root, dotted):
    mod = root
    parts = dotted.split(".")
    for p in parts[:-1]:
        mod = mod[p] if isinstance(mod, (nn.ModuleDict,)) else (mod[int(p)] if isinstance(mod, nn.ModuleList) else getattr(mod, p))
    return mod, parts[-1]


class _PiZeroLoss(torch.autograd.Function):
    """Whole-model autograd node: native forward, native backward into the grad arena."""

    @staticmethod
    def forward(ctx, anchor, model, batch):
        save = {}
        loss = model._engine().train_forward(save=save, **batch)
        ctx.model = model
        ctx.save = save
        return loss.view(())

    @staticmethod
    def backward(ctx, gloss):
        model = ctx.model
        beta = model._grads_live()
        gscale = gloss.reshape(1).to(torch.float32).contiguous()
        model._engine().train_backward(ctx.save, gscale, beta)
        ctx.save = None
        model._attach_grads()
        return None, None, None


class PiZero(nn.Module, NoSyncBase):
    def __init__(self, cfg, use_ddp: bool = False, *, device=None, dtype=None, init: str = "default"):
        super().__init__()
        self.cfg = cfg
        self.use_ddp = use_ddp
        self.vocab_size = cfg_get(cfg, "vocab_size")
        self.pad_token_id = cfg_get(cfg, "pad_token_id")
        self.image_token_index = cfg_get(cfg, "image_token_index")
        self.use_lm_head = cfg_get(cfg, "use_lm_head", False)
        self.max_image_text_tokens = cfg_get(cfg, "max_image_text_tokens", cfg_get(cfg, "max_seq_len"))
        self.num_proprio_tokens = cfg_get(cfg, "cond_steps")
        self.num_action_tokens = cfg_get(cfg, "horizon_steps")
        self.total_num_tokens = self.max_image_text_tokens + self.num_proprio_tokens + self.num_action_tokens
        self.image_text_hidden_size = cfg_get(cfg, "mixture.vlm.hidden_size")
        self.proprio_hidden_size = cfg_get(cfg, "mixture.proprio.hidden_size")
        self.action_hidden_size = cfg_get(cfg, "mixture.action.hidden_size")
        self.num_inference_steps = cfg_get(cfg, "num_inference_steps")
        self.horizon_steps = cfg_get(cfg, "horizon_steps")
        self.action_dim = cfg_get(cfg, "action_dim")
        self.proprio_dim = cfg_get(cfg, "proprio_dim")
        self.final_action_clip_value = cfg_get(cfg, "final_action_clip_value", None)
        self.flow_sig_min = cfg_get(cfg, "flow_sig_min", 0.001)
        self.action_expert_adaptive_mode = cfg_get(cfg, "action_expert_adaptive_mode", None)
        if self.action_expert_adaptive_mode:
            raise NotImplementedError("adaLN action expert is out of scope (SURVEY 2.1)")
        with torch.device("meta"):
            self.embed_tokens = nn.Embedding(self.vocab_size, self.image_text_hidden_size, self.pad_token_id)
            self.vision_tower = instantiate(cfg_get(cfg, "vision"))
            self.multi_modal_projector = instantiate(cfg_get(cfg, "vision_projector"))
            self.joint_model = instantiate(cfg_get(cfg, "joint"))
            self.action_encoder = ActionEncoder(self.action_dim, self.action_hidden_size, time_cond=True)
            self.time_embedding = SinusoidalPosEmb(self.action_hidden_size, cfg_get(cfg, "time_max_period"))
            self.proprio_encoder = nn.Linear(self.proprio_dim, self.proprio_hidden_size)
            self.action_decoder = nn.Linear(self.action_hidden_size, self.action_dim)
            if self.use_lm_head:  # optional text output (pizero.py:106-112), tied to embed_tokens
                self.lm_head = nn.Linear(self.image_text_hidden_size, self.vocab_size, bias=False)
        self._tied = False
        self._eng = None
        self._kv = None
        self._build_arena(torch.device(device or "cpu"), dtype or torch.float32, init=init)

    # ================================================================ arena ==
    def _layout(self):
        """(name, region) in backward-completion order (see pizero_native/arena.py)."""
        nL = self.joint_model.num_hidden_layers
        vL = len(self.vision_tower.vision_model.encoder.layers)
        mp = "joint_model.mixtures."
        out = []

        def gemma(mix, l, region):
            p = f"{mp}{mix}.layers.{l}."
            for n in ("mlp.down_proj.weight", "mlp.gate_proj.weight", "mlp.up_proj.weight",
                      "post_attention_layernorm.weight", "self_attn.o_proj.weight", "self_attn.q_proj.weight",
                      "self_attn.k_proj.weight", "self_attn.v_proj.weight", "input_layernorm.weight"):
                out.append((p + n, region))

        out += [("action_decoder.weight", "action"), ("action_decoder.bias", "action"),
                (mp + "action.norm.weight", "action")]
        if not self._tied:
            out.append((mp + "proprio.norm.weight", "action"))
        for l in reversed(range(nL)):
            gemma("action", l, "action")
            if not self._tied:
                gemma("proprio", l, "action")
        for n in ("action_encoder.linear_3", "action_encoder.linear_2", "action_encoder.linear_1", "proprio_encoder"):
            out += [(n + ".weight", "action"), (n + ".bias", "action")]
        if hasattr(self.joint_model.mixtures["vlm"], "norm"):  # use_final_norm (text generation config)
            out.append((mp + "vlm.norm.weight", "vlm"))
        for l in reversed(range(nL)):
            gemma("vlm", l, "vlm")
        out += [("multi_modal_projector.linear.weight", "vlm"), ("multi_modal_projector.linear.bias", "vlm")]
        vt = "vision_tower.vision_model."
        out += [(vt + "post_layernorm.weight", "vlm"), (vt + "post_layernorm.bias", "vlm")]
        for i in reversed(range(vL)):
            p = f"{vt}encoder.layers.{i}."
            for n in ("mlp.fc2.weight", "mlp.fc2.bias", "mlp.fc1.weight", "mlp.fc1.bias", "layer_norm2.weight",
                      "layer_norm2.bias", "self_attn.out_proj.weight", "self_attn.out_proj.bias",
                      "self_attn.q_proj.weight", "self_attn.k_proj.weight", "self_attn.v_proj.weight",
                      "self_attn.q_proj.bias", "self_attn.k_proj.bias", "self_attn.v_proj.bias",
                      "layer_norm1.weight", "layer_norm1.bias"):
                out.append((p + n, "vlm"))
        out += [(vt + "embeddings.position_embedding.weight", "vlm"),
                (vt + "embeddings.patch_embedding.weight", "vlm"), (vt + "embeddings.patch_embedding.bias", "vlm")]
        out += [("embed_tokens.weight", "frozen")]
        return out

    def _build_arena(self, device, dtype, init="keep"):
        from pizero_native.arena import Arena

        entries, binds = [], {}
        for name, region in self._layout():
            mod, attr = _resolve(self, name)
            p = mod._parameters[attr]
            entries.append((name, tuple(p.shape), region, p))
            binds[name] = (mod, attr, p.requires_grad)
        self._arena = Arena(entries, device, dtype)
        self._arena.bind(binds)
        self._tie_lm_head()
        self._pmap = {name: _resolve(self, name) for name, _ in self._layout()}
        if init == "default":
            self._init_weights()
        self._eng = None

    @torch.no_grad()
    def _init_weights(self):
        """Default init: U(+-1/sqrt(fan_in)) for Linear/Conv, N(0,1)->U for embeddings,
        LayerNorm (1, 0), Gemma RMSNorm 0 (modules.py:11)."""
        import zlib

        g = torch.Generator(device="cpu").manual_seed(0)
        for name in self._arena.order:
            v = self._arena.view(name)
            if "layer_norm" in name or "post_layernorm" in name:
                v.fill_(1.0 if name.endswith("weight") else 0.0)
                continue
            if name.endswith("norm.weight") or "layernorm" in name:
                v.zero_()
                continue
            if name in ("embed_tokens.weight", "vision_tower.vision_model.embeddings.position_embedding.weight"):
                bound = 1.0
            else:
                owner = name.rsplit(".", 1)[0] + ".weight" if name.endswith(".bias") else name
                w = self._arena.view(owner)
                bound = 1.0 / math.sqrt(max(1, w[0].numel() if w.dim() > 1 else w.numel()))
            if v.device.type == "cuda":
                from pizero_native import ops

                ops.fill_uniform(v, zlib.crc32(name.encode()), 0.0, bound)
            else:
                v.copy_(torch.empty(v.shape, dtype=torch.float32).uniform_(-bound, bound, generator=g))

    def _apply(self, fn, recurse=True):
        """.to(device/dtype) converts the whole arena at once and rebinds the views."""
        if getattr(self, "_arena", None) is None:
            return super()._apply(fn, recurse)
        rg = {n: self._pmap[n][0]._parameters[self._pmap[n][1]].requires_grad for n in self._pmap}
        self._arena.apply(fn)
        self._arena.bind({n: (m, a, rg[n]) for n, (m, a) in self._pmap.items()})
        self._tie_lm_head()
        self._eng = None
        self._kv = None
        return self

    def _tie_lm_head(self):
        """pizero.py:112: lm_head.weight IS embed_tokens.weight (one arena tensor, two state_dict keys)"""
        if getattr(self, "use_lm_head", False) and hasattr(self, "lm_head"):
            self.lm_head._parameters["weight"] = self.embed_tokens._parameters["weight"]

    def _param(self, name):
        m, a = self._pmap[name]
        return m._parameters[a]

    def _requires_grad(self, name):
        return self._param(name).requires_grad

    def _vlm_needs_grad(self):
        a, z = self._arena.region_range["vlm"]
        return any(self._param(n).requires_grad for n in self._arena.order if self._arena.slots[n].region == "vlm")

    def _trainable_names(self):
        return [n for n in self._arena.order if self._param(n).requires_grad]

    def _grads_live(self):
        g = self._arena.grad
        for n in self._trainable_names():
            p = self._param(n)
            if p.grad is not None and g is not None and p.grad.data_ptr() == self._arena.view(n, g).data_ptr():
                return True
        return False

    def _attach_grads(self):
        g = self._arena.ensure_grad()
        for n in self._trainable_names():
            p = self._param(n)
            v = self._arena.view(n, g)
            if p.grad is None or p.grad.data_ptr() != v.data_ptr():
                p.grad = v

    def _engine(self):
        if self._eng is None:
            from pizero_native.engine import Engine

            if self._arena.data.device.type != "cuda":
                raise RuntimeError("PiZero runs on the MI355X HIP path only: move the model to a GPU (.to('cuda'))")
            self._eng = Engine(self)
            if getattr(self, "_fp8_infer", False):
                self._eng.prepare_fp8()
        return self._eng

    def use_fp8_inference(self, enabled: bool = True):
        """Config C5 (BASELINE.json configs[4], "fp8 MFMA attention/MLP"): run inference (infer_action,
        infer_text) with OCP e4m3 weights -- per-tensor scales -- for every Linear of SigLIP, the vlm
        mixture and the action expert: prefill MLP GEMMs W8A8 on the fp8 MFMA (per-row activation scales),
        prefill q|k|v / o projections and denoise rows W8A16.  Training never uses them.  The codes are a snapshot of the current weights:
        call again after the weights change.  An extension: the reference has no fp8 path."""
        self._fp8_infer = bool(enabled)
        eng = self._engine()
        if enabled:
            eng.prepare_fp8()
        else:
            eng.f8 = None
        return self

    # ========================================================= param groups ==
    @property
    def action_expert_parameters(self):
        return (list(self.action_encoder.parameters()) + list(self.action_decoder.parameters())
                + list(self.proprio_encoder.parameters()) + list(self.joint_model.mixtures["action"].parameters()))

    @property
    def trainable_vlm_parameters(self):
        return (list(self.vision_tower.parameters()) + list(self.multi_modal_projector.parameters())
                + self.trainable_gemma_parameters)

    @property
    def lora_trainable_vlm_parameters(self):
        return []  # LoRA out of scope (lora: False)

    @property
    def trainable_gemma_parameters(self):
        return [p for n, p in self.joint_model.mixtures["vlm"].named_parameters()
                if not self._check_gemma_unused_parameter_by_name(n)]

    def _check_gemma_unused_parameter_by_name(self, name: str) -> bool:
        last = self.joint_model.num_hidden_layers - 1
        return (f"{last}.post" in name or f"{last}.mlp" in name or f"{last}.self_attn.o_proj" in name
                or f"{last}.self_attn.v_proj" in name)

    def load_pretrained_weights(self):
        """pizero.py:160-222: PaliGemma safetensors -> embed / vision / projector / Gemma."""
        import glob
        import os

        from safetensors import safe_open

        files = glob.glob(os.path.join(cfg_get(self.cfg, "pretrained_model_path"), "*.safetensors"))
        if not files:
            raise FileNotFoundError(f"no *.safetensors under {cfg_get(self.cfg, 'pretrained_model_path')}")
        sd = {}
        for f in files:
            with safe_open(f, framework="pt", device="cpu") as h:
                for k in h.keys():
                    t = h.get_tensor(k)
                    if "embed_tokens" in k:
                        sd[k.replace("language_model.model.embed_tokens.", "embed_tokens.")] = t
                    elif "vision_tower" in k:
                        sd[k] = t
                    elif "multi_modal_projector" in k:
                        sd[k] = t
                    elif "language_model.model" in k:
                        sd[k.replace("language_model.model.", "joint_model.mixtures.vlm.")] = t
        missing, _ = self.load_state_dict(sd, strict=False)
        log.info("Loaded pre-trained PaliGemma weights (%d tensors, %d keys not in checkpoint)", len(sd), len(missing))

    def freeze_non_lora_weights_in_vlm(self):
        raise NotImplementedError("LoRA is out of scope (SURVEY 2.1)")

    def freeze_unused_weights(self):
        self.embed_tokens.weight.requires_grad = False
        for name, param in self.joint_model.mixtures["vlm"].named_parameters():
            if self._check_gemma_unused_parameter_by_name(name):
                param.requires_grad = False

    def freeze_all_weights(self):
        for _, p in self.named_parameters():
            p.requires_grad = False

    def tie_action_proprio_weights(self):
        """pizero.py:262-264; the arena is repacked without the proprio copy."""
        self.joint_model.mixtures["proprio"] = self.joint_model.mixtures["action"]
        self._tied = True
        self._build_arena(self._arena.data.device, self._arena.data.dtype, init="keep")

    def build_text_cache(self):
        return KVCache()

    # ===================================================== input preparation ==
    def build_causal_mask_and_position_ids(self, attention_mask: torch.Tensor, dtype: torch.dtype):
        """pizero.py:271-324 (vectorised; same values)."""
        bsz = attention_mask.size(0)
        P, C, H = self.max_image_text_tokens, self.num_proprio_tokens, self.num_action_tokens
        L = self.total_num_tokens
        dev = attention_mask.device
        cnt = attention_mask.sum(1)
        i = torch.arange(L, device=dev)
        c = cnt[:, None, None]
        ii, jj = i[None, :, None], i[None, None, :]
        vlm = (ii < c) & (jj < c) & (ii < P)
        prefix = (ii >= P) & (jj < c)
        prop = (ii >= P) & (ii < P + C) & (jj >= P) & (jj < P + C)
        act = (ii >= P + C) & (jj >= P)
        allowed = vlm | prefix | prop | act
        mask = torch.where(allowed, torch.zeros((), dtype=dtype, device=dev),
                           torch.full((), torch.finfo(dtype).min, dtype=dtype, device=dev)).unsqueeze(1)
        vpos = torch.arange(1, P + 1, device=dev).repeat(bsz, 1)
        ppos = torch.arange(1, C + 1, device=dev).repeat(bsz, 1)
        apos = torch.arange(C + 1, C + H + 1, device=dev).repeat(bsz, 1)
        # built here from cnt: known block pattern (finfo.min absorbs), so forward() skips validation
        if torch.finfo(dtype).min <= -1e30:
            self._mask_remember([mask], cnt.to(torch.int32).contiguous())
        return mask, vpos, ppos, apos

    def split_full_mask_into_submasks(self, causal_mask):
        """pizero.py:326-336 (views); a validated full mask passes its prefix counts on to the pair."""
        n = self.max_image_text_tokens + self.num_proprio_tokens
        itp, am = causal_mask[..., :n, :n], causal_mask[..., -self.num_action_tokens:, :]
        spec = self._mask_lookup([causal_mask])
        if spec is not None:
            self._mask_remember([itp, am], spec)
        return itp, am

    def _prefix_counts(self, mask):
        """Per-sample image+text token count from the proprio row of the block mask."""
        P = self.max_image_text_tokens
        return (mask[:, 0, P, :P] == 0).sum(-1).to(torch.int32).contiguous()

    def _block_allowed(self, cnt, rows, ncols):
        """[B, len(rows), ncols] bool: the Pi0 block pattern of pizero.py:271-306 for prefix counts cnt."""
        P, C = self.max_image_text_tokens, self.num_proprio_tokens
        i = rows.view(1, -1, 1)
        j = torch.arange(ncols, device=cnt.device).view(1, 1, -1)
        c = cnt.view(-1, 1, 1).to(torch.int64)
        return torch.where(i < P, (i < c) & (j < c),
                           torch.where(i < P + C, (j < c) | ((j >= P) & (j < P + C)), (j < c) | (j >= P)))

    @staticmethod
    def _is_block(mask, allowed):
        """mask == 0 where allowed and <= -1e30 elsewhere (finfo.min of bf16/fp32, which absorbs any
        logit exactly like the block kernels' 'excluded' -- a fully masked row is then uniform)."""
        m = mask[:, 0]
        return bool(torch.where(allowed, m == 0, m <= -1e30).all())

    def _mask_spec(self, masks, rows_list):
        """Validate the caller's additive mask(s) once per new tensor: the Pi0 block
        pattern -> int32 per-sample prefix counts (the fused kernels regenerate the mask from them);
        anything else -> engine.GeneralMask (the GEMM+softmax path adds it like joint_model.py:271).
        The cache holds the mask tensors themselves (identity + version), so a freed-and-reused address
        can never alias a stale entry."""
        from pizero_native.engine import GeneralMask

        hit = self._mask_lookup(masks)
        if hit is not None:
            return hit
        itp = masks[0]
        P = self.max_image_text_tokens
        cnt = self._prefix_counts(itp) if itp.shape[2] > P else None
        ok = cnt is not None
        if ok:
            for m, rows in zip(masks, rows_list):
                if not self._is_block(m, self._block_allowed(cnt, rows, m.shape[-1])):
                    ok = False
                    break
        if ok:
            spec = cnt
        else:
            f = [m[:, 0].to(torch.float32).contiguous() for m in masks]
            spec = GeneralMask(full=f[0]) if len(f) == 1 else GeneralMask(itp=f[0], act=f[1])
            log.warning("attention mask is not the Pi0 block pattern: using the general additive-mask path")
        self._mask_remember(masks, spec)
        return spec

    _MASK_CACHE = 6

    def _mask_lookup(self, masks):
        for ms, vers, spec in self.__dict__.get("_mask_cache", ()):
            if len(ms) == len(masks) and all(a is b and a._version == v for a, b, v in zip(ms, masks, vers)):
                return spec
        return None

    def _mask_remember(self, masks, spec):
        cache = [e for e in self.__dict__.get("_mask_cache", []) if not all(a is b for a, b in zip(e[0], masks))]
        cache.append((tuple(masks), tuple(m._version for m in masks), spec))
        self.__dict__["_mask_cache"] = cache[-self._MASK_CACHE:]

    def block_prefix_counts(self, image_text_proprio_mask, action_mask):
        """int32 prefix counts for the static hipGraph path, which supports the Pi0 block mask only."""
        dev = self._dev()
        itp, am = image_text_proprio_mask.to(dev), action_mask.to(dev)
        L1 = itp.shape[2]
        spec = self._mask_spec([itp, am], [torch.arange(L1, device=dev), torch.arange(L1, L1 + am.shape[2], device=dev)])
        if not isinstance(spec, torch.Tensor):
            raise ValueError("the hipGraph inference path needs the Pi0 block mask (pizero.py:271-306); "
                             "call infer_action eagerly for a general mask")
        return spec

    def _dev(self):
        return self._arena.data.device

    def _cat_pos(self, *pos):
        return torch.cat([p.to(self._dev(), torch.int64) for p in pos], dim=1).contiguous()

    # ============================================================== forward ==
    def psi_t(self, x, x1, t):
        t = t[:, None, None]
        return (1 - (1 - self.flow_sig_min) * t) * x + t * x1

    def forward(self, input_ids, pixel_values, causal_mask, vlm_position_ids, proprio_position_ids,
                action_position_ids, proprios, actions, t, noise: Optional[torch.Tensor] = None):
        """Flow-matching loss (pizero.py:607-661); ``noise`` = x0 (default torch.randn_like)."""
        dev = self._dev()
        cdt = self._arena.data.dtype
        if cdt != torch.bfloat16:
            raise RuntimeError("the native path computes in bf16: call model.to(torch.bfloat16)")
        x1 = actions.to(dev, torch.float32).contiguous()
        x0 = (torch.randn_like(x1) if noise is None else noise.to(dev, torch.float32)).contiguous()
        cm = causal_mask.to(dev)
        tied = self._tied
        pos = {"vlm": vlm_position_ids.to(dev, torch.int64).contiguous()}
        if tied:
            pos["expert"] = self._cat_pos(proprio_position_ids, action_position_ids)
        else:
            pos["proprio"] = proprio_position_ids.to(dev, torch.int64).contiguous()
            pos["action"] = action_position_ids.to(dev, torch.int64).contiguous()
        batch = dict(ids=input_ids.to(dev, torch.int64).contiguous(),
                     pix=pixel_values.to(dev, torch.bfloat16).contiguous(),
                     cnt=self._mask_spec([cm], [torch.arange(cm.shape[2], device=dev)]), pos=pos,
                     proprios=proprios.to(dev, torch.float32).contiguous(), actions=x1,
                     t=t.to(dev, torch.float32).contiguous(), x0=x0)
        anchor = next((self._param(n) for n in self._trainable_names()), None)
        if anchor is not None and torch.is_grad_enabled():
            self._check_ddp_wrapper()
        if anchor is None or not torch.is_grad_enabled():
            save = {}
            return self._engine().train_forward(save=save, **batch).view(())
        return _PiZeroLoss.apply(anchor, self, batch)

    def _check_ddp_wrapper(self):
        """torch DDP (train.py:121-126) cannot reduce this model's gradients: the native backward writes
        them into the flat arena, so no per-parameter autograd hook ever fires and DDP would either skip
        the all-reduce or fail on the next step.  Multi-rank training must use PiZeroDDP."""
        import torch.distributed as dist

        if (dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
                and getattr(self, "_ddp_wrapper", None) is None):
            raise RuntimeError(
                "PiZero's native backward does not fire torch.nn.parallel.DistributedDataParallel's "
                "per-parameter hooks: wrap the model with pizero_native.ddp.PiZeroDDP (same .module / "
                "no_sync() / forward surface, bucketed RCCL all-reduce overlapped with the backward) "
                "instead of DistributedDataParallel (reference train.py:121-126)")

    # ============================================================ inference ==
    def _kv_buffers(self, B):
        e = self._engine()
        d = e.d
        if self._kv is None or self._kv[0].shape[1] != B:
            k = torch.zeros(d.nL, B, d.Lp, d.hd, device=self._dev(), dtype=torch.bfloat16)
            v = torch.zeros_like(k)
            self._kv = (k, v)
        return self._kv

    @torch.no_grad()
    def infer_action(self, input_ids, pixel_values, image_text_proprio_mask, action_mask, vlm_position_ids,
                     proprio_position_ids, action_position_ids, proprios, noise: Optional[torch.Tensor] = None,
                     clip: bool = True):
        """pizero.py:416-490: prefill caches vlm+proprio K/V once, 10 Euler steps on the action expert."""
        dev = self._dev()
        B = input_ids.shape[0]
        dtype = pixel_values.dtype
        if noise is None:
            noise = torch.randn(B, self.horizon_steps, self.action_dim, device=dev, dtype=torch.float32)
        k, v = self._kv_buffers(B)
        itp, am = image_text_proprio_mask.to(dev), action_mask.to(dev)
        L1 = itp.shape[2]
        spec = self._mask_spec([itp, am], [torch.arange(L1, device=dev),
                                           torch.arange(L1, L1 + am.shape[2], device=dev)])
        a = self._engine().infer_action(
            input_ids.to(dev, torch.int64).contiguous(), pixel_values.to(dev, torch.bfloat16).contiguous(),
            spec, vlm_position_ids.to(dev, torch.int64).contiguous(),
            proprio_position_ids.to(dev, torch.int64).contiguous(), action_position_ids.to(dev, torch.int64).contiguous(),
            proprios.to(dev, torch.float32).contiguous(), noise.to(dev, torch.float32).contiguous(), k, v,
            clip=clip and self.final_action_clip_value is not None)
        return a.to(dtype)

    @torch.no_grad()
    def infer_action_naive(self, input_ids, pixel_values, causal_mask, vlm_position_ids, proprio_position_ids,
                           action_position_ids, proprios, noise: Optional[torch.Tensor] = None, clip: bool = True):
        """pizero.py:492-557.  Re-running the prefix every step gives identical math (the vlm/proprio rows
        never attend to actions), so the native path reuses the cached prefix (fp32-exact equivalence:
        SURVEY 8(c) measured |naive - cached| = 1.8e-7)."""
        itp, amask = self.split_full_mask_into_submasks(causal_mask)
        return self.infer_action(input_ids, pixel_values, itp, amask, vlm_position_ids, proprio_position_ids,
                                 action_position_ids, proprios, noise=noise, clip=clip)

    def build_causal_mask_and_position_ids_for_text(self, q_len, attention_mask, kv_cache=None):
        """pizero.py:336-365: the all-zeros text mask (no masking: prefix-LM prefill, cached decode) and the
        positions cumsum(attention_mask) (pads -> 1; a cached decode step takes the last one).  The
        reference reads an undefined global ``bsz`` here; the batch size comes from attention_mask."""
        bsz = attention_mask.shape[0]
        dtype, device = attention_mask.dtype, attention_mask.device
        if kv_cache is None or kv_cache.num_items() == 0:
            mask = torch.zeros(bsz, q_len, q_len, dtype=dtype, device=device)
        else:
            if q_len != 1:
                raise ValueError("Using KV cache so should only use one single token")
            mask = torch.zeros(bsz, q_len, kv_cache.num_items() + q_len, dtype=dtype, device=device)
        mask = mask.unsqueeze(1)
        if kv_cache is not None and kv_cache.num_items() > 0:
            pos = attention_mask.cumsum(-1)[:, -1:]
        else:
            pos = attention_mask.cumsum(-1).masked_fill_(attention_mask == 0, 1)
        return mask, pos

    @torch.no_grad()
    def infer_text(self, input_ids, pixel_values, attention_mask, kv_cache: Optional[KVCache] = None):
        """pizero.py:559-593: {"logits": [B, q_len, vocab]} (+ "kv_cache").  The prompt prefill runs the
        vlm mixture over q_len tokens (image tokens merged from SigLIP); each later call feeds ONE new
        token that attends to the cache.  ``kv_cache`` is this repo's static KVCache (rows appended in
        place, grown when full); ``None`` -> a standalone prefill, like the reference."""
        if not self.use_lm_head:
            raise RuntimeError("infer_text needs use_lm_head: true (pizero.py:106-112)")
        dev = self._dev()
        ids = input_ids.to(dev, torch.int64).contiguous()
        B, q = ids.shape
        am = attention_mask.to(dev)
        _, pos = self.build_causal_mask_and_position_ids_for_text(q, am, kv_cache)
        eng = self._engine()
        d = eng.d
        cache = kv_cache if kv_cache is not None else KVCache()
        start = cache.num_items()
        if start == 0:
            cap = (q + 256 + 7) // 8 * 8
            cache.allocate(d.nL, B, cap, d.hd, dev)
        elif start + q > cache.k.shape[2]:  # grow (amortised) keeping the cached rows
            old_k, old_v = cache.k, cache.v
            cache.k = torch.zeros(d.nL, B, (start + q + 256 + 7) // 8 * 8, d.hd, device=dev, dtype=old_k.dtype)
            cache.v = torch.zeros_like(cache.k)
            cache.k[:, :, :start].copy_(old_k[:, :, :start])
            cache.v[:, :, :start].copy_(old_v[:, :, :start])
        n_img = int((ids == self.image_token_index).sum(1).max().item()) if start == 0 else 0
        pix = None
        if n_img:
            pix = pixel_values.to(dev, torch.bfloat16).contiguous()
            n_img = d.n_img
        # positions are cumsum(attention_mask) <= its length (pizero.py:363-371): bounds the RoPE table
        logits = eng.text_forward(ids, pix, pos.to(torch.int64).contiguous(), cache.k, cache.v, start, n_img,
                                  maxpos=am.shape[1])
        cache.length = start + q
        out = {"logits": logits}
        if kv_cache is not None:
            out["kv_cache"] = kv_cache
        return out


class PiZeroInference(PiZero):
    def forward(self, input_ids, pixel_values, image_text_proprio_mask, action_mask, vlm_position_ids,
                proprio_position_ids, action_position_ids, proprios, noise=None):
        return super().infer_action(input_ids, pixel_values, image_text_proprio_mask, action_mask,
                                    vlm_position_ids, proprio_position_ids, action_position_ids, proprios, noise=noise)
