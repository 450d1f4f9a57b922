"""Native layer executor for the Pi0 hot path (SigLIP + joint model, fwd/bwd/infer).

The executor walks the model with HIP kernels from libpizero_hip.so only; it
never calls torch math on the hot path (torch provides device memory and the
current stream).  Layout decisions (MI355X-first):

* residual streams are bf16 row-major ``[tokens, hidden]`` per weight group:
  the VLM group (image+text prefix, Gemma weights) and the action-expert group
  (proprio + action rows, shared weights after ``tie_action_proprio_weights``);
  every Linear is one MFMA GEMM on that stream (q|k|v and gate|up fused);
* the joint attention of the mixture-of-transformers (joint_model.py:130-304)
  gathers all groups' post-RoPE Q/K/V into joint token buffers
  ``Q[B, L, nh*hd]``, ``K/V[B, Lp, hd]`` (MQA: one KV head, so the 8 query
  heads are stacked as rows and no ``repeat_kv`` copy exists), then runs
  S = Q K^T and O = P V as per-sample batched MFMA GEMMs around a softmax
  kernel that applies the Gemma soft-cap and generates the block-causal mask
  arithmetically from per-sample prefix counts;
* backward reuses the same GEMM kernel in its k-strided layouts (dgrad /
  wgrad / attention products), writes parameter gradients straight into the
  flat gradient arena, and reports each finished layer to an optional hook
  (used by the data-parallel wrapper to start RCCL all-reduces of finished
  gradient buckets while the backward continues).
"""

from __future__ import annotations

import contextlib
import math
import os
import weakref
from dataclasses import dataclass

import torch

from . import ops
from .ops import PZ_EPI_DGEGLU, PZ_EPI_DGELU, PZ_EPI_GEGLU, PZ_EPI_GELU, PZ_EPI_NONE, PZ_EPI_SILU

BF16 = torch.bfloat16
F32 = torch.float32


def _cfg(cfg, key, default=None):
    from src.utils.config import cfg_get

    return cfg_get(cfg, key, default)


@dataclass
class Dims:
    P: int
    C: int
    H: int
    A: int
    Pd: int
    vocab: int
    image_token: int
    pad_token: int
    img: int
    ps: int
    n_img: int  # image tokens per sample (= img_tok x n_images)
    vH: int
    vI: int
    vL: int
    vheads: int
    ln_eps: float
    proj: int
    nL: int
    nh: int
    nkv: int
    hd: int
    rms_eps: float
    gH: int
    gI: int
    g_theta: float
    aH: int
    aI: int
    a_theta: float
    p_theta: float
    tmax: float
    sig_min: float
    steps: int
    clip: float | None
    time_bf16: bool = False  # pz_time_embed mode 1: the reference's bf16 arithmetic (see modules.py)
    n_images: int = 1  # images per sample (C5, the Pi0-paper shape: 3)

    @property
    def img_tok(self):
        """SigLIP tokens per image"""
        return (self.img // self.ps) ** 2

    @staticmethod
    def from_cfg(cfg):
        v = _cfg(cfg, "vision.config")
        j = _cfg(cfg, "joint.config")
        mix = _cfg(cfg, "mixture") or _cfg(j, "mixture")
        img = int(_cfg(v, "image_size"))
        ps = int(_cfg(v, "patch_size"))
        clip = _cfg(cfg, "final_action_clip_value", None)
        return Dims(
            P=int(_cfg(cfg, "max_image_text_tokens", _cfg(cfg, "max_seq_len"))), C=int(_cfg(cfg, "cond_steps")),
            H=int(_cfg(cfg, "horizon_steps")), A=int(_cfg(cfg, "action_dim")), Pd=int(_cfg(cfg, "proprio_dim")),
            vocab=int(_cfg(cfg, "vocab_size")), image_token=int(_cfg(cfg, "image_token_index")),
            pad_token=int(_cfg(cfg, "pad_token_id")), img=img, ps=ps,
            n_img=(img // ps) ** 2 * int(_cfg(cfg, "num_images", 1)),
            vH=int(_cfg(v, "hidden_size")), vI=int(_cfg(v, "intermediate_size")),
            vL=int(_cfg(v, "num_hidden_layers")), vheads=int(_cfg(v, "num_attention_heads")),
            ln_eps=float(_cfg(v, "layer_norm_eps", 1e-6)),
            proj=int(_cfg(cfg, "vision_projector.config.vision_config.projection_dim")),
            nL=int(_cfg(j, "num_hidden_layers")), nh=int(_cfg(j, "num_attention_heads")),
            nkv=int(_cfg(j, "num_key_value_heads")), hd=int(_cfg(j, "head_dim")),
            rms_eps=float(_cfg(j, "rms_norm_eps", 1e-6)),
            gH=int(_cfg(mix, "vlm.hidden_size")), gI=int(_cfg(mix, "vlm.intermediate_size")),
            g_theta=float(_cfg(mix, "vlm.rope_theta", 10000.0)),
            aH=int(_cfg(mix, "action.hidden_size")), aI=int(_cfg(mix, "action.intermediate_size")),
            a_theta=float(_cfg(mix, "action.rope_theta", 10000.0)),
            p_theta=float(_cfg(mix, "proprio.rope_theta", _cfg(mix, "action.rope_theta", 10000.0))),
            tmax=float(_cfg(cfg, "time_max_period", 10000.0)), sig_min=float(_cfg(cfg, "flow_sig_min", 0.001)),
            steps=int(_cfg(cfg, "num_inference_steps")), clip=None if clip is None else float(clip),
            time_bf16=bool(_cfg(cfg, "time_embed_bf16_reference", False)),
            n_images=int(_cfg(cfg, "num_images", 1)),
        )

    @property
    def L(self):
        return self.P + self.C + self.H

    @property
    def Lp(self):
        return (self.L + 7) // 8 * 8

    @property
    def kcols(self):
        return (3 * self.ps * self.ps + 31) // 32 * 32


def check_finite(where, **tensors):
    """Synchronise the device and raise FloatingPointError if a floating-point tensor holds NaN / Inf, naming the
    stage, the tensor and the native launches since the previous check (PZ_CHECK_FINITE debug instrument)."""
    from ._lib import recent_launches

    torch.cuda.synchronize()
    for k, t in tensors.items():
        if isinstance(t, dict):
            for k2, t2 in t.items():
                check_finite(where, **{f"{k}[{k2}]": t2})
            continue
        if not isinstance(t, torch.Tensor) or not t.is_floating_point() or t.numel() == 0:
            continue
        if not bool(torch.isfinite(t).all()):
            bad = int((~torch.isfinite(t)).sum())
            launches = recent_launches()
            raise FloatingPointError(f"PZ_CHECK_FINITE: {where}: {k} {tuple(t.shape)} {t.dtype} has {bad} non-finite "
                                     f"values; native launches since the previous check ({len(launches)}): "
                                     f"{launches[-40:]}")
    recent_launches()


class _Token:
    """Lifetime marker of the forward state that borrows the engine's joint K/V buffers."""


class GeneralMask:
    """A caller attention mask that is NOT the Pi0 block pattern (pizero.py:271-306).

    The reference adds any additive mask to the soft-capped logits (joint_model.py:261-287); such a
    mask is applied here by the GEMM + softmax path (pz_attn_softmax mask_mode 2, fp32 additive),
    never by the fused kernels, which generate the block mask from per-sample prefix counts.
    ``full``: fp32 [B, L, L] (training); ``itp``: fp32 [B, P+C, P+C] and ``act``: fp32 [B, H, L]
    (inference, pizero.py:326-336 split)."""

    def __init__(self, full=None, itp=None, act=None):
        self.full, self.itp, self.act = full, itp, act


def _mask_kw(d, cnt, which):
    """pz_attn_softmax mask arguments: block mask from cnt, or the general additive mask."""
    if isinstance(cnt, GeneralMask):
        m = getattr(cnt, which)
        return dict(mask_mode=2, mask=m, ldm=m.shape[2], mask_bstride=m.shape[1] * m.shape[2])
    return dict(mask_mode=1, cnt=cnt, prefix=d.P, cond=d.C)


class Group:
    """Rows of the joint sequence that share one set of mixture weights."""

    def __init__(self, name, prefix, mixtures, T, joint_off, hidden, inter, theta, skip_last, pos_key):
        self.name, self.prefix, self.mixtures = name, prefix, mixtures
        self.T, self.off, self.hid, self.inter, self.theta = T, joint_off, hidden, inter, theta
        self.skip_last = skip_last
        self.pos_key = pos_key


class Engine:
    def __init__(self, model):
        self.m = model
        self.d = Dims.from_cfg(model.cfg)
        self._tables = {}
        self._ws = {}
        self._jkv_holder = None
        # joint attention kernel: "gemm" = MFMA GEMMs around the soft-cap/block-mask softmax, "flash" = the
        # fused pz_flash kernels fwd + bwd (no L x L tensors), "probs" = fused forward that exports the
        # bf16 softmax (pz_flash_fwd_probs: no fp32 S, no softmax launch) + the GEMM-path backward
        # (default "probs": measured 237.5 vs 235.4 samples/s for "gemm" and 227.5 vs 231.1 for "flash")
        ja = os.environ.get("PZ_JOINT_ATTN", "probs")
        self.joint_flash = ja == "flash"
        self.joint_probs = ja == "probs"
        # GEMM-path backward's dS: "1" (default) = pz_flash_bwd_ds from the exported P (no fp32 dP), "0" = the
        # dP GEMM + pz_attn_softmax_bwd (A/B)
        self.joint_ds = os.environ.get("PZ_JOINT_DS", "1") == "1"
        # ... and dQ = dS K inside that launch ("0": the batched dQ GEMM, A/B)
        self.joint_ds_dq = os.environ.get("PZ_JOINT_DS_DQ", "1") == "1"
        # inference (prefill / denoise) attention: fused kernel unless PZ_INFER_ATTN=gemm
        self.infer_flash = os.environ.get("PZ_INFER_ATTN", "flash") == "flash"
        # activation backward of the training MLPs (PZ_SPLIT_DACT, A/B): "1" (default) = plain dgrad GEMM + a
        # vectorised elementwise pass; "0" = fused into the dgrad GEMM's epilogue, which the 8-phase kernel
        # cannot overlap with its main loop (measured: "1" +0.7 % samples/s)
        self.split_dact = os.environ.get("PZ_SPLIT_DACT", "1") == "1"
        # ... and of the Gemma GeGLU MLPs (PZ_SPLIT_DGEGLU, A/B): "0" (default) = d(gate|up) in the down-proj dgrad
        # epilogue, which became the faster form once the activations ran on the hardware exp / rcp (vlm layer
        # 1.390 vs 1.553 ms, action 24.2 vs 26.0 us, tools/dact_ab.py, profiles/r03/dact_ab.log); "1" = plain dgrad
        # + the separate geglu_bwd pass
        self.split_dgeglu = os.environ.get("PZ_SPLIT_DGEGLU", "0") == "1"
        # q|k|v GEMM with the RoPE + Q/K/V scatter in its epilogue (pz_gemm_qkv_rope) where the 8-phase kernel
        # runs; PZ_FUSE_QKV_ROPE=0: GEMM + pz_qkv_rope_split (A/B, bit-identical)
        self.fuse_qkv_rope = os.environ.get("PZ_FUSE_QKV_ROPE", "1") == "1" and self.d.hd == 256
        # backward of the action-expert group (M = B*(C+H) = 320 rows: latency-bound GEMMs) on a second HIP
        # stream, concurrent with the vlm group's (PZ_EXPERT_STREAM=0: one stream, A/B)
        self.expert_stream = os.environ.get("PZ_EXPERT_STREAM", "1") == "1"
        # ... and in the forward (PZ_EXPERT_STREAM_FWD=1): measured no faster than backward-only (bench 238.9 vs
        # 239.3 samples/s), and its expert GEMMs then share the CUs with the vlm GeGLU GEMM (the dominant
        # kernel: live roofline 2.32 vs 2.19 ms per launch), so off by default
        self.expert_stream_fwd = os.environ.get("PZ_EXPERT_STREAM_FWD", "0") == "1"
        # row pitch of SigLIP's MLP activations (fc1 output / pre-activation / their gradient, 4304 wide): rounded up
        # to 64 elements, so every row starts on a 128-B line (8704 B instead of 8608 B).  The GEMMs that stream
        # these rows run 2-8 % faster with bitwise-equal results (profiles/r04/ld_pad_ab.txt); the pad columns are
        # never read (K tails clamp their sources into the row).  PZ_SIG_PITCH=0: natural pitch (A/B)
        vI = self.d.vI
        self.sig_pitch = vI if os.environ.get("PZ_SIG_PITCH", "1") == "0" else (vI + 63) // 64 * 64
        self._side = {}
        # PZ_CHECK_FINITE=1 (debug): after every layer / stage of the training forward and backward (and in
        # FusedAdamW.step) synchronise and check the stage's outputs; the first non-finite tensor raises
        # FloatingPointError naming the stage, the tensor and the kernels launched since the previous check
        self.check_finite = os.environ.get("PZ_CHECK_FINITE", "0") == "1"
        # fp8 inference (C5): weight key -> (e4m3 codes, per-tensor scale); built by prepare_fp8()
        # in fp8 mode the prefill's joint attention runs S = Q K^T and P V on the fp8 MFMA (pz_flash_fwd_f8;
        # PZ_FP8_ATTN=0: the bf16 kernel, A/B) and the 65..1024-row q|k|v / o projections run W8A8 on the row-slab
        # kernel (activation rows quantised per row; PZ_ROWS_W8A8=0: W8A16 as in round 5)
        self.f8_attn = os.environ.get("PZ_FP8_ATTN", "1") == "1"
        self.f8 = None
        self.f8_version = None
        if self.d.nkv != 1:
            raise NotImplementedError("joint attention kernel path assumes MQA (num_key_value_heads=1, bridge.yaml:176)")

    def _chk(self, where, **tensors):
        """PZ_CHECK_FINITE: raise on the first non-finite tensor of this stage (no-op otherwise)"""
        if not self.check_finite:
            return
        check_finite(where, **tensors)

    # ------------------------------------------------------------- weights --
    @property
    def ar(self):
        return self.m._arena

    def w(self, name):
        return self.ar.view(name)

    def gw(self, name):
        return self.ar.grad_view(name)

    def rg(self, name):
        return self.m._requires_grad(name)

    def qkv_w(self, p):
        return self.ar.span(p + "self_attn.q_proj.weight", p + "self_attn.v_proj.weight")

    def gu_w(self, p):
        return self.ar.span(p + "mlp.gate_proj.weight", p + "mlp.up_proj.weight")

    # ------------------------------------------------------------ fp8 (C5) --
    def prepare_fp8(self):
        """fp8 e4m3 copies (per-tensor scale max|W|/448) of every inference Linear of SigLIP, the vlm
        mixture and the action expert (BASELINE.json configs[4]: fp8 attention / MLP GEMMs).  Prefill
        GEMMs (>= 65 rows) run W8A8 on the fp8 MFMA with per-row activation scales, except the row-slab
        shapes (<= 1024 rows, K <= 2048, <= 4096 columns: q|k|v / o), which run W8A16 like the denoise rows
        (<= 64: codes expanded to bf16 in registers, RMSNorm still fused).  Taken from the
        current weights; the codes carry the arena's weight version (``weights_version``) and every
        inference entry point re-quantises them when the weights changed since (fp8_refresh)."""
        d = self.d
        self.f8_version = self.weights_version()
        vt = "vision_tower.vision_model.encoder.layers."
        keys = []
        for i in range(d.vL):
            p = f"{vt}{i}."
            keys += [("span", p + "self_attn.q_proj.weight", p + "self_attn.v_proj.weight"),
                     ("w", p + "self_attn.out_proj.weight"), ("w", p + "mlp.fc1.weight"), ("w", p + "mlp.fc2.weight")]
        for mix in ("vlm", "action"):
            for l in range(d.nL):
                p = f"joint_model.mixtures.{mix}.layers.{l}."
                keys += [("span", p + "self_attn.q_proj.weight", p + "self_attn.v_proj.weight"),
                         ("w", p + "self_attn.o_proj.weight"),
                         ("span", p + "mlp.gate_proj.weight", p + "mlp.up_proj.weight"),
                         ("w", p + "mlp.down_proj.weight")]
        f8 = {}
        for k in keys:
            W = self.ar.span(k[1], k[2]) if k[0] == "span" else self.w(k[1])
            sc = ops.fp8_weight_scale(W)
            q = torch.empty(W.shape, device=W.device, dtype=torch.uint8)
            ops.fp8_quant_tensor(W, q, sc)
            f8[k[1]] = (q, sc)
        self.f8 = f8

    def weights_version(self):
        """Version of the weight arena: the shared version counter of arena.data, which torch bumps for
        every in-place write through a parameter view (load_state_dict, load_pretrained_weights,
        ``p.copy_``) and FusedAdamW.step bumps after its raw-pointer kernel writes."""
        return self.ar.data._version

    def fp8_refresh(self):
        """Re-quantise the fp8 weight copies if the weights changed after prepare_fp8 (stale
        e4m3 codes after an optimizer step / checkpoint load).  Returns True if it re-quantised."""
        if self.f8 is None or self.f8_version == self.weights_version():
            return False
        self.prepare_fp8()
        return True

    def lin(self, x, key, W, out, *, bias=None, resid=None, epi=PZ_EPI_NONE, aux=None, norm=None):
        """ops.linear, or its fp8 form when prepare_fp8() holds codes for ``key`` (the weight name; the
        first name of a span): W8A16 for <= 64 rows (norm may stay fused), else per-row quantised
        activations (norm must already be applied) and W8A8."""
        f = self.f8.get(key) if self.f8 else None
        if f is None:
            return ops.linear(x, W, out, bias=bias, resid=resid, epi=epi, aux=aux, norm=norm)
        q, sc = f
        if isinstance(x, tuple):  # (e4m3 codes, row scales) from a fused norm + quantisation (w8a8_in): W8A8
            return ops.linear_fp8(x[0], q, sc, out, bias=bias, resid=resid, epi=epi, aux=aux, x_scale=x[1])
        M, K = x.shape
        if M <= 64:
            if K % 64:  # (SigLIP fc2, K = 4304, never has so few rows in practice)
                return ops.linear(x, W, out, bias=bias, resid=resid, epi=epi, aux=aux, norm=norm)
            return ops.linear_fp8(x, q, sc, out, bias=bias, resid=resid, epi=epi, aux=aux, norm=norm)
        ncols = W.shape[0] // 2 if epi == PZ_EPI_GEGLU else W.shape[0]
        if norm is None and ops.rows_w8a16_ok(M, K, ncols):
            # bf16 rows from a producer that cannot emit codes (the attention output into o_proj): W8A16 on the
            # row-slab kernel -- quantising them costs a launch (~5 us) that the latency-bound W8A8 GEMM does not win
            # back (profiles/r06/c5_fp8_ab.txt)
            return ops.linear_fp8(x, q, sc, out, bias=bias, resid=resid, epi=epi, aux=aux)
        if norm is not None:
            raise ValueError("lin: a fused norm needs <= 64 rows")
        if K % 16 or x.stride(0) % 16:  # W8A8 stages K in 16-code steps (tiny test widths: bf16)
            return ops.linear(x, W, out, bias=bias, resid=resid, epi=epi, aux=aux)
        xq = torch.empty(x.shape, device=x.device, dtype=torch.uint8)
        xs = torch.empty(M, device=x.device, dtype=F32)
        ops.fp8_quant_rows(x, xq, xs)
        return ops.linear_fp8(xq, q, sc, out, bias=bias, resid=resid, epi=epi, aux=aux, x_scale=xs)

    def w8a8_in(self, key, M, K):
        """fp8 mode: True if the Linear ``key`` on M > 64 rows should get its A operand as e4m3 codes from a fused norm
        (pz_rmsnorm_fwd_f8 / pz_layernorm_fwd_f8): W8A8 on the fp8 MFMA (row slab or 8-phase) with no quantisation
        launch (PZ_FUSED_NORM_F8=0: bf16 norm output, lin() quantises or runs W8A16)"""
        return (self.f8 is not None and key in self.f8 and M > 64 and K % 16 == 0 and
                os.environ.get("PZ_FUSED_NORM_F8", "1") != "0")

    def norm_codes(self, x, w, eps, b=None):
        """(codes [M, K], row scales [M]) of RMSNorm (b None) / LayerNorm (b given) of x, in one launch"""
        xq = torch.empty(x.shape, device=x.device, dtype=torch.uint8)
        xs = torch.empty(x.shape[0], device=x.device, dtype=F32)
        if b is None:
            ops.rmsnorm_f8(x, w, xq, xs, eps)
        else:
            ops.layernorm_f8(x, w, b, xq, xs, eps)
        return xq, xs

    def rope(self, theta, maxpos=None):
        """fp32 cos|sin table for positions 0..maxpos (default L + 8: every training / action position);
        text generation asks for longer tables (a new, power-of-two sized table: graphs captured on the
        default one keep it)"""
        dev = self.ar.data.device
        base = self.d.L + 8
        if maxpos is not None and maxpos > base:
            base = 1 << (int(maxpos) - 1).bit_length()
        key = (float(theta), dev, base)
        if key not in self._tables:
            maxpos = base
            cs = torch.empty((maxpos + 1) * self.d.hd, device=dev, dtype=F32)
            ops.rope_table(cs, maxpos, self.d.hd, theta)
            self._tables[key] = cs
        return self._tables[key]

    def colsum_ws_rows(self, rows, n):
        """fp32 [rows, n] partial-sum scratch (pz_act_bwd_colsum), one per device, grown on demand"""
        dev = self.ar.data.device
        t = self._ws.get(("colsum_rows", dev))
        if t is None or t.numel() < rows * n:
            t = torch.empty(rows * n, device=dev, dtype=F32)
            self._ws[("colsum_rows", dev)] = t
        return t[: rows * n].view(rows, n)

    def colsum_ws(self, n):
        dev = self.ar.data.device
        t = self._ws.get(("colsum", dev))
        if t is None or t.numel() < 64 * n:
            t = torch.empty(64 * max(n, 4608), device=dev, dtype=F32)
            self._ws[("colsum", dev)] = t
        return t

    def groups(self, tied, active=("vlm", "proprio", "action")):
        d = self.d
        out = []
        mp = "joint_model.mixtures."
        if "vlm" in active:
            out.append(Group("vlm", mp + "vlm.layers.", ["vlm"], d.P, 0, d.gH, d.gI, d.g_theta, True, "vlm"))
        if tied:
            mix = [m for m in ("proprio", "action") if m in active]
            T = (d.C if "proprio" in mix else 0) + (d.H if "action" in mix else 0)
            if T:
                off = d.P if "proprio" in mix else d.P + d.C
                out.append(Group("expert", mp + "action.layers.", mix, T, off, d.aH, d.aI, d.a_theta,
                                 mix == ["proprio"], "expert"))
        else:
            if "proprio" in active:
                out.append(Group("proprio", mp + "proprio.layers.", ["proprio"], d.C, d.P, d.aH, d.aI, d.p_theta,
                                 True, "proprio"))
            if "action" in active:
                out.append(Group("action", mp + "action.layers.", ["action"], d.H, d.P + d.C, d.aH, d.aI,
                                 d.a_theta, False, "action"))
        return out

    # ------------------------------------------------------- second stream --
    def _side_stream(self, dev):
        st = self._side.get(dev)
        if st is None:
            st = self._side[dev] = torch.cuda.Stream(device=dev)
        return st

    @staticmethod
    def _on(side, g):
        """Context of one group's work: the action-expert group on the side stream with its own GEMM scratch
        (ops.workspace_slot), the vlm group on the current stream."""
        if side is None or g.name == "vlm":
            return contextlib.nullcontext()
        stack = contextlib.ExitStack()
        stack.enter_context(torch.cuda.stream(side))
        stack.enter_context(ops.workspace_slot(1))
        return stack

    # ================================================================ SigLIP ==
    def _sig_rows(self, M, dev):
        """[M, vI] bf16 rows at the SigLIP MLP row pitch (a view of [M, sig_pitch])"""
        return torch.empty(M, self.sig_pitch, device=dev, dtype=BF16)[:, : self.d.vI]

    def siglip_forward(self, pix, save):
        """siglip.py:34-300 + projector (siglip.py:9-31). pix bf16 [B,3,H,W] or [B,n_images,3,H,W] ->
        img [B*n_img, proj] (a sample's images' tokens consecutive, in image order)."""
        d = self.d
        pix = pix.reshape(-1, 3, d.img, d.img)
        B = pix.shape[0]  # images
        Nt = d.img_tok
        M = B * Nt
        dev = pix.device
        vt = "vision_tower.vision_model."
        kc = d.kcols
        cols = torch.empty(M, kc, device=dev, dtype=BF16)
        ops.patchify(pix, cols, d.ps)
        # patch-embedding weight with its K padded to a multiple of 32 columns: an engine-owned buffer whose
        # pad columns are zeroed once; the weight columns are refreshed by every forward (weights change)
        wpad = self._ws.get(("wpad", dev))
        if wpad is None:
            wpad = self._ws[("wpad", dev)] = torch.zeros(d.vH, kc, device=dev, dtype=BF16)
        wpatch = self.w(vt + "embeddings.patch_embedding.weight").view(d.vH, -1)
        ops.copy_rows(wpatch, wpatch.shape[1], 0, wpad, kc, 0, 1, d.vH, wpatch.shape[1])
        x = torch.empty(M, d.vH, device=dev, dtype=BF16)
        ops.gemm(Nt, d.vH, kc, cols, kc, True, wpad, kc, True, x, d.vH, batch=B, sA=(Nt * kc, 0),
                 sC=(Nt * d.vH, 0), bias=self.w(vt + "embeddings.patch_embedding.bias"),
                 resid=self.w(vt + "embeddings.position_embedding.weight"), ld_resid=d.vH, sR=(0, 0))
        if save is not None:
            save["cols"] = cols
        nh, hd = d.vheads, d.vH // d.vheads
        Np = Nt
        layers = []

        def L(x_, key, W, out, **kw):  # fp8 codes (prepare_fp8) serve inference only
            return self.lin(x_, p + key, W, out, **kw) if save is None else ops.linear(x_, W, out, **kw)

        for i in range(d.vL):
            p = f"{vt}encoder.layers.{i}."
            st = {"x": x}
            if save is None and self.w8a8_in(p + "self_attn.q_proj.weight", M, d.vH):  # fp8: LayerNorm -> codes
                h1 = self.norm_codes(x, self.w(p + "layer_norm1.weight"), d.ln_eps, self.w(p + "layer_norm1.bias"))
                mu1 = r1 = None
            else:
                h1 = torch.empty_like(x)
                mu1 = torch.empty(M, device=dev, dtype=F32)
                r1 = torch.empty(M, device=dev, dtype=F32)
                ops.layernorm(x, self.w(p + "layer_norm1.weight"), self.w(p + "layer_norm1.bias"), h1, mu1, r1,
                              d.ln_eps)
            qkv = torch.empty(M, 3 * d.vH, device=dev, dtype=BF16)
            L(h1, "self_attn.q_proj.weight", self.ar.span(p + "self_attn.q_proj.weight", p + "self_attn.v_proj.weight"),
              qkv, bias=self.ar.span(p + "self_attn.q_proj.bias", p + "self_attn.v_proj.bias"))
            # fused attention (siglip.py:108-166) in place on the q|k|v rows: O and one fp32
            # log-sum-exp per (head, query) row; no [B, heads, N, N] tensor exists
            O = torch.empty(M, d.vH, device=dev, dtype=BF16)
            lse = torch.empty(B * nh, Np, device=dev, dtype=F32)
            ops.flash_fwd(ops.siglip_flash_args(qkv, O, lse, B, nh, hd, Np))
            xm = torch.empty_like(x)
            L(O, "self_attn.out_proj.weight", self.w(p + "self_attn.out_proj.weight"), xm,
              bias=self.w(p + "self_attn.out_proj.bias"), resid=x)
            if save is None and self.w8a8_in(p + "mlp.fc1.weight", M, d.vH):  # fp8: LayerNorm -> codes
                h2 = self.norm_codes(xm, self.w(p + "layer_norm2.weight"), d.ln_eps, self.w(p + "layer_norm2.bias"))
                mu2 = r2 = None
            else:
                h2 = torch.empty_like(x)
                mu2 = torch.empty(M, device=dev, dtype=F32)
                r2 = torch.empty(M, device=dev, dtype=F32)
                ops.layernorm(xm, self.w(p + "layer_norm2.weight"), self.w(p + "layer_norm2.bias"), h2, mu2, r2,
                              d.ln_eps)
            a1 = self._sig_rows(M, dev) if save is not None else None
            g1 = self._sig_rows(M, dev)
            L(h2, "mlp.fc1.weight", self.w(p + "mlp.fc1.weight"), g1, bias=self.w(p + "mlp.fc1.bias"), epi=PZ_EPI_GELU,
              aux=a1)
            xn = torch.empty_like(x)
            L(g1, "mlp.fc2.weight", self.w(p + "mlp.fc2.weight"), xn, bias=self.w(p + "mlp.fc2.bias"), resid=xm)
            if save is not None:
                st.update(h1=h1, mu1=mu1, r1=r1, qkv=qkv, lse=lse, O=O, xm=xm, h2=h2, mu2=mu2, r2=r2, a1=a1, g1=g1)
                layers.append(st)
                self._chk(f"siglip fwd layer {i}", h1=h1, qkv=qkv, O=O, lse=lse, xm=xm, h2=h2, g1=g1, x=xn)
            x = xn
        y = torch.empty_like(x)
        mu = torch.empty(M, device=dev, dtype=F32)
        r = torch.empty(M, device=dev, dtype=F32)
        ops.layernorm(x, self.w(vt + "post_layernorm.weight"), self.w(vt + "post_layernorm.bias"), y, mu, r, d.ln_eps)
        img = torch.empty(M, d.proj, device=dev, dtype=BF16)
        ops.linear(y, self.w("multi_modal_projector.linear.weight"), img, bias=self.w("multi_modal_projector.linear.bias"))
        if save is not None:
            save.update(layers=layers, x_last=x, y=y, mu=mu, r=r, B=B)
            self._chk("siglip fwd post-LN + projector", y=y, img=img)
        return img

    def siglip_backward(self, sv, dimg, beta):
        d = self.d
        B = sv["B"]  # images
        M = B * d.img_tok
        dev = dimg.device
        vt = "vision_tower.vision_model."
        rpp = ops.rows_per_part()
        P = (M + rpp - 1) // rpp
        ws = self.colsum_ws(max(d.vI, 3 * d.vH))
        pw = torch.empty(P, d.vH, device=dev, dtype=F32)
        pb = torch.empty(P, d.vH, device=dev, dtype=F32)
        # bias gradients fused into the passes that produce their output gradients (LayerNorm backward -> the
        # column sums of dx: fc2 / out_proj; GELU backward -> fc1); PZ_FUSED_BIAS_GRAD=0: separate colsum passes
        fb = os.environ.get("PZ_FUSED_BIAS_GRAD", "1") != "0" and os.environ.get("PZ_NORM_BWD", "row")[:1] != "w"
        pd = torch.empty(P, d.vH, device=dev, dtype=F32) if fb else None  # column partials of the current dx
        pdn = torch.empty(P, d.vH, device=dev, dtype=F32) if fb else None  # ... of the next layer's dx
        pd2 = torch.empty(P, d.vH, device=dev, dtype=F32) if fb else None  # ... of dxm
        # a layer's LayerNorm weight / bias and Linear bias reductions go out as one launch at its end
        # (pz_reduce_parts_multi; PZ_REDUCE_MULTI=0: one launch each)
        multi = os.environ.get("PZ_REDUCE_MULTI", "1") != "0"
        pw2 = torch.empty(P, d.vH, device=dev, dtype=F32) if multi else pw
        pb2 = torch.empty(P, d.vH, device=dev, dtype=F32) if multi else pb
        ws_act = self.colsum_ws_rows(1024, d.vI) if fb else None
        # projector
        nm = "multi_modal_projector.linear."
        if self.rg(nm + "weight"):
            ops.linear_wgrad(dimg, sv["y"], self.gw(nm + "weight"), beta=beta)
        if self.rg(nm + "bias"):
            ops.colsum(dimg, self.gw(nm + "bias"), ws, beta=beta)
        dy = torch.empty(M, d.vH, device=dev, dtype=BF16)
        ops.linear_dgrad(dimg, self.w(nm + "weight"), dy)
        dx = torch.empty_like(dy)
        ops.layernorm_bwd(dy, sv["x_last"], self.w(vt + "post_layernorm.weight"), sv["mu"], sv["r"], dx,
                          dw_part=pw, db_part=pb, dx_part=pd)
        self._norm_grads(vt + "post_layernorm.", pw, pb, beta)
        nh, hd = d.vheads, d.vH // d.vheads
        Np = d.img_tok
        W3 = 3 * d.vH
        dg = self._sig_rows(M, dev)
        delta = torch.empty(B * nh, Np, device=dev, dtype=F32)
        dqkv = torch.empty(M, W3, device=dev, dtype=BF16)
        dh = torch.empty(M, d.vH, device=dev, dtype=BF16)
        dxm = torch.empty(M, d.vH, device=dev, dtype=BF16)
        dO = torch.empty(M, d.vH, device=dev, dtype=BF16)
        for i in reversed(range(d.vL)):
            p = f"{vt}encoder.layers.{i}."
            st = sv["layers"][i]
            red = [] if multi else None  # deferred (partials, gradient) reductions of this layer
            # MLP: x' = xm + fc2(gelu(fc1(ln2(xm))))
            # dgrad through fc2, then the GELU derivative at the saved pre-activation a1
            fc1b = self.rg(p + "mlp.fc1.bias")
            if self.split_dact:  # plain dgrad GEMM, then the GELU backward (HBM-bound) in place
                ops.linear_dgrad(dx, self.w(p + "mlp.fc2.weight"), dg)
                if fb and fc1b:  # + the fc1 bias gradient from the same pass
                    ops.act_bwd_colsum(dg, st["a1"], dg, PZ_EPI_GELU, ws_act, self.gw(p + "mlp.fc1.bias"), beta=beta)
                else:
                    ops.act_bwd(dg, st["a1"], dg, None, PZ_EPI_GELU)
            else:
                ops.linear_dgrad(dx, self.w(p + "mlp.fc2.weight"), dg, epi=PZ_EPI_DGELU, aux=st["a1"])
            if self.rg(p + "mlp.fc2.weight"):
                ops.linear_wgrad(dx, st["g1"], self.gw(p + "mlp.fc2.weight"), beta=beta)
            st["g1"] = None
            if self.rg(p + "mlp.fc2.bias"):
                if fb:  # column sums of dx from the LayerNorm backward that produced it
                    self._reduce(red, pd, self.gw(p + "mlp.fc2.bias"), beta)
                else:
                    ops.colsum(dx, self.gw(p + "mlp.fc2.bias"), ws, beta=beta)
            if self.rg(p + "mlp.fc1.weight"):
                ops.linear_wgrad(dg, st["h2"], self.gw(p + "mlp.fc1.weight"), beta=beta)
            if fc1b and not (fb and self.split_dact):
                ops.colsum(dg, self.gw(p + "mlp.fc1.bias"), ws, beta=beta)
            ops.linear_dgrad(dg, self.w(p + "mlp.fc1.weight"), dh)
            ops.layernorm_bwd(dh, st["xm"], self.w(p + "layer_norm2.weight"), st["mu2"], st["r2"], dxm, dres=dx,
                              dw_part=pw2, db_part=pb2, dx_part=pd2)
            self._norm_grads(p + "layer_norm2.", pw2, pb2, beta, red)
            # attention out-proj
            if self.rg(p + "self_attn.out_proj.weight"):
                ops.linear_wgrad(dxm, st["O"], self.gw(p + "self_attn.out_proj.weight"), beta=beta)
            if self.rg(p + "self_attn.out_proj.bias"):
                if fb:
                    self._reduce(red, pd2, self.gw(p + "self_attn.out_proj.bias"), beta)
                else:
                    ops.colsum(dxm, self.gw(p + "self_attn.out_proj.bias"), ws, beta=beta)
            ops.linear_dgrad(dxm, self.w(p + "self_attn.out_proj.weight"), dO)
            # fused attention backward: dQ | dK | dV straight into the q|k|v gradient rows
            ops.flash_bwd(ops.siglip_flash_args(st["qkv"], st["O"], st["lse"], B, nh, hd, Np, dO=dO, delta=delta,
                                                dqkv=dqkv))
            qn, vn = p + "self_attn.q_proj.", p + "self_attn.v_proj."
            if all(self.rg(p + f"self_attn.{k}_proj.weight") for k in "qkv"):
                ops.linear_wgrad(dqkv, st["h1"], self.ar.grad_span(qn + "weight", vn + "weight"), beta=beta)
            else:
                for k, c0 in (("q", 0), ("k", d.vH), ("v", 2 * d.vH)):
                    if self.rg(p + f"self_attn.{k}_proj.weight"):
                        ops.linear_wgrad(dqkv[:, c0:c0 + d.vH], st["h1"], self.gw(p + f"self_attn.{k}_proj.weight"),
                                         beta=beta)
            if all(self.rg(p + f"self_attn.{k}_proj.bias") for k in "qkv"):
                ops.colsum(dqkv, self.ar.grad_span(qn + "bias", vn + "bias"), ws, beta=beta)
            ops.linear_dgrad(dqkv, self.qkv_siglip(p), dh)
            dxn = torch.empty_like(dx)
            ops.layernorm_bwd(dh, st["x"], self.w(p + "layer_norm1.weight"), st["mu1"], st["r1"], dxn, dres=dxm,
                              dw_part=pw, db_part=pb, dx_part=pdn)
            self._norm_grads(p + "layer_norm1.", pw, pb, beta, red)
            if red:
                ops.reduce_parts_multi(red, beta=beta)
            pd, pdn = pdn, pd  # this layer's dxn partials: the next (lower) layer's fc2 bias gradient
            dx = dxn
            self._chk(f"siglip bwd layer {i}", dg=dg, dO=dO, dqkv=dqkv, dxm=dxm, dx=dxn)
            self._notify("vision", i)
        # patch embedding + position embedding
        pe = vt + "embeddings."
        if self.rg(pe + "position_embedding.weight"):
            ops.batch_sum(dx, B, d.img_tok * d.vH, d.img_tok * d.vH, self.gw(pe + "position_embedding.weight"),
                          beta=beta)
        if self.rg(pe + "patch_embedding.bias"):
            ops.colsum(dx, self.gw(pe + "patch_embedding.bias"), ws, beta=beta)
        if self.rg(pe + "patch_embedding.weight"):
            kc = d.kcols
            tmp = torch.empty(d.vH, kc, device=dev, dtype=BF16)
            ops.linear_wgrad(dx, sv["cols"], tmp)
            g = self.gw(pe + "patch_embedding.weight").view(d.vH, -1)
            ops.copy_rows(tmp, kc, 0, g, g.shape[1], 0, 1, d.vH, g.shape[1], beta=beta)
        self._notify("vision", -1)

    def qkv_siglip(self, p):
        return self.ar.span(p + "self_attn.q_proj.weight", p + "self_attn.v_proj.weight")

    def _norm_grads(self, prefix, pw, pb, beta, red=None):
        if pw is not None and self.rg(prefix + "weight"):
            self._reduce(red, pw, self.gw(prefix + "weight"), beta)
        if pb is not None and self.rg(prefix + "bias"):
            self._reduce(red, pb, self.gw(prefix + "bias"), beta)

    @staticmethod
    def _reduce(red, part, out, beta):
        """reduce_parts now (red None) or deferred into the layer's list for one pz_reduce_parts_multi launch"""
        if red is None:
            ops.reduce_parts(part, out, beta=beta)
        else:
            red.append((part, out))

    # ============================================================ embeddings ==
    def embed_prefix(self, ids, img):
        d = self.d
        B = ids.shape[0]
        X = torch.empty(B * d.P, d.gH, device=ids.device, dtype=BF16)
        # pizero.py:395 (/sqrt(hidden)) and joint_model.py:355 (*sqrt(hidden)) cancel for image rows
        ops.embed_merge(ids, self.w("embed_tokens.weight"), img, X, d.n_img, d.image_token, d.pad_token,
                        math.sqrt(d.gH), 1.0)
        return X

    def _action_embed_tail(self, cat, alpha=1.0):
        """the action encoder after its concat input (inference): Linear + SiLU, Linear -- the last one times alpha
        (a power of two: the bias is pre-scaled by it, exactly, and cached per weight version)"""
        d = self.d
        e2 = torch.empty(cat.shape[0], d.aH, device=cat.device, dtype=BF16)
        ops.linear(cat, self.w("action_encoder.linear_2.weight"), e2, bias=self.w("action_encoder.linear_2.bias"),
                   epi=PZ_EPI_SILU)
        e3 = torch.empty_like(e2)
        b3 = self.w("action_encoder.linear_3.bias")
        if alpha != 1.0:
            if getattr(self, "_b3s_alpha", None) != alpha:
                self._b3s = torch.empty_like(b3)
                self._b3s_alpha, self._b3s_version = alpha, None
            self.derived_refresh()
            b3 = self._b3s
        ops.linear(e2, self.w("action_encoder.linear_3.weight"), e3, bias=b3, alpha=alpha)
        return e3

    def derived_refresh(self):
        """Recompute the weight-derived bf16 tensors (the alpha-scaled action-encoder bias) IN PLACE when the
        weights changed: a captured InferenceGraph holds their pointers, so InferenceGraph.replay calls this
        before every replay.  Returns True if it recomputed."""
        if getattr(self, "_b3s_alpha", None) is None or self._b3s_version == self.weights_version():
            return False
        b3 = self.w("action_encoder.linear_3.bias")
        self._b3s.copy_(b3.float() * self._b3s_alpha)  # exact: alpha is a power of two
        self._b3s_version = self.weights_version()
        return True

    def action_embed(self, psi_bf, t, save):
        """ActionEncoder (vla/modules.py:39-53) with time embedding (vla/modules.py:15-22).  Inference (save None):
        the first Linear and the time embedding write straight into the concat input (pz_time_embed_rows: no
        separate embedding buffer or concat launch) and no pre-activation is kept."""
        d = self.d
        rows = psi_bf.shape[0]
        B = t.shape[0]
        dev = psi_bf.device
        if save is None:
            cat = torch.empty(rows, 2 * d.aH, device=dev, dtype=BF16)
            ops.small_linear(psi_bf, self.w("action_encoder.linear_1.weight"), cat[:, d.aH:],
                             bias=self.w("action_encoder.linear_1.bias"))
            ops.time_embed_rows(t, cat[:, : d.aH], rows // B, d.tmax, ref_bf16=d.time_bf16)
            e2 = torch.empty(rows, d.aH, device=dev, dtype=BF16)
            ops.linear(cat, self.w("action_encoder.linear_2.weight"), e2, bias=self.w("action_encoder.linear_2.bias"),
                       epi=PZ_EPI_SILU)
            e3 = torch.empty(rows, d.aH, device=dev, dtype=BF16)
            ops.linear(e2, self.w("action_encoder.linear_3.weight"), e3, bias=self.w("action_encoder.linear_3.bias"))
            return e3
        e1 = torch.empty(rows, d.aH, device=dev, dtype=BF16)
        ops.small_linear(psi_bf, self.w("action_encoder.linear_1.weight"), e1, bias=self.w("action_encoder.linear_1.bias"))
        temb = torch.empty(B, d.aH, device=dev, dtype=BF16)
        ops.time_embed(t, temb, d.tmax, ref_bf16=d.time_bf16)
        cat = torch.empty(rows, 2 * d.aH, device=dev, dtype=BF16)
        ops.concat_time(temb, e1, cat, B, rows // B, d.aH)
        pre = torch.empty(rows, d.aH, device=dev, dtype=BF16)
        e2 = torch.empty(rows, d.aH, device=dev, dtype=BF16)
        ops.linear(cat, self.w("action_encoder.linear_2.weight"), e2, bias=self.w("action_encoder.linear_2.bias"),
                   epi=PZ_EPI_SILU, aux=pre)
        e3 = torch.empty(rows, d.aH, device=dev, dtype=BF16)
        ops.linear(e2, self.w("action_encoder.linear_3.weight"), e3, bias=self.w("action_encoder.linear_3.bias"))
        if save is not None:
            save.update(ae_psi=psi_bf, ae_cat=cat, ae_pre=pre, ae_e2=e2)
        return e3

    # ======================================================== joint layers ==
    def _joint_flash(self, groups, Q, K, V, Os, lse, cnt, B, Lq, dO=None, delta=None, dq=None, dk=None, dv=None):
        """pz_flash_args of the joint attention: query rows r = token*nh + head of Q [B, Lq*nh, hd],
        keys/values K, V [B, Lp, hd]; output groups = the mixtures' O buffers [B*T, nh*hd] in
        token order (joint_model.py:259-292 with the Pi0 block mask, pizero.py:271-306)."""
        d = self.d
        nh, hd, Lp = d.nh, d.hd, K.shape[1]
        gs = sorted(groups, key=lambda g: g.off)
        return ops.flash_args(
            B, 1, Lq * nh, d.L, hd, Q, (hd, Lq * nh * hd, 0), K, (hd, Lp * hd, 0), V, (hd, Lp * hd, 0),
            [(g.off * nh, Os[g.name], g.T * nh * hd, hd) for g in gs], 0, lse, 1.0 / math.sqrt(hd), cap=50.0,
            mask_mode=1, cnt=cnt, prefix=d.P, cond=d.C, rows_per_token=nh,
            dgroups=None if dO is None else [dO.get(g.name) for g in gs], delta=delta, dq=dq, dk=dk, dv=dv)

    def _joint_kv(self, B, Lp, dev, save):
        """Joint K/V buffers [nL, B, Lp, hd] for one training forward.  The engine owns one zeroed set
        (the Lp - L pad rows stay zero for the GEMM path; rows < L are rewritten by every forward) and
        lends it to the forward whose saved state (``save``) holds the token; while that state is alive
        (its backward has not run and its graph still exists) another forward gets fresh buffers, so
        interleaved forwards never share saved K/V."""
        holder = self._jkv_holder() if self._jkv_holder is not None else None
        if holder is not None:
            k = torch.zeros(self.d.nL, B, Lp, self.d.hd, device=dev, dtype=BF16)
            return k, torch.zeros_like(k)
        key = ("jkv", B, Lp, dev)
        kv = self._ws.get(key)
        if kv is None:
            self._ws = {k: v for k, v in self._ws.items() if k[0] != "jkv"}  # one shape at a time
            k = torch.zeros(self.d.nL, B, Lp, self.d.hd, device=dev, dtype=BF16)
            kv = self._ws[key] = (k, torch.zeros_like(k))
        tok = _Token()
        save["_jkv_token"] = tok
        self._jkv_holder = weakref.ref(tok)
        return kv

    def _pre_attn_train(self, g, l, X, pos, st, Qj, Kj, Vj, dev):
        """One group's input RMSNorm + q|k|v projection + RoPE + joint Q / K / V scatter of joint layer l
        (paligemma/modules.py:7-21, mixture.py:162-215, joint_model.py:170-257)."""
        d = self.d
        L, Lp, nh, hd = d.L, d.Lp, d.nh, d.hd
        B = Qj.shape[0]
        p = f"{g.prefix}{l}."
        x = X[g.name]
        M = x.shape[0]
        h = torch.empty_like(x)
        r = torch.empty(M, device=dev, dtype=F32)
        ops.rmsnorm(x, self.w(p + "input_layernorm.weight"), h, r, d.rms_eps)
        # q|k|v projection + RoPE + joint scatter: one 8-phase GEMM whose epilogue rotates and writes
        # Q / K / V (N1: no [M, 2560] qkv tensor, no split launch); rows too few for the 8-phase
        # kernel (the action expert's 320) take GEMM + qkv_rope_split (same bits)
        if not (self.fuse_qkv_rope and ops.gemm_qkv_rope(h, self.qkv_w(p), pos[g.pos_key], self.rope(g.theta),
                                                         Qj, Kj, Vj, g.T, nh, hd, L, g.off, Lp, g.off)):
            W = (nh + 2) * hd
            qkv = torch.empty(M, W, device=dev, dtype=BF16)
            ops.linear(h, self.qkv_w(p), qkv)
            ops.qkv_rope_split(qkv, pos[g.pos_key], self.rope(g.theta), Qj, Kj, Vj, B, g.T, nh, 1, hd, L,
                               g.off, Lp, g.off)
        st["g"][g.name] = {"x": x, "h": h, "r": r}

    def _post_attn_train(self, g, l, X, gs, Os, dev):
        """One group's o_proj (+ residual), post-attention RMSNorm and GeGLU MLP (+ residual) of joint layer l
        (mixture.py:216-242, paligemma/modules.py:86-95), activations saved in gs for the backward."""
        d = self.d
        p = f"{g.prefix}{l}."
        x = X[g.name]
        M = x.shape[0]
        O = Os[g.name]
        xm = torch.empty_like(x)
        ops.linear(O, self.w(p + "self_attn.o_proj.weight"), xm, resid=x)
        h2 = torch.empty_like(x)
        r2 = torch.empty(M, device=dev, dtype=F32)
        ops.rmsnorm(xm, self.w(p + "post_attention_layernorm.weight"), h2, r2, d.rms_eps)
        gu = torch.empty(M, 2 * g.inter, device=dev, dtype=BF16)
        hm = torch.empty(M, g.inter, device=dev, dtype=BF16)
        ops.linear(h2, self.gu_w(p), hm, epi=PZ_EPI_GEGLU, aux=gu)
        xn = torch.empty_like(x)
        ops.linear(hm, self.w(p + "mlp.down_proj.weight"), xn, resid=xm)
        gs.update(O=O, xm=xm, h2=h2, r2=r2, gu=gu, hm=hm, skip=False)
        X[g.name] = xn

    def _joint_layers_train(self, groups, X, pos, cnt, B, save):
        """joint_model.py:24-304 x nL for the training pass (all mixtures active)."""
        d = self.d
        dev = X[groups[0].name].device
        L, Lp, nh, hd = d.L, d.Lp, d.nh, d.hd
        S = None
        layers = []
        Kall, Vall = self._joint_kv(B, Lp, dev, save)
        # the action-expert group's pre- and post-attention work on the second stream, concurrent with the vlm
        # group's; the streams meet at the joint attention (as in _joint_layers_backward)
        main = torch.cuda.current_stream(dev)
        side = None
        if self.expert_stream and self.expert_stream_fwd and len(groups) > 1 and dev.type == "cuda":
            side = self._side_stream(dev)
            side.wait_stream(main)
            for t in X.values():
                if t is not None:
                    t.record_stream(side)
        for l in range(d.nL):
            last = l == d.nL - 1
            Qj = torch.empty(B, L, nh * hd, device=dev, dtype=BF16)
            if side is not None:
                Qj.record_stream(side)
            Kj, Vj = Kall[l], Vall[l]
            st = {"Q": Qj, "K": Kj, "V": Vj, "g": {}}
            for g in groups:
                with self._on(side, g):
                    self._pre_attn_train(g, l, X, pos, st, Qj, Kj, Vj, dev)
            if side is not None:
                main.wait_stream(side)  # every group's Q / K / V rows before the joint attention
            Os = {g.name: torch.empty(B * g.T, nh * hd, device=dev, dtype=BF16) for g in groups}
            if self.joint_flash and not isinstance(cnt, GeneralMask):
                # fused joint attention (joint_model.py:259-292): soft-cap, block mask from cnt, O rows
                # scattered into each mixture's o_proj input; one fp32 log-sum-exp per (token, head) row
                lse = torch.empty(B, L * nh, device=dev, dtype=F32)
                ops.flash_fwd(self._joint_flash(groups, Qj, Kj, Vj, Os, lse, cnt, B, L))
                st["lse"], st["O"] = lse, Os
            elif self.joint_probs and not isinstance(cnt, GeneralMask) and L <= 320 and hd == 256:
                # (pz_flash_fwd_probs keeps a whole score row in registers: <= 320 keys; C5's 839 take the
                # GEMM path)
                # one fused kernel: S = Q K^T with K staged in LDS, soft-cap + block mask + exact row softmax
                # in registers, P / tanh(cap) exported in bf16 for the GEMM-path backward, O = P V
                Pm = torch.empty(B, L * nh, Lp, device=dev, dtype=BF16)
                tc = torch.empty(B, L * nh, Lp, device=dev, dtype=BF16)
                ops.flash_fwd_probs(self._joint_flash(groups, Qj, Kj, Vj, Os, None, cnt, B, L), Pm, tc, Lp)
                st["P"], st["tc"], st["O"] = Pm, tc, Os
            else:
                # S = Q K^T per sample (MQA heads stacked as rows), soft-cap + block-mask softmax, O = P V
                if S is None:
                    S = torch.empty(B, L * nh, Lp, device=dev, dtype=F32)
                ops.gemm(L * nh, L, hd, Qj, hd, True, Kj, hd, True, S, Lp, batch=B, sA=(L * nh * hd, 0),
                         sB=(Lp * hd, 0), sC=(L * nh * Lp, 0))
                Pm = torch.empty(B, L * nh, Lp, device=dev, dtype=BF16)
                tc = torch.empty(B, L * nh, Lp, device=dev, dtype=BF16)
                ops.attn_softmax(S, Lp, Pm, Lp, B * L * nh, L, 1.0 / math.sqrt(hd), cap=50.0, tcap=tc,
                                 rows_per_batch=L * nh, heads=nh, qoff=0, **_mask_kw(d, cnt, "full"))
                st["P"], st["tc"] = Pm, tc
                for g in groups:
                    if not (last and g.skip_last):
                        ops.gemm(g.T * nh, hd, Lp, Pm[:, g.off * nh:], Lp, True, Vj, hd, False, Os[g.name], hd, batch=B,
                                 sA=(L * nh * Lp, 0), sB=(Lp * hd, 0), sC=(g.T * nh * hd, 0))
                st["O"] = Os
            if side is not None:
                side.wait_stream(main)  # the attention outputs
                for t in Os.values():
                    t.record_stream(side)
            for g in groups:
                gs = st["g"][g.name]
                if last and g.skip_last:
                    X[g.name] = None
                    gs["skip"] = True
                    continue
                with self._on(side, g):
                    self._post_attn_train(g, l, X, gs, Os, dev)
            layers.append(st)
            self._chk(f"joint fwd layer {l}", Q=Qj, K=Kj, V=Vj, O=Os, P=st.get("P"), tc=st.get("tc"), X=X)
        if side is not None:  # the expert output and its saved activations are read on the main stream later
            main.wait_stream(side)
            for t in X.values():
                if t is not None:
                    t.record_stream(main)
            for st in layers:
                for g in groups:
                    if g.name != "vlm":
                        for t in st["g"][g.name].values():
                            if isinstance(t, torch.Tensor):
                                t.record_stream(main)
        save["joint"] = layers
        return X

    def _mlp_oproj_backward(self, g, gs, p, dX, dO, dXm, beta, rpp, nh, hd, dev):
        """One group's GeGLU MLP + post-attention RMSNorm + o_proj backward of a joint layer
        (paligemma/modules.py:86-95, mixture.py:216-242): dX[g] -> dO[g] (the attention output gradient)
        and dXm[g] (the residual gradient into the input RMSNorm backward)."""
        dx = dX[g.name]
        M = dx.shape[0]
        part = torch.empty((M + rpp - 1) // rpp, g.hid, device=dev, dtype=F32)
        # MLP
        # dgrad through down_proj with the GeGLU derivative fused into its epilogue:
        # gu (saved g|u) <- d(gate|up) in place; hm (saved GeGLU output) feeds the down_proj wgrad
        gu = gs["gu"]
        if self.split_dgeglu:  # plain dgrad GEMM, then the HBM-bound GeGLU backward in place on gu
            dh = torch.empty(M, g.inter, device=dev, dtype=BF16)
            ops.linear_dgrad(dx, self.w(p + "mlp.down_proj.weight"), dh)
            ops.geglu_bwd(dh, gu, gu, None, M, g.inter)
            del dh
        else:
            ops.linear_dgrad(dx, self.w(p + "mlp.down_proj.weight"), gu, epi=PZ_EPI_DGEGLU, aux=gu)
        if self.rg(p + "mlp.down_proj.weight"):
            ops.linear_wgrad(dx, gs["hm"], self.gw(p + "mlp.down_proj.weight"), beta=beta)
        gs["hm"] = None
        if self.rg(p + "mlp.gate_proj.weight") and self.rg(p + "mlp.up_proj.weight"):
            ops.linear_wgrad(gu, gs["h2"], self.ar.grad_span(p + "mlp.gate_proj.weight", p + "mlp.up_proj.weight"),
                             beta=beta)
        dh2 = torch.empty(M, g.hid, device=dev, dtype=BF16)
        ops.linear_dgrad(gu, self.gu_w(p), dh2)
        dxm = torch.empty_like(dx)
        ops.rmsnorm_bwd(dh2, gs["xm"], self.w(p + "post_attention_layernorm.weight"), gs["r2"], dxm, dres=dx,
                        dw_part=part)
        self._norm_grads(p + "post_attention_layernorm.", part, None, beta)
        # o_proj
        if self.rg(p + "self_attn.o_proj.weight"):
            ops.linear_wgrad(dxm, gs["O"], self.gw(p + "self_attn.o_proj.weight"), beta=beta)
        o = torch.empty(M, nh * hd, device=dev, dtype=BF16)
        ops.linear_dgrad(dxm, self.w(p + "self_attn.o_proj.weight"), o)
        dO[g.name] = o
        dXm[g.name] = dxm

    def _qkv_backward(self, g, gs, p, dQ, dK, dV, dX, dXm, pos, B, L, Lp, beta, rpp, nh, hd, dev):
        """One group's q|k|v projection + input RMSNorm backward of a joint layer (mixture.py:162-215,
        joint_model.py:170-257 + inverse RoPE): dQ / dK / dV rows of the group -> dX[g]."""
        x = gs["x"]
        M = x.shape[0]
        W = (nh + 2) * hd
        dqkv = torch.empty(M, W, device=dev, dtype=BF16)
        ops.qkv_rope_split_bwd(None if gs.get("skip") else dQ, dK, dV, pos[g.pos_key], self.rope(g.theta), dqkv,
                               B, g.T, nh, 1, hd, L, g.off, Lp, g.off)
        names = [p + f"self_attn.{k}_proj.weight" for k in "qkv"]
        rgs = [self.rg(n) for n in names]
        if gs.get("skip"):
            # last vlm layer: its query rows feed nothing (the post-attention block is skipped), so dQ = 0 exactly --
            # the q_proj gradient is zero (written as such, not computed: pizero.py:231's frozen v_proj and the zero
            # q_proj grad) and only the k|v columns enter the weight / input gradients
            if rgs[0] and not beta:
                self.gw(names[0]).zero_()
            for n, rgk, c0, c1 in zip(names[1:], rgs[1:], (nh * hd, (nh + 1) * hd), ((nh + 1) * hd, W)):
                if rgk:
                    ops.linear_wgrad(dqkv[:, c0:c1], gs["h"], self.gw(n), beta=beta)
            dh = torch.empty(M, g.hid, device=dev, dtype=BF16)
            ops.linear_dgrad(dqkv[:, nh * hd:], self.ar.span(names[1], names[2]), dh)
        else:
            if all(rgs):
                ops.linear_wgrad(dqkv, gs["h"], self.ar.grad_span(names[0], names[2]), beta=beta)
            elif rgs[0] and rgs[1]:  # e.g. last-layer vlm v_proj frozen (pizero.py:231)
                ops.linear_wgrad(dqkv[:, : (nh + 1) * hd], gs["h"], self.ar.grad_span(names[0], names[1]),
                                 beta=beta)
            else:
                for n, rgk, c0, c1 in zip(names, rgs, (0, nh * hd, (nh + 1) * hd), (nh * hd, (nh + 1) * hd, W)):
                    if rgk:
                        ops.linear_wgrad(dqkv[:, c0:c1], gs["h"], self.gw(n), beta=beta)
            dh = torch.empty(M, g.hid, device=dev, dtype=BF16)
            ops.linear_dgrad(dqkv, self.qkv_w(p), dh)
        part = torch.empty((M + rpp - 1) // rpp, g.hid, device=dev, dtype=F32)
        dxn = torch.empty(M, g.hid, device=dev, dtype=BF16)
        ops.rmsnorm_bwd(dh, x, self.w(p + "input_layernorm.weight"), gs["r"], dxn, dres=dXm.get(g.name),
                        dw_part=part)
        self._norm_grads(p + "input_layernorm.", part, None, beta)
        dX[g.name] = dxn

    def _joint_layers_backward(self, groups, dX, pos, cnt, B, sv, beta):
        d = self.d
        L, Lp, nh, hd = d.L, d.Lp, d.nh, d.hd
        dev = next(v for v in dX.values() if v is not None).device
        delta = dP = dS = None
        rpp = ops.rows_per_part()
        # the non-vlm group (action expert, 320 rows at micro-batch 64) runs its MLP / o_proj / q|k|v backward
        # on a second stream while the vlm group's run on the main stream; they meet at the joint attention
        # backward (events both ways).  Tensors one stream allocated and the other reads are record_stream'ed,
        # so the caching allocator never hands their memory out while the other stream may still read it.
        main = torch.cuda.current_stream(dev)
        side = None
        if self.expert_stream and len(groups) > 1 and dev.type == "cuda":
            side = self._side_stream(dev)
            side.wait_stream(main)
            for st in sv["joint"]:
                for g in groups:
                    if g.name != "vlm":
                        for t in st["g"][g.name].values():
                            if isinstance(t, torch.Tensor):
                                t.record_stream(side)
            for t in dX.values():
                if t is not None:
                    t.record_stream(side)
        for l in reversed(range(d.nL)):
            st = sv["joint"][l]
            dQ = torch.empty(B, L, nh * hd, device=dev, dtype=BF16)
            dK = torch.empty(B, Lp, hd, device=dev, dtype=BF16)
            dV = torch.empty(B, Lp, hd, device=dev, dtype=BF16)
            dO = {}
            dXm = {}
            any_skip = False
            for g in groups:
                gs = st["g"][g.name]
                p = f"{g.prefix}{l}."
                if gs.get("skip"):
                    any_skip = True
                    continue
                with self._on(side, g):
                    self._mlp_oproj_backward(g, gs, p, dX, dO, dXm, beta, rpp, nh, hd, dev)
                if side is not None and g.name != "vlm":
                    dO[g.name].record_stream(main)
            if side is not None:
                main.wait_stream(side)  # the expert dO for the joint attention backward
            if "lse" in st:
                # fused attention backward (skipped mixtures' outputs reach nothing: dO = 0)
                for g in groups:
                    if g.name not in dO:
                        dO[g.name] = torch.zeros(B * g.T, nh * hd, device=dev, dtype=BF16)
                if delta is None:
                    delta = torch.empty(B, L * nh, device=dev, dtype=F32)
                ops.flash_bwd(self._joint_flash(groups, st["Q"], st["K"], st["V"], st["O"], st["lse"], cnt, B, L,
                                                dO=dO, delta=delta, dq=dQ, dk=dK, dv=dV))
            else:
                Pm, tc, Qj, Kj, Vj = st["P"], st["tc"], st["Q"], st["K"], st["V"]
                dq_done = False
                if self.joint_ds and not isinstance(cnt, GeneralMask) and L <= 320 and hd == 256:
                    # dS in one kernel: dP = dO V^T in registers, delta and the soft-cap/softmax backward
                    # from the exported P / tanh(cap) (no fp32 dP tensor), then dQ = dS K in the same launch;
                    # a mixture without dO adds 0
                    if dS is None:
                        dS = torch.empty(B, L * nh, Lp, device=dev, dtype=BF16)
                    ops.flash_bwd_ds(self._joint_flash(groups, Qj, Kj, Vj, st["O"], None, cnt, B, L, dO=dO,
                                                       dq=dQ if self.joint_ds_dq else None), Pm, tc, dS, Lp)
                    dq_done = self.joint_ds_dq
                else:
                    if dP is None:
                        dP = torch.empty(B, L * nh, Lp, device=dev, dtype=F32)
                    if dS is None:
                        dS = torch.empty(B, L * nh, Lp, device=dev, dtype=BF16)
                    if any_skip:
                        dP.zero_()
                    for g in groups:
                        if g.name not in dO:
                            continue
                        ops.gemm(g.T * nh, L, hd, dO[g.name], hd, True, Vj, hd, True, dP[:, g.off * nh:], Lp,
                                 batch=B, sA=(g.T * nh * hd, 0), sB=(Lp * hd, 0), sC=(L * nh * Lp, 0))
                    ops.attn_softmax_bwd(Pm, dP, Lp, tc, dS, Lp, B * L * nh, L, 1.0 / math.sqrt(hd), 50.0)
                # dQ = dS K ; dK = dS^T Q ; dV = sum_g P_g^T dO_g
                if not dq_done:
                    ops.gemm(L * nh, hd, Lp, dS, Lp, True, Kj, hd, False, dQ, hd, batch=B, sA=(L * nh * Lp, 0),
                             sB=(Lp * hd, 0), sC=(L * nh * hd, 0))
                ops.gemm(Lp, hd, L * nh, dS, Lp, False, Qj, hd, False, dK, hd, batch=B, sA=(L * nh * Lp, 0),
                         sB=(L * nh * hd, 0), sC=(Lp * hd, 0))
                first = True
                # the shortest mixture first (the action expert's 5 rows x heads: its launch then writes dV
                # instead of reading + writing it, and the long vlm launch accumulates in its epilogue)
                for g in sorted(groups, key=lambda g: g.T):
                    if g.name not in dO:
                        continue
                    ops.gemm(Lp, hd, g.T * nh, Pm[:, g.off * nh:], Lp, False, dO[g.name], hd, False, dV, hd, batch=B,
                             sA=(L * nh * Lp, 0), sB=(g.T * nh * hd, 0), sC=(Lp * hd, 0), beta=not first)
                    first = False
                if first:
                    dV.zero_()
            if side is not None:  # dQ / dK / dV of the joint attention backward feed the expert's q|k|v backward
                side.wait_stream(main)
                for t in (dQ, dK, dV):
                    t.record_stream(side)
            for g in groups:
                with self._on(side, g):
                    self._qkv_backward(g, st["g"][g.name], f"{g.prefix}{l}.", dQ, dK, dV, dX, dXm, pos, B, L, Lp, beta,
                                       rpp, nh, hd, dev)
            # the layer's expert gradients were produced on the side stream: the reducer's communication stream waits
            # for both streams before it reads them (the compute streams keep running; no main <- side join per layer)
            self._chk(f"joint bwd layer {l}", dO=dO, dS=dS, dQ=dQ, dK=dK, dV=dV, dX=dX)
            self._notify("joint", l, (side,) if side is not None else ())
        if side is not None:
            main.wait_stream(side)
            for t in dX.values():
                if t is not None:
                    t.record_stream(main)
        sv.pop("_jkv_token", None)  # the joint K/V buffers are free for the next forward
        return dX

    # ============================================================ training ==
    def train_forward(self, ids, pix, cnt, pos, proprios, actions, t, x0, save):
        """pizero.py:607-661: returns fp32 loss [1]; ``save`` collects activations."""
        d = self.d
        dev = pix.device
        B = ids.shape[0]
        tied = self.m._tied
        sv_v = {}
        img = self.siglip_forward(pix, sv_v)
        Xv = self.embed_prefix(ids, img)
        prop = proprios.reshape(B * d.C, d.Pd).to(BF16)
        pe = torch.empty(B * d.C, d.aH, device=dev, dtype=BF16)
        ops.small_linear(prop, self.w("proprio_encoder.weight"), pe, bias=self.w("proprio_encoder.bias"))
        psi = torch.empty(B * d.H, d.A, device=dev, dtype=BF16)
        ops.flow_psi(x0, actions, t, psi, d.sig_min)
        e3 = self.action_embed(psi, t, save)
        sa = math.sqrt(d.aH)
        if tied:
            Xe = torch.empty(B * (d.C + d.H), d.aH, device=dev, dtype=BF16)
            T = d.C + d.H
            ops.copy_rows(pe, d.aH, d.C * d.aH, Xe, d.aH, T * d.aH, B, d.C, d.aH, scale=sa)
            ops.copy_rows(e3, d.aH, d.H * d.aH, Xe[d.C:], d.aH, T * d.aH, B, d.H, d.aH, scale=sa)
            X = {"vlm": Xv, "expert": Xe}
        else:
            Xp = torch.empty(B * d.C, d.aH, device=dev, dtype=BF16)
            Xa = torch.empty(B * d.H, d.aH, device=dev, dtype=BF16)
            ops.copy_rows(pe, d.aH, 0, Xp, d.aH, 0, 1, B * d.C, d.aH, scale=sa)
            ops.copy_rows(e3, d.aH, 0, Xa, d.aH, 0, 1, B * d.H, d.aH, scale=sa)
            X = {"vlm": Xv, "proprio": Xp, "action": Xa}
        groups = self.groups(tied)
        X = self._joint_layers_train(groups, X, pos, cnt, B, save)
        ag = "expert" if tied else "action"
        aoff = d.C if tied else 0
        Tg = d.C + d.H if tied else d.H
        Xl = X[ag]
        ya = torch.empty_like(Xl)
        ra = torch.empty(Xl.shape[0], device=dev, dtype=F32)
        ops.rmsnorm(Xl, self.w("joint_model.mixtures.action.norm.weight"), ya, ra, d.rms_eps)
        v = torch.empty(B * Tg, 8, device=dev, dtype=BF16)  # columns 0..A-1 written and read (8: 16-B rows)
        ops.small_linear(ya, self.w("action_decoder.weight"), v, bias=self.w("action_decoder.bias"))
        loss = torch.empty(1, device=dev, dtype=F32)
        ops.flow_loss(v[aoff:], 8, Tg * 8, x0, actions, loss, None, None, B, d.H, d.A, d.sig_min)
        save.update(sv_v=sv_v, ids=ids, cnt=cnt, pos=pos, B=B, prop=prop, pe=pe, tied=tied, Xl=Xl, ya=ya, ra=ra,
                    x0=x0, x1=actions, v=v, ag=ag, aoff=aoff, Tg=Tg, groups=groups)
        self._chk("train fwd head (action norm, decoder, flow loss)", embed=Xv, ya=ya, v=v, loss=loss)
        return loss

    def train_backward(self, sv, grad_loss, beta):
        """Backward of train_forward; grad_loss: device fp32 [1] (d loss)."""
        d = self.d
        B = sv["B"]
        dev = sv["v"].device
        Tg, aoff = sv["Tg"], sv["aoff"]
        ws = self.colsum_ws(2 * d.aH)
        rpp = ops.rows_per_part()
        # loss + decoder
        dv = torch.zeros(B * Tg, 8, device=dev, dtype=BF16)
        tmp = torch.empty(1, device=dev, dtype=F32)
        ops.flow_loss(sv["v"][aoff:], 8, Tg * 8, sv["x0"], sv["x1"], tmp, dv[aoff:], grad_loss, B, d.H, d.A, d.sig_min)
        R = B * Tg
        if self.rg("action_decoder.weight"):
            ops.small_gemm(d.A, d.aH, R, dv, 1, 8, sv["ya"], d.aH, 1, self.gw("action_decoder.weight"), d.aH, beta=beta)
        if self.rg("action_decoder.bias"):
            ops.colsum(dv[:, : d.A], self.gw("action_decoder.bias"), ws, beta=beta)
        dya = torch.empty(R, d.aH, device=dev, dtype=BF16)
        ops.small_gemm(R, d.aH, d.A, dv, 8, 1, self.w("action_decoder.weight"), d.aH, 1, dya, d.aH)
        dXl = torch.empty_like(dya)
        part = torch.empty((R + rpp - 1) // rpp, d.aH, device=dev, dtype=F32)
        ops.rmsnorm_bwd(dya, sv["Xl"], self.w("joint_model.mixtures.action.norm.weight"), sv["ra"], dXl, dw_part=part)
        self._norm_grads("joint_model.mixtures.action.norm.", part, None, beta)
        self._chk("train bwd head", dv=dv, dya=dya, dXl=dXl)
        groups = sv["groups"]
        dX = {g.name: None for g in groups}
        dX[sv["ag"]] = dXl
        dX = self._joint_layers_backward(groups, dX, sv["pos"], sv["cnt"], B, sv, beta)
        # expert embeddings (joint_model.py:355 scale) -> encoders
        sa = math.sqrt(d.aH)
        dpe = torch.empty(B * d.C, d.aH, device=dev, dtype=BF16)
        de3 = torch.empty(B * d.H, d.aH, device=dev, dtype=BF16)
        if sv["tied"]:
            T = d.C + d.H
            ops.copy_rows(dX["expert"], d.aH, T * d.aH, dpe, d.aH, d.C * d.aH, B, d.C, d.aH, scale=sa)
            ops.copy_rows(dX["expert"][d.C:], d.aH, T * d.aH, de3, d.aH, d.H * d.aH, B, d.H, d.aH, scale=sa)
        else:
            ops.copy_rows(dX["proprio"], d.aH, 0, dpe, d.aH, 0, 1, B * d.C, d.aH, scale=sa)
            ops.copy_rows(dX["action"], d.aH, 0, de3, d.aH, 0, 1, B * d.H, d.aH, scale=sa)
        if self.rg("proprio_encoder.weight"):
            ops.small_gemm(d.aH, d.Pd, B * d.C, dpe, 1, d.aH, sv["prop"], d.Pd, 1, self.gw("proprio_encoder.weight"),
                           d.Pd, beta=beta)
        if self.rg("proprio_encoder.bias"):
            ops.colsum(dpe, self.gw("proprio_encoder.bias"), ws, beta=beta)
        ae = "action_encoder."
        if self.rg(ae + "linear_3.weight"):
            ops.linear_wgrad(de3, sv["ae_e2"], self.gw(ae + "linear_3.weight"), beta=beta)
        if self.rg(ae + "linear_3.bias"):
            ops.colsum(de3, self.gw(ae + "linear_3.bias"), ws, beta=beta)
        de2 = torch.empty_like(de3)
        ops.linear_dgrad(de3, self.w(ae + "linear_3.weight"), de2)
        ops.act_bwd(de2, sv["ae_pre"], de2, None, PZ_EPI_SILU)
        if self.rg(ae + "linear_2.weight"):
            ops.linear_wgrad(de2, sv["ae_cat"], self.gw(ae + "linear_2.weight"), beta=beta)
        if self.rg(ae + "linear_2.bias"):
            ops.colsum(de2, self.gw(ae + "linear_2.bias"), ws, beta=beta)
        dcat = torch.empty(B * d.H, 2 * d.aH, device=dev, dtype=BF16)
        ops.linear_dgrad(de2, self.w(ae + "linear_2.weight"), dcat)
        de1 = torch.empty_like(de3)
        ops.split_time_grad(dcat, de1, B * d.H, d.aH)
        if self.rg(ae + "linear_1.weight"):
            ops.small_gemm(d.aH, d.A, B * d.H, de1, 1, d.aH, sv["ae_psi"], d.A, 1, self.gw(ae + "linear_1.weight"), d.A,
                           beta=beta)
        if self.rg(ae + "linear_1.bias"):
            ops.colsum(de1, self.gw(ae + "linear_1.bias"), ws, beta=beta)
        self._notify("encoders", -1)
        # VLM prefix -> projector -> SigLIP
        if self.m._vlm_needs_grad():
            dimg = torch.empty(B * d.n_img, d.gH, device=dev, dtype=BF16)
            ops.embed_merge_bwd(sv["ids"], dX["vlm"], dimg, d.n_img, d.image_token, 1.0)
            self._chk("train bwd embed-merge", dimg=dimg)
            self.siglip_backward(sv["sv_v"], dimg, beta)
        self._chk("train bwd end (gradient arena)", grad=self.ar.grad)
        if self.post_backward is not None:
            self.post_backward()

    # ================================================== JointModel alone ==
    def joint_train(self, embeds, pos, cnt, dout, beta=False):
        """JointModel.forward + backward alone (joint_model.py:328-383) on given embeddings -- the
        harness of config C5 (3 images + chunk 50, which the reference composes at this level since
        its PiZero takes one image per sample).  embeds: {"vlm": [B, P, gH], "proprio": [B, C, aH],
        "action": [B, H, aH]} bf16 (scaled by sqrt(hidden) here, joint_model.py:348-355); dout: d(loss)
        wrt the final-normed action hidden states [B, H, aH].  Accumulates parameter gradients into
        the gradient arena and returns (action hidden [B, H, aH] bf16, {name: d embeds})."""
        d = self.d
        Ev, Ep, Ea = embeds["vlm"], embeds["proprio"], embeds["action"]
        B = Ev.shape[0]
        dev = Ev.device
        if not self.m._tied:
            raise NotImplementedError("joint_train expects tie_action_proprio_weights() (pizero.py:262-264)")
        Xv = torch.empty(B * d.P, d.gH, device=dev, dtype=BF16)
        ops.copy_rows(Ev.reshape(B * d.P, d.gH), d.gH, 0, Xv, d.gH, 0, 1, B * d.P, d.gH, scale=math.sqrt(d.gH))
        T = d.C + d.H
        sa = math.sqrt(d.aH)
        Xe = torch.empty(B * T, d.aH, device=dev, dtype=BF16)
        ops.copy_rows(Ep.reshape(B * d.C, d.aH), d.aH, d.C * d.aH, Xe, d.aH, T * d.aH, B, d.C, d.aH, scale=sa)
        ops.copy_rows(Ea.reshape(B * d.H, d.aH), d.aH, d.H * d.aH, Xe[d.C:], d.aH, T * d.aH, B, d.H, d.aH, scale=sa)
        groups = self.groups(True)
        save = {}
        X = self._joint_layers_train(groups, {"vlm": Xv, "expert": Xe}, pos, cnt, B, save)
        Xl = X["expert"]
        ya = torch.empty_like(Xl)
        ra = torch.empty(Xl.shape[0], device=dev, dtype=F32)
        ops.rmsnorm(Xl, self.w("joint_model.mixtures.action.norm.weight"), ya, ra, d.rms_eps)
        dya = torch.zeros_like(ya)  # proprio rows are not outputs (joint_model.py:375-380 skip list)
        ops.copy_rows(dout.reshape(B * d.H, d.aH).to(BF16), d.aH, d.H * d.aH, dya[d.C:], d.aH, T * d.aH, B, d.H, d.aH)
        rpp = ops.rows_per_part()
        dXl = torch.empty_like(dya)
        part = torch.empty((B * T + rpp - 1) // rpp, d.aH, device=dev, dtype=F32)
        ops.rmsnorm_bwd(dya, Xl, self.w("joint_model.mixtures.action.norm.weight"), ra, dXl, dw_part=part)
        self._norm_grads("joint_model.mixtures.action.norm.", part, None, beta)
        dX = self._joint_layers_backward(groups, {"vlm": None, "expert": dXl}, pos, cnt, B, save, beta)
        dEv = torch.empty(B, d.P, d.gH, device=dev, dtype=BF16)
        ops.copy_rows(dX["vlm"], d.gH, 0, dEv.view(B * d.P, d.gH), d.gH, 0, 1, B * d.P, d.gH, scale=math.sqrt(d.gH))
        dEp = torch.empty(B, d.C, d.aH, device=dev, dtype=BF16)
        dEa = torch.empty(B, d.H, d.aH, device=dev, dtype=BF16)
        ops.copy_rows(dX["expert"], d.aH, T * d.aH, dEp.view(B * d.C, d.aH), d.aH, d.C * d.aH, B, d.C, d.aH, scale=sa)
        ops.copy_rows(dX["expert"][d.C:], d.aH, T * d.aH, dEa.view(B * d.H, d.aH), d.aH, d.H * d.aH, B, d.H, d.aH,
                      scale=sa)
        out = torch.empty(B, d.H, d.aH, device=dev, dtype=BF16)
        ops.copy_rows(ya[d.C:], d.aH, T * d.aH, out.view(B * d.H, d.aH), d.aH, d.H * d.aH, B, d.H, d.aH)
        return out, {"vlm": dEv, "proprio": dEp, "action": dEa}

    # ============================================================ inference ==
    def decode_attn_ok(self):
        """pz_decode_attn for the denoise attention (head_dim 256, up to 1024 query rows per sample in 32-row
        tiles: C4's 4 tokens x 8 heads = one tile, C5's 50 x 8 = 13 tiles with 2 key chunks per workgroup --
        measured 23.5 vs 24.3 ms per C5 chunk against the key-split flash kernel); PZ_DECODE_ATTN=0 uses
        the flash kernel + combine"""
        d = self.d
        return d.hd == 256 and os.environ.get("PZ_DECODE_ATTN", "1") != "0" and d.H * d.nh <= 1024

    def _qkv_w_f8(self, p):
        """(q|k|v weights, fp8 scale): the e4m3 codes and their scale when prepare_fp8() holds them for layer p,
        else (bf16 weights, None)"""
        f = self.f8.get(p + "self_attn.q_proj.weight") if self.f8 else None
        return (self.qkv_w(p), None) if f is None else (f[0], f[1])

    def few_rows(self, M, K):
        """row counts the few-row GEMM kernels take with the RMSNorm fused (pz_gemm skinny paths:
        M <= 16 with K % 32 == 0, 16 < M <= 64 with K % 64 == 0)"""
        return (M <= 16 and K % 32 == 0) or (M <= 64 and K % 64 == 0)

    def gemv_ok(self, M, K):
        """few-row GEMV kernels (pz_gemv.hip): M <= 8 rows, K % 512 == 0 (PZ_GEMV=0 disables)"""
        return M <= 8 and K % 512 == 0 and os.environ.get("PZ_GEMV", "1") != "0"

    def prefill(self, ids, pix, cnt, vpos, ppos, proprios, kcache, vcache):
        """pizero.py:430-451: SigLIP + prefix pass over {vlm, proprio}; writes post-RoPE K/V caches."""
        d = self.d
        dev = pix.device
        B = ids.shape[0]
        nh, hd, Lp = d.nh, d.hd, d.Lp
        L1 = d.P + d.C
        img = self.siglip_forward(pix, None)
        Xv = self.embed_prefix(ids, img)
        prop = proprios.reshape(B * d.C, d.Pd).to(BF16)
        pe = torch.empty(B * d.C, d.aH, device=dev, dtype=BF16)
        ops.small_linear(prop, self.w("proprio_encoder.weight"), pe, bias=self.w("proprio_encoder.bias"))
        Xp = torch.empty(B * d.C, d.aH, device=dev, dtype=BF16)
        ops.copy_rows(pe, d.aH, 0, Xp, d.aH, 0, 1, B * d.C, d.aH, scale=math.sqrt(d.aH))
        tied = self.m._tied
        pprefix = "joint_model.mixtures." + ("action" if tied else "proprio") + ".layers."
        groups = [Group("vlm", "joint_model.mixtures.vlm.layers.", ["vlm"], d.P, 0, d.gH, d.gI, d.g_theta, True, "vlm"),
                  Group("proprio", pprefix, ["proprio"], d.C, d.P, d.aH, d.aI, d.p_theta if not tied else d.a_theta,
                        True, "proprio")]
        X = {"vlm": Xv, "proprio": Xp}
        pos = {"vlm": vpos, "proprio": ppos}
        Q = torch.empty(B, L1, nh * hd, device=dev, dtype=BF16)
        S = Pm = None
        for l in range(d.nL):
            last = l == d.nL - 1
            Kj, Vj = kcache[l], vcache[l]
            hs = {}
            for g in groups:
                p = f"{g.prefix}{l}."
                x = X[g.name]
                M = x.shape[0]
                if self.gemv_ok(M, x.shape[1]):  # few rows (the proprio token): one fused launch
                    if last:
                        self._kv_only_gemv(x, p, pos[g.pos_key], g, Kj, Vj, L1, Lp)
                    else:
                        ops.gemv_qkv_rope(x, self.qkv_w(p), pos[g.pos_key], self.rope(g.theta), Q, Kj, Vj, g.T, nh,
                                          hd, L1, g.off, Lp, g.off,
                                          norm=(self.w(p + "input_layernorm.weight"), d.rms_eps))
                    continue
                if not last and self.w8a8_in(p + "self_attn.q_proj.weight", M, x.shape[1]):
                    # fp8 (C5): input RMSNorm straight to e4m3 codes, q|k|v W8A8 on the fp8 MFMA, RoPE + scatter
                    qkv = torch.empty(M, (nh + 2) * hd, device=dev, dtype=BF16)
                    self.lin(self.norm_codes(x, self.w(p + "input_layernorm.weight"), d.rms_eps),
                             p + "self_attn.q_proj.weight", self.qkv_w(p), qkv)
                    ops.qkv_rope_split(qkv, pos[g.pos_key], self.rope(g.theta), Q, Kj, Vj, B, g.T, nh, 1, hd, L1,
                                       g.off, Lp, g.off)
                    continue
                h = torch.empty_like(x)
                ops.rmsnorm(x, self.w(p + "input_layernorm.weight"), h, None, d.rms_eps)
                if last:  # only K/V are consumed downstream (pizero.py:451, skipped post-attn)
                    kv = torch.empty(M, 2 * hd, device=dev, dtype=BF16)
                    ops.linear(h, self.ar.span(p + "self_attn.k_proj.weight", p + "self_attn.v_proj.weight"), kv)
                    qkv = torch.empty(M, (nh + 2) * hd, device=dev, dtype=BF16)
                    ops.copy_rows(kv, 2 * hd, 0, qkv[:, nh * hd:], (nh + 2) * hd, 0, 1, M, 2 * hd)
                    ops.qkv_rope_split(qkv, pos[g.pos_key], self.rope(g.theta), None, Kj, Vj, B, g.T, nh, 1, hd, L1,
                                       g.off, Lp, g.off)
                    continue
                hs[g.name] = h
                if self.fuse_qkv_rope and not (self.f8 and (p + "self_attn.q_proj.weight") in self.f8) and \
                        ops.gemm_qkv_rope(h, self.qkv_w(p), pos[g.pos_key], self.rope(g.theta), Q, Kj, Vj, g.T, nh, hd,
                                          L1, g.off, Lp, g.off):
                    continue  # many rows (B >= 16): projection + RoPE + scatter in one 8-phase GEMM
                qkv = torch.empty(M, (nh + 2) * hd, device=dev, dtype=BF16)
                self.lin(h, p + "self_attn.q_proj.weight", self.qkv_w(p), qkv)
                ops.qkv_rope_split(qkv, pos[g.pos_key], self.rope(g.theta), Q, Kj, Vj, B, g.T, nh, 1, hd, L1, g.off,
                                   Lp, g.off)
            if last:
                break
            if self.infer_flash and not isinstance(cnt, GeneralMask):  # fused attention over the L1 prefix keys
                Os = {g.name: torch.empty(B * g.T, nh * hd, device=dev, dtype=BF16) for g in groups}
                fa = self._attn_flash_infer(Q, Kj, Vj, [(g.off, g.T, Os[g.name]) for g in groups], L1, L1, 0, cnt, B)
                if self.f8 is not None and self.f8_attn and hd == 256:
                    self._flash_f8(fa, Q, Kj, Vj, B, L1 * nh, L1)  # fp8 MFMA attention (C5, configs[4])
                else:
                    ops.flash_fwd(fa)
                for g in groups:
                    p = f"{g.prefix}{l}."
                    X[g.name] = self._post_attn_O(g, p, X[g.name], Os[g.name])
                continue
            if S is None:
                S = torch.empty(B, L1 * nh, Lp, device=dev, dtype=F32)
                Pm = torch.empty(B, L1 * nh, Lp, device=dev, dtype=BF16)
            ops.gemm(L1 * nh, L1, hd, Q, hd, True, Kj, hd, True, S, Lp, batch=B, sA=(L1 * nh * hd, 0),
                     sB=(Lp * hd, 0), sC=(L1 * nh * Lp, 0))
            ops.attn_softmax(S, Lp, Pm, Lp, B * L1 * nh, L1, 1.0 / math.sqrt(hd), cap=50.0,
                             rows_per_batch=L1 * nh, heads=nh, qoff=0, **_mask_kw(d, cnt, "itp"))
            for g in groups:
                p = f"{g.prefix}{l}."
                x = X[g.name]
                X[g.name] = self._post_attn(g, p, x, Pm, Vj, B, L1, Lp)
        return kcache, vcache

    # ========================================================= text generation ==
    def text_forward(self, ids, pix, pos, kc, vc, start, n_img, maxpos):
        """PiZero.infer_text (pizero.py:559-593): the vlm mixture alone through all layers (cache_mode
        "append", no last-layer skip, the all-zeros text mask of pizero.py:336-365 -> no masking), the
        new tokens ids [B, q] written at cache rows [start, start + q) of kc / vc [nL, B, Lcap, hd] and
        attending to rows [0, start + q); then the vlm final norm (if the mixture has one) and the
        lm_head tied to embed_tokens (pizero.py:106-112).  pix / n_img: images of a prefill (None / 0
        for decode steps).  maxpos: an upper bound of the positions (sizes the RoPE table).  Returns bf16
        logits [B, q, vocab]."""
        d = self.d
        B, q = ids.shape
        dev = ids.device
        nh, hd = d.nh, d.hd
        Lcap = kc.shape[2]
        self.fp8_refresh()
        nk = start + q
        table = self.w("embed_tokens.weight")
        img = table if pix is None else self.siglip_forward(pix, None)
        X = torch.empty(B * q, d.gH, device=dev, dtype=BF16)
        ops.embed_merge(ids, table, img, X, n_img, d.image_token, d.pad_token, math.sqrt(d.gH), 1.0)
        g = Group("vlm", "joint_model.mixtures.vlm.layers.", ["vlm"], q, 0, d.gH, d.gI, d.g_theta, False, "vlm")
        Q = torch.empty(B, q, nh * hd, device=dev, dtype=BF16)
        O = torch.empty(B * q, nh * hd, device=dev, dtype=BF16)
        few = self.gemv_ok(B * q, d.gH) and q * nh <= 32
        cs = self.rope(g.theta, maxpos)
        x = X
        for l in range(d.nL):
            p = f"{g.prefix}{l}."
            Kl, Vl = kc[l], vc[l]
            if few:
                ops.gemv_qkv_rope(x, self.qkv_w(p), pos, cs, Q, Kl, Vl, q, nh, hd, q, 0, Lcap, start,
                                  norm=(self.w(p + "input_layernorm.weight"), d.rms_eps))
                ops.decode_attn(Q, q, 0, Kl, Vl, O, B, nh, q, nk, 1.0 / math.sqrt(hd), 50.0, None, 0, 0, start)
            else:
                h = torch.empty_like(x)
                ops.rmsnorm(x, self.w(p + "input_layernorm.weight"), h, None, d.rms_eps)
                qkv = torch.empty(B * q, (nh + 2) * hd, device=dev, dtype=BF16)
                ops.linear(h, self.qkv_w(p), qkv)
                ops.qkv_rope_split(qkv, pos, cs, Q, Kl, Vl, B, q, nh, 1, hd, q, 0, Lcap, start)
                ops.flash_fwd(ops.flash_args(
                    B, 1, q * nh, nk, hd, Q, (hd, q * nh * hd, 0), Kl, (hd, Lcap * hd, 0), Vl, (hd, Lcap * hd, 0),
                    [(0, O, q * nh * hd, hd)], 0, None, 1.0 / math.sqrt(hd), cap=50.0, mask_mode=0,
                    rows_per_token=nh, key_split=True))
            x = self._post_attn_O(g, p, x, O)
        nw = "joint_model.mixtures.vlm.norm.weight"
        if nw in self.ar.slots:
            y = torch.empty_like(x)
            ops.rmsnorm(x, self.w(nw), y, None, d.rms_eps)
            x = y
        logits = torch.empty(B * q, table.shape[0], device=dev, dtype=BF16)
        ops.linear(x, table, logits)
        return logits.view(B, q, -1)

    def _kv_only_gemv(self, x, p, pos, g, Kj, Vj, L1, Lp):
        """last prefill layer, few rows: only the k|v projection (+RoPE on k) is consumed"""
        d = self.d
        ops.gemv_qkv_rope(x, self.ar.span(p + "self_attn.k_proj.weight", p + "self_attn.v_proj.weight"), pos,
                          self.rope(g.theta), None, Kj, Vj, g.T, 0, d.hd, L1, g.off, Lp, g.off,
                          norm=(self.w(p + "input_layernorm.weight"), d.rms_eps))

    def _flash_f8(self, fa, Q, K, V, B, nq, nk):
        """the joint attention of fa on the fp8 MFMA: Q rows / key rows quantised per row, V^T per head dim
        (pz_fp8_quant_rows, pz_fp8_quant_vt), then pz_flash_fwd_f8 (+ its key-split combine)"""
        dev = Q.device
        hd, Lp = self.d.hd, K.shape[1]
        qc = torch.empty(B * nq, hd, device=dev, dtype=torch.uint8)
        qs = torch.empty(B * nq, device=dev, dtype=F32)
        kc = torch.empty(B * Lp, hd, device=dev, dtype=torch.uint8)
        ks = torch.empty(B * Lp, device=dev, dtype=F32)
        vt = torch.empty(B, hd, (nk + 127) // 128 * 128, device=dev, dtype=torch.uint8)
        vs = torch.empty(B, hd, device=dev, dtype=F32)
        ops.fp8_quant_attn(Q.reshape(B * nq, hd), K.reshape(B * Lp, hd), V, B, nk, qc, qs, kc, ks, vt, vs)
        ops.flash_fwd_f8(fa, qc, qs, kc, ks, Lp, vt, vs)

    def _attn_flash_infer(self, Q, K, V, outs, Lq, nk, tok0, cnt, B):
        """pz_flash_args for the inference attention: queries = Lq tokens starting at joint token tok0
        (rows token*nh + head of Q [B, Lq*nh, hd]), keys = the first nk cached tokens; outs =
        [(token offset, T, O [B*T, nh*hd])] in token order."""
        d = self.d
        nh, hd, Lp = d.nh, d.hd, K.shape[1]
        return ops.flash_args(
            B, 1, Lq * nh, nk, hd, Q, (hd, Lq * nh * hd, 0), K, (hd, Lp * hd, 0), V, (hd, Lp * hd, 0),
            [((off - tok0) * nh, O, T * nh * hd, hd) for off, T, O in outs], 0, None, 1.0 / math.sqrt(hd), cap=50.0,
            mask_mode=1, cnt=cnt, prefix=d.P, cond=d.C, rows_per_token=nh, mask_row0=tok0 * nh,
            key_split=True)

    def _post_attn_O(self, g, p, x, O):
        """o_proj (+resid), post-attention RMSNorm, GeGLU MLP (+resid) of one mixture."""
        d = self.d
        M = x.shape[0]
        dev = x.device
        xm = torch.empty_like(x)
        self.lin(O, p + "self_attn.o_proj.weight", self.w(p + "self_attn.o_proj.weight"), xm, resid=x)
        hm = torch.empty(M, g.inter, device=dev, dtype=BF16)
        if self.few_rows(M, x.shape[1]):  # few rows (denoise / proprio): RMSNorm fused into the gate|up GEMM
            self.lin(xm, p + "mlp.gate_proj.weight", self.gu_w(p), hm, epi=PZ_EPI_GEGLU,
                     norm=(self.w(p + "post_attention_layernorm.weight"), d.rms_eps))
        elif self.w8a8_in(p + "mlp.gate_proj.weight", M, x.shape[1]):  # fp8: RMSNorm -> codes -> W8A8 GeGLU
            self.lin(self.norm_codes(xm, self.w(p + "post_attention_layernorm.weight"), d.rms_eps),
                     p + "mlp.gate_proj.weight", self.gu_w(p), hm, epi=PZ_EPI_GEGLU)
        else:
            h2 = torch.empty_like(x)
            ops.rmsnorm(xm, self.w(p + "post_attention_layernorm.weight"), h2, None, d.rms_eps)
            self.lin(h2, p + "mlp.gate_proj.weight", self.gu_w(p), hm, epi=PZ_EPI_GEGLU)
        xn = torch.empty_like(x)
        self.lin(hm, p + "mlp.down_proj.weight", self.w(p + "mlp.down_proj.weight"), xn, resid=xm)
        return xn

    def _post_attn(self, g, p, x, Pm, Vj, B, Lq, Lp, qrow0=None):
        d = self.d
        nh, hd = d.nh, d.hd
        M = x.shape[0]
        dev = x.device
        q0 = g.off if qrow0 is None else qrow0
        O = torch.empty(M, nh * hd, device=dev, dtype=BF16)
        ops.gemm(g.T * nh, hd, Lp, Pm[:, q0 * nh:], Lp, True, Vj, hd, False, O, hd, batch=B,
                 sA=(Lq * nh * Lp, 0), sB=(Lp * hd, 0), sC=(g.T * nh * hd, 0))
        xm = torch.empty_like(x)
        ops.linear(O, self.w(p + "self_attn.o_proj.weight"), xm, resid=x)
        h2 = torch.empty_like(x)
        ops.rmsnorm(xm, self.w(p + "post_attention_layernorm.weight"), h2, None, d.rms_eps)
        hm = torch.empty(M, g.inter, device=dev, dtype=BF16)
        ops.linear(h2, self.gu_w(p), hm, epi=PZ_EPI_GEGLU)
        xn = torch.empty_like(x)
        ops.linear(hm, self.w(p + "mlp.down_proj.weight"), xn, resid=xm)
        return xn

    def denoise_step(self, action, t, apos, cnt, kcache, vcache, B):
        """One Euler step of pizero.py:461-481 against the cached vlm+proprio K/V."""
        d = self.d
        dev = action.device
        nh, hd, Lp, L = d.nh, d.hd, d.Lp, d.L
        # the step's glue in two launches (pz_action_in / pz_action_out, bit-identical to cast + Linear + time
        # embedding and RMSNorm + decoder + Euler; PZ_FUSED_GLUE=0: the separate kernels)
        glue = (d.aH <= 1024 and d.aH % 8 == 0 and d.A <= 8 and os.environ.get("PZ_FUSED_GLUE", "1") != "0" and
                all(self.w(k).data_ptr() % 16 == 0 for k in ("joint_model.mixtures.action.norm.weight",
                                                             "action_decoder.weight")))
        if glue:
            cat = torch.empty(B * d.H, 2 * d.aH, device=dev, dtype=BF16)
            ops.action_in(action, self.w("action_encoder.linear_1.weight"), self.w("action_encoder.linear_1.bias"), t,
                          cat, B, d.H, d.aH, d.tmax, ref_bf16=d.time_bf16)
            sq = math.sqrt(d.aH)
            if sq.is_integer() and (int(sq) & (int(sq) - 1)) == 0 and os.environ.get("PZ_FOLD_SCALE", "1") != "0":
                # the joint model's sqrt(hidden) input scaling is a power of two (32 at hidden 1024): folded into the
                # last encoder Linear as alpha with a pre-scaled bias -- 2^k (acc + b) rounds exactly like rounding
                # first and scaling the bf16 after (the copy_rows launch it replaces), so the bits are unchanged
                x = self._action_embed_tail(cat, alpha=sq)
            else:
                e3 = self._action_embed_tail(cat)
                x = torch.empty_like(e3)
                ops.copy_rows(e3, d.aH, 0, x, d.aH, 0, 1, B * d.H, d.aH, scale=sq)
        else:
            psi = torch.empty(B * d.H, d.A, device=dev, dtype=BF16)
            ops.cast_to_bf16(action, psi)
            e3 = self.action_embed(psi, t, None)
            x = torch.empty_like(e3)
            ops.copy_rows(e3, d.aH, 0, x, d.aH, 0, 1, B * d.H, d.aH, scale=math.sqrt(d.aH))
        g = Group("action", "joint_model.mixtures.action.layers.", ["action"], d.H, d.P + d.C, d.aH, d.aI, d.a_theta,
                  False, "action")
        Q = torch.empty(B, d.H, nh * hd, device=dev, dtype=BF16)
        S = Pm = O = None
        for l in range(d.nL):
            p = f"{g.prefix}{l}."
            Kj, Vj = kcache[l], vcache[l]
            M = x.shape[0]
            nrm = (self.w(p + "input_layernorm.weight"), d.rms_eps)
            if self.gemv_ok(M, d.aH):  # one launch: RMSNorm + q|k|v GEMV + RoPE + Q / K-cache / V-cache scatter
                ops.gemv_qkv_rope(x, self.qkv_w(p), apos, self.rope(g.theta), Q, Kj, Vj, d.H, nh, hd, d.H, 0, Lp,
                                  g.off, norm=nrm)
            elif self.fuse_qkv_rope and self.few_rows(M, d.aH) and \
                    ops.gemm_qkv_rope(x, self._qkv_w_f8(p)[0], apos, self.rope(g.theta), Q, Kj, Vj, d.H, nh, hd, d.H,
                                      0, Lp, g.off, norm=nrm, w_scale=self._qkv_w_f8(p)[1]):
                pass  # C5's 50-row chunk: RMSNorm + skinny-64 q|k|v (bf16 or W8A16) + RoPE + scatter in one launch
            else:
                qkv = torch.empty(M, (nh + 2) * hd, device=dev, dtype=BF16)
                if self.few_rows(M, d.aH):  # RMSNorm fused into the q|k|v GEMM
                    self.lin(x, p + "self_attn.q_proj.weight", self.qkv_w(p), qkv,
                             norm=(self.w(p + "input_layernorm.weight"), d.rms_eps))
                else:
                    h = torch.empty_like(x)
                    ops.rmsnorm(x, self.w(p + "input_layernorm.weight"), h, None, d.rms_eps)
                    self.lin(h, p + "self_attn.q_proj.weight", self.qkv_w(p), qkv)
                ops.qkv_rope_split(qkv, apos, self.rope(g.theta), Q, Kj, Vj, B, d.H, nh, 1, hd, d.H, 0, Lp, g.off)
            if self.infer_flash and not isinstance(cnt, GeneralMask):  # fused attention over every cached key
                if O is None:
                    O = torch.empty(B * d.H, nh * hd, device=dev, dtype=BF16)
                if self.decode_attn_ok():  # one workgroup per (head, sample), no key split / combine launch
                    ops.decode_attn(Q, d.H, 0, Kj, Vj, O, B, nh, d.H, L, 1.0 / math.sqrt(hd), 50.0, cnt, d.P, d.C,
                                    g.off)
                else:
                    ops.flash_fwd(self._attn_flash_infer(Q, Kj, Vj, [(g.off, d.H, O)], d.H, L, g.off, cnt, B))
                x = self._post_attn_O(g, p, x, O)
                continue
            if S is None:
                S = torch.empty(B, d.H * nh, Lp, device=dev, dtype=F32)
                Pm = torch.empty(B, d.H * nh, Lp, device=dev, dtype=BF16)
            ops.gemm(d.H * nh, L, hd, Q, hd, True, Kj, hd, True, S, Lp, batch=B, sA=(d.H * nh * hd, 0),
                     sB=(Lp * hd, 0), sC=(d.H * nh * Lp, 0))
            ops.attn_softmax(S, Lp, Pm, Lp, B * d.H * nh, L, 1.0 / math.sqrt(hd), cap=50.0,
                             rows_per_batch=d.H * nh, heads=nh, qoff=d.P + d.C, **_mask_kw(d, cnt, "act"))
            x = self._post_attn(g, p, x, Pm, Vj, B, d.H, Lp, qrow0=0)
        if glue:
            ops.action_out(x, self.w("joint_model.mixtures.action.norm.weight"), d.rms_eps,
                           self.w("action_decoder.weight"), self.w("action_decoder.bias"), action, t, B, d.H,
                           1.0 / d.steps)
            return
        y = torch.empty_like(x)
        ops.rmsnorm(x, self.w("joint_model.mixtures.action.norm.weight"), y, None, d.rms_eps)
        v = torch.empty(B * d.H, 8, device=dev, dtype=BF16)
        ops.small_linear(y, self.w("action_decoder.weight"), v[:, : d.A], bias=self.w("action_decoder.bias"))
        ops.euler_step(action, v, 8, d.H * 8, t, B, d.H, d.A, 1.0 / d.steps)

    def infer_action(self, ids, pix, cnt, vpos, ppos, apos, proprios, noise, kcache, vcache, clip=True):
        d = self.d
        B = ids.shape[0]
        self.fp8_refresh()
        self.prefill(ids, pix, cnt, vpos, ppos, proprios, kcache, vcache)
        action = noise.clone()
        t = torch.zeros(B, device=pix.device, dtype=F32)
        for _ in range(d.steps):
            self.denoise_step(action, t, apos, cnt, kcache, vcache, B)
        if clip and d.clip is not None:
            ops.clamp_(action, -d.clip, d.clip)
        return action

    # --------------------------------------------------------------- hooks --
    hook = None  # called as hook(stage, layer, streams) when a layer's parameter gradients are final
    post_backward = None  # called once at the end of train_backward (gradient all-reduce flush)

    def _notify(self, stage, layer, streams=()):
        """streams: side streams (besides the current one) whose enqueued work produced some of those gradients"""
        if self.hook is not None:
            self.hook(stage, layer, streams)
