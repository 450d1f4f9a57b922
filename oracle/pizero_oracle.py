"""CPU fp32 restatement of the reference Pi0 hot path (TEST INFRASTRUCTURE).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg may import this module.  It is the checker, never the
product: the product path lives in ``open-pi-zero_amd/`` and calls HIP kernels
through the C ABI in ``include/pz_abi.h``.

Every function restates the reference's math in plain PyTorch-CPU fp32 on a
flat ``{state_dict key: tensor}`` dict (reference key layout), citing the
reference file:line it follows (paths relative to shroglck/open-pi-zero).
Autograd through these functions is the backward oracle.  The restatement is
pinned against fixtures produced by the reference itself
(``tests/golden/make_golden.py``, run in the build container).
"""

from __future__ import annotations

import math

import torch
import torch.nn.functional as F

# ----------------------------------------------------------------- dims ----

FULL_DIMS = dict(
    vocab_size=257216, image_token_index=257152, pad_token_id=0,
    max_seq_len=276, num_image_tokens=256, cond_steps=1, horizon_steps=4,
    action_dim=7, proprio_dim=7,
    image_size=224, patch_size=14, vis_hidden=1152, vis_inter=4304,
    vis_layers=27, vis_heads=16, ln_eps=1e-6, proj_dim=2048,
    n_layers=18, n_heads=8, n_kv=1, head_dim=256, rms_eps=1e-6,
    vlm_hidden=2048, vlm_inter=16384, vlm_theta=10000.0,
    act_hidden=1024, act_inter=4096, act_theta=100.0,
    time_max_period=100.0, flow_sig_min=0.001, num_inference_steps=10,
    final_action_clip_value=1.0,
)

# small structural twin of the bridge config (fast on CPU, same code paths)
TINY_DIMS = dict(
    vocab_size=1024, image_token_index=1000, pad_token_id=0,
    max_seq_len=24, num_image_tokens=16, cond_steps=1, horizon_steps=4,
    action_dim=7, proprio_dim=7,
    image_size=56, patch_size=14, vis_hidden=64, vis_inter=136,
    vis_layers=2, vis_heads=4, ln_eps=1e-6, proj_dim=128,
    n_layers=3, n_heads=8, n_kv=1, head_dim=32, rms_eps=1e-6,
    vlm_hidden=128, vlm_inter=256, vlm_theta=10000.0,
    act_hidden=64, act_inter=128, act_theta=100.0,
    time_max_period=100.0, flow_sig_min=0.001, num_inference_steps=10,
    final_action_clip_value=1.0,
)


def param_shapes(d: dict) -> dict:
    """Reference state_dict keys -> shapes (after tie_action_proprio_weights).

    Follows the module tree of pizero.py:61-103, siglip.py:34-320,
    joint_model.py:308-323, mixture.py:23-185.
    """
    s = {}
    s["embed_tokens.weight"] = (d["vocab_size"], d["vlm_hidden"])
    vt = "vision_tower.vision_model."
    H, I, ps = d["vis_hidden"], d["vis_inter"], d["patch_size"]
    npatch = (d["image_size"] // ps) ** 2
    s[vt + "embeddings.patch_embedding.weight"] = (H, 3, ps, ps)
    s[vt + "embeddings.patch_embedding.bias"] = (H,)
    s[vt + "embeddings.position_embedding.weight"] = (npatch, H)
    for i in range(d["vis_layers"]):
        p = f"{vt}encoder.layers.{i}."
        for nm in ("k_proj", "v_proj", "q_proj", "out_proj"):
            s[p + f"self_attn.{nm}.weight"] = (H, H)
            s[p + f"self_attn.{nm}.bias"] = (H,)
        s[p + "layer_norm1.weight"] = (H,)
        s[p + "layer_norm1.bias"] = (H,)
        s[p + "mlp.fc1.weight"] = (I, H)
        s[p + "mlp.fc1.bias"] = (I,)
        s[p + "mlp.fc2.weight"] = (H, I)
        s[p + "mlp.fc2.bias"] = (H,)
        s[p + "layer_norm2.weight"] = (H,)
        s[p + "layer_norm2.bias"] = (H,)
    s[vt + "post_layernorm.weight"] = (H,)
    s[vt + "post_layernorm.bias"] = (H,)
    s["multi_modal_projector.linear.weight"] = (d["proj_dim"], H)
    s["multi_modal_projector.linear.bias"] = (d["proj_dim"],)
    nh, nkv, hd = d["n_heads"], d["n_kv"], d["head_dim"]
    for mix, hid, inter in (("vlm", d["vlm_hidden"], d["vlm_inter"]),
                            ("proprio", d["act_hidden"], d["act_inter"]),
                            ("action", d["act_hidden"], d["act_inter"])):
        for i in range(d["n_layers"]):
            p = f"joint_model.mixtures.{mix}.layers.{i}."
            s[p + "self_attn.q_proj.weight"] = (nh * hd, hid)
            s[p + "self_attn.k_proj.weight"] = (nkv * hd, hid)
            s[p + "self_attn.v_proj.weight"] = (nkv * hd, hid)
            s[p + "self_attn.o_proj.weight"] = (hid, nh * hd)
            s[p + "mlp.gate_proj.weight"] = (inter, hid)
            s[p + "mlp.up_proj.weight"] = (inter, hid)
            s[p + "mlp.down_proj.weight"] = (hid, inter)
            s[p + "input_layernorm.weight"] = (hid,)
            s[p + "post_attention_layernorm.weight"] = (hid,)
        if mix != "vlm" or d.get("vlm_final_norm"):
            s[f"joint_model.mixtures.{mix}.norm.weight"] = (hid,)
    A, Ah = d["action_dim"], d["act_hidden"]
    s["action_encoder.linear_1.weight"] = (Ah, A)
    s["action_encoder.linear_1.bias"] = (Ah,)
    s["action_encoder.linear_2.weight"] = (Ah, 2 * Ah)
    s["action_encoder.linear_2.bias"] = (Ah,)
    s["action_encoder.linear_3.weight"] = (Ah, Ah)
    s["action_encoder.linear_3.bias"] = (Ah,)
    s["proprio_encoder.weight"] = (Ah, d["proprio_dim"])
    s["proprio_encoder.bias"] = (Ah,)
    s["action_decoder.weight"] = (A, Ah)
    s["action_decoder.bias"] = (A,)
    return s


def unique_param_names(d: dict) -> list:
    """Names without the tied proprio aliases (proprio == action module)."""
    return [k for k in param_shapes(d) if ".mixtures.proprio." not in k]


def synth_weights(d: dict, seed: int = 0) -> dict:
    """Generator-defined fp32 weights; proprio keys alias the action tensors."""
    import numpy as np  # noqa: F401

    from oracle.synth import synth_state_dict

    shp = {k: v for k, v in param_shapes(d).items() if ".mixtures.proprio." not in k}
    W = {k: torch.from_numpy(v) for k, v in synth_state_dict(shp, seed).items()}
    for k in list(W):
        if ".mixtures.action." in k:
            W[k.replace(".mixtures.action.", ".mixtures.proprio.")] = W[k]
    if d.get("use_lm_head"):
        W["lm_head.weight"] = W["embed_tokens.weight"]  # tied (pizero.py:112)
    return W


# ------------------------------------------------------------ primitives ----


def gemma_rmsnorm(x, w, eps):
    """paligemma/modules.py:7-21: fp32 x*rsqrt(mean(x^2)+eps)*(1+w)."""
    xf = x.float()
    y = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)
    return (y * (1.0 + w.float())).type_as(x)


def rope_cos_sin(pos, head_dim, theta):
    """paligemma/modules.py:24-67: inv_freq = 1/theta^(2i/d), emb = cat(f, f)."""
    inv = 1.0 / (theta ** (torch.arange(0, head_dim, 2, dtype=torch.int64).float() / head_dim))
    freqs = pos[:, :, None].float() * inv[None, None, :]
    emb = torch.cat((freqs, freqs), dim=-1)
    return emb.cos(), emb.sin()


def apply_rope(x, cos, sin):
    """model/utils.py:4-16, x [B, h, L, D], cos/sin [B, L, D]."""
    c, s = cos[:, None], sin[:, None]
    half = x.shape[-1] // 2
    rot = torch.cat((-x[..., half:], x[..., :half]), dim=-1)
    return x * c + rot * s


def linear(x, W, name, bias=True):
    b = W.get(name + ".bias") if bias else None
    return F.linear(x, W[name + ".weight"], b)


# ---------------------------------------------------------------- SigLIP ----


def siglip_forward(W, d, pixel_values):
    """siglip.py:34-78 (patch embed), 81-238 (encoder layer), 273-300."""
    vt = "vision_tower.vision_model."
    H, nh = d["vis_hidden"], d["vis_heads"]
    hd = H // nh
    x = F.conv2d(pixel_values, W[vt + "embeddings.patch_embedding.weight"],
                 W[vt + "embeddings.patch_embedding.bias"], stride=d["patch_size"])
    x = x.flatten(2).transpose(1, 2)
    x = x + W[vt + "embeddings.position_embedding.weight"][None]
    B, L, _ = x.shape
    for i in range(d["vis_layers"]):
        p = f"{vt}encoder.layers.{i}."
        r = x
        h = F.layer_norm(x, (H,), W[p + "layer_norm1.weight"], W[p + "layer_norm1.bias"], d["ln_eps"])
        q = linear(h, W, p + "self_attn.q_proj").view(B, L, nh, hd).transpose(1, 2)
        k = linear(h, W, p + "self_attn.k_proj").view(B, L, nh, hd).transpose(1, 2)
        v = linear(h, W, p + "self_attn.v_proj").view(B, L, nh, hd).transpose(1, 2)
        a = torch.matmul(q, k.transpose(2, 3)) * (hd ** -0.5)
        a = torch.softmax(a.float(), dim=-1).to(q.dtype)
        o = torch.matmul(a, v).transpose(1, 2).reshape(B, L, H)
        x = r + linear(o, W, p + "self_attn.out_proj")
        r = x
        h = F.layer_norm(x, (H,), W[p + "layer_norm2.weight"], W[p + "layer_norm2.bias"], d["ln_eps"])
        h = F.gelu(linear(h, W, p + "mlp.fc1"), approximate="tanh")
        x = r + linear(h, W, p + "mlp.fc2")
    return F.layer_norm(x, (H,), W[vt + "post_layernorm.weight"], W[vt + "post_layernorm.bias"], d["ln_eps"])


def embed_siglip_and_text(W, d, input_ids, pixel_values):
    """pizero.py:376-414: gather text rows, SigLIP+projector, /sqrt(hidden), merge."""
    emb = F.embedding(input_ids, W["embed_tokens.weight"])
    # several images per sample (config C5, the Pi0-paper shape; the reference PiZero takes one image,
    # pizero.py:389-413): SigLIP runs per image and the images' tokens are concatenated in image order
    # into the sample's image-token slots -- an extension, pinned by composition, not by a reference run
    B = input_ids.shape[0]
    H = d["image_size"]
    img = siglip_forward(W, d, pixel_values.reshape(-1, 3, H, H))
    img = linear(img, W, "multi_modal_projector.linear") / (d["vlm_hidden"] ** 0.5)
    img = img.reshape(B, -1, img.shape[-1])
    out = torch.zeros_like(emb)
    text = (input_ids != d["image_token_index"]) & (input_ids != d["pad_token_id"])
    out = torch.where(text[..., None], emb, out)
    for b in range(input_ids.shape[0]):
        idx = (input_ids[b] == d["image_token_index"]).nonzero(as_tuple=True)[0]
        out[b, idx] = img[b, : len(idx)].to(out.dtype)  # (autocast: img may be bf16)
    return out


# ---------------------------------------------------------- mask / pos ----


def build_mask_and_positions(d, attention_mask, dtype=torch.float32):
    """pizero.py:271-324 block mask (finfo.min / 0) and 1-based positions."""
    B = attention_mask.shape[0]
    P, C, Hz = d["max_seq_len"], d["cond_steps"], d["horizon_steps"]
    L = P + C + Hz
    cnt = attention_mask.sum(1)
    m = torch.full((B, L, L), torch.finfo(dtype).min, dtype=dtype)
    for b in range(B):
        c = int(cnt[b])
        m[b, :c, :c] = 0
        m[b, P:, :c] = 0
    m[:, P:P + C, P:P + C] = 0
    m[:, P + C:, P:] = 0
    vpos = torch.arange(1, P + 1).repeat(B, 1)
    ppos = torch.arange(1, C + 1).repeat(B, 1)
    apos = torch.arange(C + 1, C + Hz + 1).repeat(B, 1)
    return m[:, None], vpos, ppos, apos


def split_mask(d, mask):
    """pizero.py:326-336."""
    n = d["max_seq_len"] + d["cond_steps"]
    return mask[..., :n, :n], mask[..., -d["horizon_steps"]:, :]


# ---------------------------------------------------------- joint model ----

_MIX = {"vlm": ("vlm_hidden", "vlm_theta"), "proprio": ("act_hidden", "act_theta"),
        "action": ("act_hidden", "act_theta")}


def joint_forward(W, d, embeds, positions, mask, cache=None, return_cache=False,
                  skip_last=("vlm", "proprio")):
    """joint_model.py:24-304 (layer + joint attention) and 328-383 (model).

    ``embeds``: ordered dict name -> [B, len, hidden] (scaled in place by
    sqrt(hidden) like joint_model.py:348-355).  ``cache``: name -> list of
    per-layer (K, V) post-RoPE for non-active mixtures ("append_non_active").
    Returns {name: final-normed hidden} for non-skipped mixtures with a final
    norm, plus the new cache if ``return_cache``.
    """
    names = list(embeds)
    nh, nkv, hd = d["n_heads"], d["n_kv"], d["head_dim"]
    x = {n: embeds[n] * torch.tensor(embeds[n].shape[-1] ** 0.5, dtype=embeds[n].dtype) for n in names}
    new_cache = {n: [] for n in names}
    nL = d["n_layers"]
    for li in range(nL):
        last = li == nL - 1
        skip = skip_last if last else ()
        qs, ks, vs, lens = [], [], [], []
        if cache is not None:
            for cn, kvl in cache.items():
                if cn not in names:
                    ks.append(kvl[li][0])
                    vs.append(kvl[li][1])
        for n in names:
            p = f"joint_model.mixtures.{n}.layers.{li}."
            h = gemma_rmsnorm(x[n], W[p + "input_layernorm.weight"], d["rms_eps"])
            B, T, _ = h.shape
            q = F.linear(h, W[p + "self_attn.q_proj.weight"]).view(B, T, nh, hd).transpose(1, 2)
            k = F.linear(h, W[p + "self_attn.k_proj.weight"]).view(B, T, nkv, hd).transpose(1, 2)
            v = F.linear(h, W[p + "self_attn.v_proj.weight"]).view(B, T, nkv, hd).transpose(1, 2)
            cos, sin = rope_cos_sin(positions[n], hd, d[_MIX[n][1]])
            k = apply_rope(k, cos, sin)
            q = apply_rope(q, cos, sin)
            if return_cache:
                new_cache[n].append((k, v))
            qs.append(q)
            ks.append(k)
            vs.append(v)
            lens.append(T)
        rep = nh // nkv
        q = torch.cat(qs, dim=2)
        k = torch.cat([t.repeat_interleave(rep, dim=1) for t in ks], dim=2)
        v = torch.cat([t.repeat_interleave(rep, dim=1) for t in vs], dim=2)
        a = torch.matmul(q, k.transpose(2, 3)) / math.sqrt(hd)
        a = torch.tanh(a / 50.0) * 50.0
        a = a + mask
        a = torch.softmax(a, dim=-1, dtype=torch.float32).to(q.dtype)
        o = torch.matmul(a, v).transpose(1, 2).reshape(q.shape[0], sum(lens), nh * hd)
        outs = torch.split(o, lens, dim=1)
        for n, on in zip(names, outs):
            if n in skip:
                x[n] = None
                continue
            p = f"joint_model.mixtures.{n}.layers.{li}."
            r = x[n] + F.linear(on, W[p + "self_attn.o_proj.weight"])
            h = gemma_rmsnorm(r, W[p + "post_attention_layernorm.weight"], d["rms_eps"])
            h = F.linear(F.gelu(F.linear(h, W[p + "mlp.gate_proj.weight"]), approximate="tanh")
                         * F.linear(h, W[p + "mlp.up_proj.weight"]), W[p + "mlp.down_proj.weight"])
            x[n] = r + h
    out = {}
    for n in names:
        key = f"joint_model.mixtures.{n}.norm.weight"
        if n not in skip_last and key in W:
            out[n] = gemma_rmsnorm(x[n], W[key], d["rms_eps"])
    if return_cache:
        return out, new_cache
    return out


# ------------------------------------------------------- action modules ----


def time_embedding(d, t):
    """vla/modules.py:9-22 (SinusoidalPosEmb, dim = action hidden)."""
    half = d["act_hidden"] // 2
    e = math.log(d["time_max_period"]) / (half - 1)
    f = torch.exp(torch.arange(half, dtype=t.dtype) * -e)
    a = t[:, None] * f[None, :]
    return torch.cat((a.sin(), a.cos()), dim=-1)


def action_encoder(W, a, temb):
    """vla/modules.py:25-53 (time_cond=True): W3 silu(W2 [temb, W1 a])."""
    e = linear(a, W, "action_encoder.linear_1")
    te = temb[:, None, :].expand(-1, a.shape[1], -1)
    e = torch.cat([te, e], dim=-1)
    e = F.silu(linear(e, W, "action_encoder.linear_2"))
    return linear(e, W, "action_encoder.linear_3")


def psi_t(d, x0, x1, t):
    """pizero.py:597-605."""
    tt = t[:, None, None]
    return (1 - (1 - d["flow_sig_min"]) * tt) * x0 + tt * x1


# ------------------------------------------------------------ top level ----


def pizero_loss(W, d, input_ids, pixel_values, causal_mask, vlm_pos, proprio_pos,
                action_pos, proprios, actions, t, x0):
    """pizero.py:607-661 with the noise x0 supplied (no RNG)."""
    x1 = actions
    psi = psi_t(d, x0, x1, t)
    emb = embed_siglip_and_text(W, d, input_ids, pixel_values)
    pe = linear(proprios, W, "proprio_encoder")
    te = time_embedding(d, t)
    ae = action_encoder(W, psi, te)
    out = joint_forward(W, d, {"vlm": emb, "proprio": pe, "action": ae},
                        {"vlm": vlm_pos, "proprio": proprio_pos, "action": action_pos},
                        causal_mask)["action"]
    v = linear(out, W, "action_decoder")
    dpsi = x1 - (1 - d["flow_sig_min"]) * x0
    return torch.mean((v - dpsi) ** 2)


def pizero_infer(W, d, input_ids, pixel_values, itp_mask, action_mask, vlm_pos,
                 proprio_pos, action_pos, proprios, noise, clip=True):
    """pizero.py:416-490 (KV-cached prefill + Euler) with supplied noise."""
    emb = embed_siglip_and_text(W, d, input_ids, pixel_values)
    pe = linear(proprios, W, "proprio_encoder")
    _, cache = joint_forward(W, d, {"vlm": emb, "proprio": pe},
                             {"vlm": vlm_pos, "proprio": proprio_pos}, itp_mask,
                             return_cache=True)
    a = noise.clone()
    n = d["num_inference_steps"]
    dt = 1.0 / n
    t = torch.zeros(a.shape[0], dtype=a.dtype)
    for _ in range(n):
        te = time_embedding(d, t)
        ae = action_encoder(W, a, te)
        h = joint_forward(W, d, {"action": ae}, {"action": action_pos}, action_mask,
                          cache=cache)["action"]
        a = a + dt * linear(h, W, "action_decoder")
        t = t + dt
    if clip and d["final_action_clip_value"] is not None:
        c = d["final_action_clip_value"]
        a = torch.clamp(a, -c, c)
    return a


def pizero_infer_naive(W, d, input_ids, pixel_values, causal_mask, vlm_pos,
                       proprio_pos, action_pos, proprios, noise, clip=True):
    """pizero.py:492-557: re-run the whole joint model every Euler step."""
    emb = embed_siglip_and_text(W, d, input_ids, pixel_values)
    pe = linear(proprios, W, "proprio_encoder")
    a = noise.clone()
    n = d["num_inference_steps"]
    dt = 1.0 / n
    t = torch.zeros(a.shape[0], dtype=a.dtype)
    for _ in range(n):
        te = time_embedding(d, t)
        ae = action_encoder(W, a, te)
        h = joint_forward(W, d, {"vlm": emb.clone(), "proprio": pe.clone(), "action": ae},
                          {"vlm": vlm_pos, "proprio": proprio_pos, "action": action_pos},
                          causal_mask)["action"]
        a = a + dt * linear(h, W, "action_decoder")
        t = t + dt
    if clip and d["final_action_clip_value"] is not None:
        c = d["final_action_clip_value"]
        a = torch.clamp(a, -c, c)
    return a


# ------------------------------------------------------ text generation ----


def text_positions(attention_mask):
    """pizero.py:336-365: positions cumsum(attention_mask), pads -> 1."""
    return attention_mask.cumsum(-1).masked_fill(attention_mask == 0, 1)


def pizero_infer_text(W, d, input_ids, pixel_values, attention_mask, new_tokens):
    """pizero.py:559-593 with a KV cache, teacher-forced with ``new_tokens`` [B, n] (the tokens fed back
    after the prefill).  The cached run's semantics as one masked pass: prompt tokens attend to the
    whole prompt (the all-zeros prefill mask), generated token k to the prompt and generated tokens
    <= k (what the cache holds when it is fed); positions cumsum(mask) for the prompt, count + 1 + k
    for generated token k.  Returns logits [B, q + n, vocab] (rows q-1.. are the next-token logits)."""
    B, q = input_ids.shape
    n = new_tokens.shape[1]
    emb = embed_siglip_and_text(W, d, input_ids, pixel_values)
    gen = F.embedding(new_tokens, W["embed_tokens.weight"])
    x = torch.cat([emb, gen], dim=1)
    pos = torch.cat([text_positions(attention_mask),
                     attention_mask.sum(-1, keepdim=True) + 1 + torch.arange(n)[None, :]], dim=1)
    N = q + n
    i = torch.arange(N)[:, None]
    j = torch.arange(N)[None, :]
    allowed = (j < q) & (i < q) | (i >= q) & ((j < q) | (j <= i))
    mask = torch.where(allowed, 0.0, torch.finfo(torch.float32).min)[None, None].expand(B, 1, N, N)
    h = joint_forward(W, d, {"vlm": x}, {"vlm": pos}, mask, skip_last=())["vlm"]
    return F.linear(h, W["embed_tokens.weight"])
