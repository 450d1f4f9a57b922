"""ctypes binding of libpizero_hip.so (the C ABI declared in include/pz_abi.h).

The library is loaded once, from the package directory only; there is no
fallback path: if it is missing or fails to load, every op raises.
"""

from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(_HERE, "libpizero_hip.so")
# A/B runs only (tools/): another in-tree build of the same ABI, e.g. a baseline of a kernel change
if os.environ.get("PZ_LIB_PATH"):
    LIB_PATH = os.path.join(_HERE, os.path.basename(os.environ["PZ_LIB_PATH"]))
    import sys as _sys

    print(f"[pizero_native] PZ_LIB_PATH override: loading {LIB_PATH} instead of the default libpizero_hip.so",
          file=_sys.stderr, flush=True)

ABI_VERSION = 20  # include/pz_abi.h PZ_ABI_VERSION
PZ_EPI_NONE, PZ_EPI_GELU, PZ_EPI_GEGLU, PZ_EPI_SILU = 0, 1, 2, 3
PZ_EPI_DGELU, PZ_EPI_DSILU, PZ_EPI_DGEGLU = 4, 5, 6
PZ_SUMSQ_PARTS = 2048  # include/pz_abi.h

i64, i32, f32, vp = C.c_int64, C.c_int32, C.c_float, C.c_void_p
fp = C.POINTER(C.c_float)


class GemmArgs(C.Structure):
    _fields_ = [
        ("M", i64), ("N", i64), ("K", i64),
        ("A", vp), ("lda", i64), ("a_kcontig", i32),
        ("B", vp), ("ldb", i64), ("b_kcontig", i32),
        ("C", vp), ("ldc", i64), ("c_fp32", i32),
        ("batch", i64), ("batch_inner", i64),
        ("sA_outer", i64), ("sA_inner", i64), ("sB_outer", i64), ("sB_inner", i64),
        ("sC_outer", i64), ("sC_inner", i64), ("sR_outer", i64), ("sR_inner", i64),
        ("epilogue", i32), ("alpha", f32), ("beta_accum", i32),
        ("bias", vp), ("resid", vp), ("ld_resid", i64), ("aux", vp), ("ld_aux", i64),
        ("geglu_inter", i64),
        ("workspace", vp), ("ws_bytes", i64),
        ("norm_w", vp), ("norm_eps", f32),
        ("fp8_mode", i32), ("a_row_scale", vp),
    ]


class SmallGemmArgs(C.Structure):
    _fields_ = [
        ("M", i64), ("N", i64), ("K", i64),
        ("A", vp), ("sAm", i64), ("sAk", i64),
        ("B", vp), ("sBk", i64), ("sBn", i64),
        ("C", vp), ("ldc", i64), ("bias", vp), ("alpha", f32), ("beta", i32),
    ]


class SoftmaxArgs(C.Structure):
    _fields_ = [
        ("S", vp), ("lds", i64), ("P", vp), ("ldp", i64), ("tcap", vp),
        ("R", i64), ("N", i64), ("scale", f32), ("cap", f32), ("mask_mode", i32),
        ("rows_per_batch", i64), ("heads", i64), ("qoff", i64),
        ("cnt", vp), ("prefix", i64), ("cond", i64),
        ("mask", vp), ("ldm", i64), ("mask_bstride", i64),
    ]


class FlashArgs(C.Structure):
    _fields_ = [
        ("Z", i64), ("H", i64), ("nq", i64), ("nk", i64), ("head_dim", i64),
        ("q", vp), ("ldq", i64), ("q_bstride", i64), ("q_hstride", i64),
        ("k", vp), ("ldk", i64), ("k_bstride", i64), ("k_hstride", i64),
        ("v", vp), ("ldv", i64), ("v_bstride", i64), ("v_hstride", i64),
        ("n_groups", i32),
        ("g_row0", i64 * 3), ("g_o", vp * 3), ("g_bstride", i64 * 3), ("g_ld", i64 * 3),
        ("o_hstride", i64),
        ("lse", vp),
        ("scale", f32), ("cap", f32),
        ("mask_mode", i32),
        ("cnt", vp), ("prefix", i64), ("cond", i64), ("rows_per_token", i64),
        ("g_do", vp * 3),
        ("delta", vp),
        ("dq", vp), ("dk", vp), ("dv", vp),
        ("ws", vp), ("ws_bytes", i64),
        ("mask_row0", i64),
    ]


class AdamW8Args(C.Structure):
    _fields_ = [
        ("p", vp), ("g", vp), ("s1", vp), ("s2", vp), ("absmax1", vp), ("absmax2", vp),
        ("m32", vp), ("v32", vp), ("seg", vp), ("nseg", i64), ("nblocks", i64),
        ("qmap1", vp), ("qmap2", vp),
        ("beta1", f32), ("beta2", f32), ("omb1", f32), ("omb2", f32), ("step", f32), ("epsc", f32),
        ("decay", f32), ("gscale", vp),
    ]


class QkvRopeArgs(C.Structure):
    _fields_ = [
        ("x", vp), ("ldx", i64), ("W", vp), ("ldw", i64), ("M", i64), ("N", i64), ("K", i64),
        ("norm_w", vp), ("norm_eps", f32), ("pos", vp), ("cs", vp), ("q_out", vp), ("k_out", vp), ("v_out", vp),
        ("T", i64), ("nh", i64), ("hd", i64), ("Lq", i64), ("qoff", i64), ("Lk", i64), ("koff", i64),
        ("w_fp8", i32), ("w_scale", f32),
    ]


class ReduceSeg(C.Structure):
    _fields_ = [("part", vp), ("P", i64), ("D", i64), ("out", vp), ("beta", i32)]


class DecodeAttnArgs(C.Structure):
    _fields_ = [
        ("q", vp), ("ldq", i64), ("Lq", i64), ("qoff", i64), ("k", vp), ("v", vp), ("k_bstride", i64),
        ("v_bstride", i64), ("o", vp), ("ldo", i64), ("B", i64), ("nh", i64), ("T", i64), ("nk", i64),
        ("head_dim", i64), ("scale", f32), ("cap", f32), ("cnt", vp), ("prefix", i64), ("cond", i64),
        ("qtok0", i64), ("ws", vp), ("ws_bytes", i64),
    ]


# name -> argtypes (restype int unless listed in _RESTYPE)
SIGNATURES = {
    "pz_gemm": [C.POINTER(GemmArgs), vp],
    "pz_fp8_quant_rows": [vp, i64, vp, i64, vp, i64, i64, vp],
    "pz_fp8_quant_tensor": [vp, i64, vp, f32, vp],
    "pz_fp8_quant_vt": [vp, i64, i64, i64, i64, vp, vp, i64, vp],
    "pz_rmsnorm_fwd_f8": [vp, i64, vp, vp, i64, vp, i64, i64, f32, vp],
    "pz_layernorm_fwd_f8": [vp, i64, vp, vp, vp, i64, vp, i64, i64, f32, vp],
    "pz_fp8_quant_attn": [vp, i64, vp, i64, vp, i64, i64, i64, i64, vp, vp, vp, vp, vp, vp, i64, vp],
    "pz_flash_fwd_f8": [C.POINTER(FlashArgs), vp, vp, vp, vp, i64, vp, vp, i64, vp],
    "pz_fp8_absmax": [vp, i64, vp, vp],
    "pz_gemm_kernel_name": [C.POINTER(GemmArgs)],
    "pz_gemm_small": [C.POINTER(SmallGemmArgs), vp],
    "pz_rmsnorm_fwd": [vp, i64, vp, vp, i64, vp, i64, i64, f32, vp],
    "pz_rmsnorm_bwd": [vp, i64, vp, i64, vp, vp, vp, vp, i64, vp, i64, i64, vp],
    "pz_layernorm_fwd": [vp, i64, vp, vp, vp, i64, vp, vp, i64, i64, f32, vp],
    "pz_layernorm_bwd": [vp, i64, vp, i64, vp, vp, vp, vp, vp, i64, vp, vp, i64, i64, vp, vp],
    "pz_act_bwd_colsum": [vp, i64, vp, i64, vp, i64, i64, i32, vp, i64, vp, i32, vp],
    "pz_reduce_parts_multi": [vp, i32, vp],
    "pz_norm_rows_per_part": [],
    "pz_reduce_parts": [vp, i64, i64, vp, i32, vp],
    "pz_colsum": [vp, i64, i64, i64, vp, i32, vp, vp],
    "pz_batch_sum": [vp, i64, i64, i64, vp, i32, vp],
    "pz_rope_table": [vp, i64, i64, f32, vp],
    "pz_qkv_rope_split": [vp, vp, vp, vp, vp, vp, i64, i64, i64, i64, i64, i64, i64, i64, i64, vp],
    "pz_qkv_rope_split_bwd": [vp, vp, vp, vp, vp, vp, i64, i64, i64, i64, i64, i64, i64, i64, i64, vp],
    "pz_gemv_qkv_rope": [C.POINTER(QkvRopeArgs), vp],
    "pz_gemm_qkv_rope": [C.POINTER(QkvRopeArgs), vp],
    "pz_decode_attn": [C.POINTER(DecodeAttnArgs), vp],
    "pz_decode_attn_ws_bytes": [i64, i64, i64],
    "pz_attn_softmax": [C.POINTER(SoftmaxArgs), vp],
    "pz_attn_softmax_bwd": [vp, vp, i64, vp, vp, i64, i64, i64, f32, f32, vp],
    "pz_flash_fwd": [C.POINTER(FlashArgs), vp],
    "pz_flash_fwd_probs": [C.POINTER(FlashArgs), vp, vp, i64, vp],
    "pz_flash_bwd_ds": [C.POINTER(FlashArgs), vp, vp, vp, i64, vp],
    "pz_flash_bwd_prep": [C.POINTER(FlashArgs), vp],
    "pz_flash_bwd": [C.POINTER(FlashArgs), vp],
    "pz_patchify": [vp, vp, i64, i64, i64, i64, i64, vp],
    "pz_embed_merge": [vp, vp, i64, vp, vp, i64, i64, i64, i64, i64, i64, f32, f32, vp],
    "pz_embed_merge_bwd": [vp, vp, vp, i64, i64, i64, i64, i64, f32, vp],
    "pz_time_embed": [vp, vp, i64, i64, f32, i32, vp],
    "pz_concat_time": [vp, vp, vp, i64, i64, i64, vp],
    "pz_split_time_grad": [vp, vp, i64, i64, vp],
    "pz_flow_psi": [vp, vp, vp, vp, i64, i64, f32, vp],
    "pz_flow_loss": [vp, i64, i64, vp, vp, vp, vp, vp, i64, i64, i64, f32, vp],
    "pz_euler_step": [vp, vp, i64, i64, vp, i64, i64, i64, f32, vp],
    "pz_action_in": [vp, i64, vp, vp, vp, vp, i64, i64, i64, i64, f32, i32, vp],
    "pz_action_out": [vp, i64, vp, f32, vp, vp, i64, i64, vp, vp, i64, i64, f32, vp],
    "pz_copy_rows": [vp, i64, i64, vp, i64, i64, i64, i64, i64, f32, i32, vp],
    "pz_time_embed_rows": [vp, vp, i64, i64, i64, i64, f32, i32, vp],
    "pz_clamp": [vp, i64, f32, f32, vp],
    "pz_geglu_bwd": [vp, i64, vp, i64, vp, vp, i64, i64, i64, vp],
    "pz_act_bwd": [vp, i64, vp, i64, vp, vp, i64, i64, i64, i32, vp],
    "pz_adamw": [vp, vp, vp, vp, i64, f32, f32, f32, f32, f32, f32, f32, vp, vp],
    "pz_adamw8bit": [C.POINTER(AdamW8Args), vp],
    "pz_sumsq": [vp, i64, vp, vp],
    "pz_clip_coef": [vp, i64, vp, vp, f32, vp],
    "pz_fill_uniform": [vp, i32, i64, C.c_uint64, f32, f32, vp],
    "pz_cast_f32_bf16": [vp, vp, i64, vp],
    "pz_cast_bf16_f32": [vp, vp, i64, vp],
    "pz_debug_poison_lds": [C.c_uint32, vp],
    "pz_debug_spin": [i64, i64, vp],
    "pz_last_error": [],
    "pz_abi_version": [],
}
_RESTYPE = {"pz_last_error": C.c_char_p, "pz_gemm_kernel_name": C.c_char_p, "pz_norm_rows_per_part": i64,
            "pz_decode_attn_ws_bytes": i64}

_lib = None


class NativeError(RuntimeError):
    pass


def lib():
    """Load libpizero_hip.so (raises if absent: there is no non-native path)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise NativeError(
                f"{LIB_PATH} not found: build it with `python open-pi-zero_amd/build_native.py` "
                "(or __graft_entry__.build()); the Pi0 path has no CPU/eager fallback")
        L = C.CDLL(LIB_PATH)
        for name, argt in SIGNATURES.items():
            fn = getattr(L, name)
            fn.argtypes = argt
            fn.restype = _RESTYPE.get(name, C.c_int)
        if L.pz_abi_version() != ABI_VERSION:
            raise NativeError(f"{LIB_PATH}: ABI version {L.pz_abi_version()} != {ABI_VERSION}; rebuild it")
        _lib = L
    return _lib


# entry points that enqueue no kernel (everything else takes the stream as its last argument)
_NO_LAUNCH = {"pz_last_error", "pz_abi_version", "pz_gemm_kernel_name", "pz_norm_rows_per_part",
              "pz_decode_attn_ws_bytes", "pz_debug_poison_lds"}
# test instrument (tests/test_train_loop_gpu.py): with a word set, every launch is preceded on its stream by
# pz_debug_poison_lds(word), so a kernel reading LDS it did not write sees NaN.  PZ_POISON_LDS=1 turns it on
# for a whole process (0xffffffff).
_POISON_LDS = [0xFFFFFFFF if os.environ.get("PZ_POISON_LDS", "0") == "1" else None]


# debug instrument (PZ_CHECK_FINITE=1, engine._chk): names of the launches since the last finiteness check
_RECENT = [[] if os.environ.get("PZ_CHECK_FINITE", "0") == "1" else None]


def recent_launches(clear=True):
    """the entry points called since the last call of this (PZ_CHECK_FINITE=1 only; else [])"""
    r = _RECENT[0] or []
    if clear and _RECENT[0] is not None:
        _RECENT[0] = []
    return r


def set_poison_lds(word):
    """word (e.g. 0xffffffff) or None: poison every CU's LDS before each kernel launch (test instrument)"""
    _POISON_LDS[0] = None if word is None else int(word) & 0xFFFFFFFF


def call(name, *args):
    if _POISON_LDS[0] is not None and name not in _NO_LAUNCH:
        rc = lib().pz_debug_poison_lds(_POISON_LDS[0], args[-1])
        if rc != 0:
            raise NativeError(f"pz_debug_poison_lds failed (rc={rc}): {lib().pz_last_error().decode(errors='replace')}")
    if _RECENT[0] is not None:
        _RECENT[0].append(name)
    rc = getattr(lib(), name)(*args)
    if rc != 0:
        msg = lib().pz_last_error().decode(errors="replace")
        raise NativeError(f"{name} failed (rc={rc}): {msg}")
    return rc
