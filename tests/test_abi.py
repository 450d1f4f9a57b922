"""The C-ABI library loads without a GPU and exports every symbol include/pz_abi.h declares."""

import os
import re

from tests.conftest import ROOT


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "pz_abi.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(pz_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_entry_points():
    syms = declared_symbols()
    assert "pz_gemm" in syms and "pz_attn_softmax" in syms and "pz_adamw" in syms
    assert len(syms) >= 30


def test_library_exports_all_declared_symbols():
    import pizero_native
    from pizero_native._lib import SIGNATURES

    L = pizero_native.lib()
    for s in declared_symbols():
        assert hasattr(L, s), s
        assert s in SIGNATURES, f"{s} has no ctypes signature"
    from pizero_native._lib import ABI_VERSION

    hdr = open(os.path.join(ROOT, "include", "pz_abi.h")).read()
    assert f"#define PZ_ABI_VERSION {ABI_VERSION}" in hdr
    assert L.pz_abi_version() == ABI_VERSION


def test_error_path_without_gpu():
    """A host-side argument check fails before any launch and reports a message."""
    import ctypes

    import pizero_native
    from pizero_native._lib import GemmArgs

    a = GemmArgs()
    rc = pizero_native.lib().pz_gemm(ctypes.byref(a), None)
    assert rc == 1
    assert b"bad dims" in pizero_native.lib().pz_last_error()


def test_gemm_planner_routes_without_gpu():
    """pz_gemm_kernel_name is host logic (no device needed): the row-slab kernel takes the measured-faster
    64 < M <= 512 forward shapes (pz_gemm.hip plan_rows), the tile kernels keep the rest."""
    from pizero_native import ops

    geglu = ops.PZ_EPI_GEGLU
    assert ops.gemm_kernel_name(256, 3456, 1152).startswith("gemm_rows_kernel<8, 4, 4")  # B=1 SigLIP q|k|v
    assert ops.gemm_kernel_name(320, 8192, 1024, epi=geglu, geglu_inter=4096).startswith("gemm_rows_kernel<4")
    assert not ops.gemm_kernel_name(256, 4304, 1152).startswith("gemm_rows")  # SigLIP fc1
    assert not ops.gemm_kernel_name(256, 1152, 4304).startswith("gemm_rows")  # SigLIP fc2
    assert not ops.gemm_kernel_name(276, 32768, 2048, epi=geglu, geglu_inter=16384).startswith("gemm_rows")
    # tall-tile kernel where it measured faster: B = 1 Gemma down, SigLIP fc2; not the B = 1 gate|up (slower inside
    # the chunk), not the action expert's 320-row down (K = 4096), not C5's 788 rows, not the training rows
    assert ops.gemm_kernel_name(276, 32768, 2048, epi=geglu, geglu_inter=16384).startswith("gemm8p_kernel")
    assert ops.gemm_kernel_name(276, 2048, 16384).startswith("gemm_tall_kernel<5, 2")
    assert ops.gemm_kernel_name(256, 1152, 4304).startswith("gemm_tall_kernel<4, 2")
    assert not ops.gemm_kernel_name(320, 1024, 4096).startswith("gemm_tall")
    assert not ops.gemm_kernel_name(789, 32768, 2048, epi=geglu, geglu_inter=16384).startswith("gemm_tall")
    assert not ops.gemm_kernel_name(35328, 2048, 16384).startswith("gemm_tall")
    assert not ops.gemm_kernel_name(64, 1024, 1024).startswith("gemm_rows")  # few-row paths keep M <= 64
    assert not ops.gemm_kernel_name(17664, 2560, 2048).startswith("gemm_rows")  # training rows: 8-phase
    assert not ops.gemm_kernel_name(320, 1024, 2048, a_kc=False).startswith("gemm_rows")  # k-strided A
    assert ops.gemm_kernel_name(16384, 1152, 1152).startswith("gemm8p_kernel")
    # fewer 256-tiles than CUs at K <= 4096 and >= 1024 rows (the action expert at micro-batch 256): 128-tile kernel
    assert ops.gemm_kernel_name(1280, 2560, 1024).startswith("gemm_kernel<")
    assert ops.gemm_kernel_name(8192, 1024, 1280, a_kc=False, b_kc=False).startswith("gemm_kernel<")
    assert ops.gemm_kernel_name(1280, 1024, 8192, b_kc=False).startswith("gemm8k_kernel")  # K 8192: 256 + tail
