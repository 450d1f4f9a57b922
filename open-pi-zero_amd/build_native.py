"""Build libpizero_hip.so in-tree for gfx950 (hipcc, no cmake, no JIT cache).

    python open-pi-zero_amd/build_native.py [--force]

Objects are rebuilt only when their source/header is newer.  The shared
library lands next to this file (open-pi-zero_amd/libpizero_hip.so) so it
travels to the GPU box with the repo snapshot.
"""

from __future__ import annotations

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libpizero_hip.so")
BUILD = os.path.join(HERE, "build")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = "gfx950"
SOURCES = ["pz_gemm.hip", "pz_gemm_rows.hip", "pz_gemm_tall.hip", "pz_norm.hip", "pz_attn.hip", "pz_misc.hip", "pz_flash.hip", "pz_optim.hip", "pz_gemv.hip", "pz_decode.hip", "pz_quant.hip"]
HEADERS = [os.path.join(CSRC, "pz_common.h"), os.path.join(CSRC, "pz_gemm_epi.h"), os.path.join(ROOT, "include", "pz_abi.h")]
FLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wno-unused-result",
         "-Wno-unused-value", "-munsafe-fp-atomics"]
# per-file extra flags: the 8-bit optimizer is held bit-exact to its float32 oracle, so no FMA contraction
FILE_FLAGS = {"pz_optim.hip": ["-ffp-contract=off"]}


def _needs(obj: str, deps: list[str]) -> bool:
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(d) > t for d in deps)


def _compile(src: str, force: bool) -> str:
    s = os.path.join(CSRC, src)
    obj = os.path.join(BUILD, src.replace(".hip", ".o"))
    if force or _needs(obj, [s] + HEADERS):
        cmd = [HIPCC, *FLAGS, *FILE_FLAGS.get(src, []), "-c", s, "-o", obj]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr}")
    return obj


def build(force: bool = False, verbose: bool = True) -> str:
    os.makedirs(BUILD, exist_ok=True)
    with ThreadPoolExecutor(max_workers=min(4, os.cpu_count() or 1)) as ex:
        objs = list(ex.map(lambda s: _compile(s, force), SOURCES))
    if force or _needs(OUT, objs):
        cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", *objs, "-o", OUT]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr}")
    if verbose:
        print("built", OUT)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
