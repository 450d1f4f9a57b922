"""A/B of the GEMM planner's knobs on the action expert's backward shapes (M = 320 rows = 64 samples x 5
tokens): dgrad (NN: B k-strided) and the short-K wgrad (TN: K = 320, bf16 gradient accumulated with beta),
hipGraph-timed per launch (HIP events).

    python tools/shape_ab.py [--n 50]
"""

import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "open-pi-zero_amd"))

import torch  # noqa: E402

from pizero_native import ops  # noqa: E402
from tools.launch_floor import graph_us  # noqa: E402

# name, M, N, K, a_kc, b_kc, beta (the census layouts: NN = dgrad, TN = wgrad)
SHAPES = [
    ("dgrad gate|up", 320, 1024, 8192, True, False, False),
    ("dgrad down", 320, 4096, 1024, True, False, False),
    ("dgrad qkv", 320, 1024, 2560, True, False, False),
    ("dgrad o", 320, 2048, 1024, True, False, False),
    ("wgrad gate|up", 8192, 1024, 320, False, False, True),
    ("wgrad down", 1024, 4096, 320, False, False, True),
    ("wgrad qkv", 2560, 1024, 320, False, False, True),
    ("wgrad o", 1024, 2048, 320, False, False, True),
]
VARIANTS = [("default", {}), ("no tail", {"PZ_GEMM_TAIL": "0"}), ("128-tile", {"PZ_GEMM_256_MINM": "1000000"}),
            ("256 any", {"PZ_GEMM_256_MINM": "1", "PZ_GEMM_256_MINUNITS": "1"}),
            ("256 any, no tail", {"PZ_GEMM_256_MINM": "1", "PZ_GEMM_256_MINUNITS": "1", "PZ_GEMM_TAIL": "0"}),
            ("no split-K", {"PZ_SPLITK": "0", "PZ_GEMM_256_MINM": "1000000"})]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=50)
    a = ap.parse_args()
    dev = "cuda"
    for name, M, N, K, akc, bkc, beta in SHAPES:
        A = torch.randn(M * K, device=dev).to(torch.bfloat16)
        B = (torch.randn(N * K, device=dev) * K ** -0.5).to(torch.bfloat16)
        C = torch.zeros(M, N, device=dev, dtype=torch.bfloat16)
        lda, ldb = (K if akc else M), (K if bkc else N)

        def run():
            ops.gemm(M, N, K, A, lda, akc, B, ldb, bkc, C, N, beta=beta)

        res = []
        for label, env in VARIANTS:
            os.environ.update(env)
            kn = ops.gemm_kernel_name(M, N, K, a_kc=akc, b_kc=bkc)
            t = graph_us(run, a.n)
            res.append(f"{label} {t:7.2f} us [{kn}]")
            for k in env:
                os.environ.pop(k)
        print(f"{name:14s} {M}x{N}x{K}: " + " | ".join(res), flush=True)


if __name__ == "__main__":
    main()
