"""A/B of the GEMM planner on the training step's smaller shapes (micro-batch 256), hipGraph-timed per launch:
  - the joint attention backward's batched dK = dS^T Q and dV = P_g^T dO_g (TN, one 288 x 256 output per sample,
    K = 2208 vlm rows x heads, 40 action rows x heads accumulated with beta; engine.py joint backward);
  - the action expert's 1280-row GEMMs (256 samples x 5 tokens): forward NT, dgrad NN, wgrad TN.

    python tools/attn_gemm_ab.py [--n 20]
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

B, LP, HD = 256, 288, 256
# name, M, N, K, a_kc, b_kc, beta, batch
SHAPES = [
    ("dK / dV vlm", LP, HD, 2208, False, False, False, B),
    ("dV action", LP, HD, 40, False, False, True, B),
    ("act fwd q|k|v", 1280, 2560, 1024, True, True, False, 1),
    ("act fwd o", 1280, 1024, 2048, True, True, False, 1),
    ("act fwd down", 1280, 1024, 4096, True, True, False, 1),
    ("act dgrad q|k|v", 1280, 1024, 2560, True, False, False, 1),
    ("act dgrad gate|up", 1280, 1024, 8192, True, False, False, 1),
    ("act dgrad o", 1280, 2048, 1024, True, False, False, 1),
    ("act wgrad gate|up", 8192, 1024, 1280, False, False, False, 1),
    ("act wgrad down", 1024, 4096, 1280, False, False, False, 1),
    ("act wgrad q|k|v", 2560, 1024, 1280, False, False, False, 1),
    ("act wgrad o", 1024, 2048, 1280, False, False, False, 1),
]
VARIANTS = [("default", {}), ("no tail", {"PZ_GEMM_TAIL": "0"}), ("128-tile", {"PZ_GEMM_256_MINM": "1000000"}),
            ("256 any", {"PZ_GEMM_256_MINM": "1", "PZ_GEMM_256_MINUNITS": "1"}),
            ("256 any, no tail", {"PZ_GEMM_256_MINM": "1", "PZ_GEMM_256_MINUNITS": "1", "PZ_GEMM_TAIL": "0"}),
            ("256 N>=256", {"PZ_GEMM_256_MINM": "1", "PZ_GEMM_256_MINN": "256"})]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=20)
    a = ap.parse_args()
    dev = "cuda"
    for name, M, N, K, akc, bkc, beta, bat in SHAPES:
        # per-sample operands laid out as the engine's: A = [bat][K][M] (k-strided), B = [bat][K][N]
        A = torch.randn(bat * M * K, device=dev).to(torch.bfloat16)
        Bm = (torch.randn(bat * N * K, device=dev) * K ** -0.5).to(torch.bfloat16)
        C = torch.zeros(bat * M * N, device=dev, dtype=torch.bfloat16)
        lda, ldb = (K if akc else M), (K if bkc else N)
        kw = dict(batch=bat, sA=(M * K, 0), sB=(N * K, 0), sC=(M * N, 0)) if bat > 1 else {}

        def run():
            ops.gemm(M, N, K, A, lda, akc, Bm, ldb, bkc, C, N, beta=beta, **kw)

        res = []
        for label, env in VARIANTS:
            os.environ.update(env)
            try:
                kn = ops.gemm_kernel_name(M, N, K, a_kc=akc, b_kc=bkc, batch=bat)
                t = graph_us(run, a.n)
                res.append(f"{label} {t:7.2f} us {2.0 * bat * M * N * K / t / 1e6:6.1f} TF/s [{kn}]")
            finally:
                for k in env:
                    os.environ.pop(k)
        print(f"{name:18s} {bat}x{M}x{N}x{K}:\n    " + "\n    ".join(res), flush=True)


if __name__ == "__main__":
    main()
