"""Tall-tile GEMM (gemm_tall_kernel, PZ_GEMM_TALL=1) vs the default planner choice on the 64 < M <= 1024 forward
shapes (B = 1 SigLIP / Gemma prefill, C5's 788-row prefill, the action expert's 320 training rows), hipGraph-timed
per launch (HIP events); the outputs of the two paths are compared (max |diff|).

    python tools/tall_bench.py [--n 100]
"""

import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "open-pi-zero_amd"))

import torch  # noqa: E402

from pizero_native import ops  # noqa: E402
from pizero_native.ops import PZ_EPI_GEGLU, PZ_EPI_GELU, PZ_EPI_NONE  # noqa: E402
from tools.launch_floor import graph_us  # noqa: E402
from tools.rows_bench import SHAPES as ROW_SHAPES  # noqa: E402

SHAPES = ROW_SHAPES + [
    ("c5 sig fc1", 768, 4304, 1152, PZ_EPI_GELU, True, False),
    ("c5 sig fc2", 768, 1152, 4304, PZ_EPI_NONE, True, True),
    ("c5 gate|up", 789, 32768, 2048, PZ_EPI_GEGLU, False, False),
    ("c5 down", 789, 2048, 16384, PZ_EPI_NONE, False, True),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=100)
    a = ap.parse_args()
    dev = "cuda"
    for name, M, N, K, epi, hb, hr in SHAPES:
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        W = (torch.randn(N, K, device=dev) * K ** -0.5).to(torch.bfloat16)
        b = torch.randn(N, device=dev).to(torch.bfloat16) if hb else None
        no = N // 2 if epi == PZ_EPI_GEGLU else N
        r = torch.randn(M, no, device=dev).to(torch.bfloat16) if hr else None
        out = torch.empty(M, no, device=dev, dtype=torch.bfloat16)
        aux = torch.empty(M, N, device=dev, dtype=torch.bfloat16) if epi != PZ_EPI_NONE else None
        gi = dict(geglu_inter=N // 2) if epi == PZ_EPI_GEGLU else {}

        def run():
            ops.linear(x, W, out, bias=b, resid=r, epi=epi, aux=aux)

        fl = 2 * M * N * K
        wb = N * K * 2
        res, outs = [], []
        variants = [("default", {"PZ_GEMM_TALL": "0"}), ("tall", {"PZ_GEMM_TALL": "1"})]
        for label, env in variants:
            os.environ.update(env)
            try:
                kn = ops.gemm_kernel_name(M, N, K, epi=epi, **gi)
                if label.startswith("tall") and not kn.startswith("gemm_tall"):
                    res.append(f"{label} n/a [{kn}]")
                    continue
                run()
                torch.cuda.synchronize()
                outs.append(out.float().clone())
                t = graph_us(run, a.n)
                res.append(f"{label} {t:7.2f} us ({fl / t / 1e6:5.0f} TF/s, {wb / t / 1e3:5.0f} GB/s wts) [{kn}]")
            finally:
                for k in env:
                    os.environ.pop(k)
        d = max((o - outs[0]).abs().max().item() for o in outs[1:]) if len(outs) > 1 else 0.0
        print(f"{name:12s} {M}x{N}x{K}: " + " | ".join(res) + f" | max|d| {d:.3g}", flush=True)
    main_nn(a.n)


NN_SHAPES = [  # dgrad layout (B = W [K][N] k-strided): the action expert's 320 training rows
    ("act dgate|up", 320, 1024, 8192), ("act ddown", 320, 4096, 1024), ("act do", 320, 2048, 1024),
    ("act dqkv", 320, 1024, 2560),
]


def main_nn(n):
    dev = "cuda"
    for name, M, N, K in NN_SHAPES:
        dy = torch.randn(M, K, device=dev).to(torch.bfloat16)
        W = (torch.randn(K, N, device=dev) * K ** -0.5).to(torch.bfloat16)
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)

        def run():
            ops.gemm(M, N, K, dy, K, True, W, N, False, out, N)

        res, outs = [], []
        for label, env in [("default", {"PZ_GEMM_TALL": "0"}), ("tall", {"PZ_GEMM_TALL": "1"})]:
            os.environ.update(env)
            kn = ops.gemm_kernel_name(M, N, K, b_kc=False)
            run()
            torch.cuda.synchronize()
            outs.append(out.float().clone())
            t = graph_us(run, n)
            res.append(f"{label} {t:7.2f} us ({2 * M * N * K / t / 1e6:5.0f} TF/s) [{kn}]")
            os.environ.pop("PZ_GEMM_TALL")
        d = (outs[0] - outs[1]).abs().max().item()
        print(f"{name:12s} NN {M}x{N}x{K}: " + " | ".join(res) + f" | max|d| {d:.3g}", flush=True)


if __name__ == "__main__":
    main()
