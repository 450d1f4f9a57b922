"""Row-slab GEMM (gemm_rows_kernel) vs the previous planner choice on the 64 < M <= 512 forward shapes
(B = 1 SigLIP / Gemma prefill, the action expert's 320 training rows), hipGraph-timed per launch (HIP events),
over the kernel's A/B knobs (PZ_ROWS_W, PZ_ROWS_TNB).

    python tools/rows_bench.py [--n 100]
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

SHAPES = [  # name, M, N, K, epilogue, bias, resid
    ("sig qkv", 256, 3456, 1152, PZ_EPI_NONE, True, False),
    ("sig o", 256, 1152, 1152, PZ_EPI_NONE, True, True),
    ("sig fc1", 256, 4304, 1152, PZ_EPI_GELU, True, False),
    ("sig fc2", 256, 1152, 4304, PZ_EPI_NONE, True, True),
    ("vlm qkv", 276, 2560, 2048, PZ_EPI_NONE, False, False),
    ("vlm o", 276, 2048, 2048, PZ_EPI_NONE, False, True),
    ("vlm gate|up", 276, 32768, 2048, PZ_EPI_GEGLU, False, False),
    ("vlm down", 276, 2048, 16384, PZ_EPI_NONE, False, True),
    ("act qkv", 320, 2560, 1024, PZ_EPI_NONE, False, False),
    ("act o", 320, 1024, 2048, PZ_EPI_NONE, False, True),
    ("act gate|up", 320, 8192, 1024, PZ_EPI_GEGLU, False, False),
    ("act down", 320, 1024, 4096, PZ_EPI_NONE, False, True),
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
        res = []
        for label, env in [("old", {"PZ_GEMM_ROWS": "0"}), ("default", {}), ("rows", {"PZ_ROWS_FIRST": "1", "PZ_GEMM_ROWS": "1"}),
                           ("rows w4", {"PZ_ROWS_FIRST": "1", "PZ_GEMM_ROWS": "1", "PZ_ROWS_W": "4"}),
                           ("rows w8", {"PZ_ROWS_FIRST": "1", "PZ_GEMM_ROWS": "1", "PZ_ROWS_W": "8"}),
                           ("rows tnb1", {"PZ_ROWS_FIRST": "1", "PZ_GEMM_ROWS": "1", "PZ_ROWS_TNB": "1"}),
                           ("rows tnb2", {"PZ_ROWS_FIRST": "1", "PZ_GEMM_ROWS": "1", "PZ_ROWS_TNB": "2"}),
                           ("rows tnb4", {"PZ_ROWS_FIRST": "1", "PZ_GEMM_ROWS": "1", "PZ_ROWS_TNB": "4"}),
                           ("rows tmb2", {"PZ_ROWS_FIRST": "1", "PZ_GEMM_ROWS": "1", "PZ_ROWS_TMB": "2"}),
                           ("rows tmb2 tnb2", {"PZ_ROWS_FIRST": "1", "PZ_GEMM_ROWS": "1", "PZ_ROWS_TMB": "2",
                                               "PZ_ROWS_TNB": "2"})]:
            os.environ.update(env)
            kn = ops.gemm_kernel_name(M, N, K, epi=epi, **gi)
            ref = None
            if label == "old":
                run()
                ref = out.float().clone()
            run()
            torch.cuda.synchronize()
            t = graph_us(run, a.n)
            err = 0.0 if ref is None else (out.float() - ref).abs().max().item()
            res.append(f"{label} {t:7.2f} us ({fl / t / 1e6:5.0f} TF/s) [{kn}]")
            for k in env:
                os.environ.pop(k)
        print(f"{name:12s} {M}x{N}x{K}: " + " | ".join(res), flush=True)


if __name__ == "__main__":
    main()
