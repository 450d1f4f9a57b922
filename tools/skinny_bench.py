"""Few-row GEMM shapes of the C5 denoise step (50 action rows x the action-expert Linears) timed in a
hipGraph (per-launch us, HIP events), over the skinny-64 kernel's A/B knobs (PZ_SK64_NC / PZ_SK64_W)
and bf16 vs fp8 weights.

    python tools/skinny_bench.py [--rows 50]
"""

import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "open-pi-zero_amd"))

import torch  # noqa: E402

from pizero_native import ops  # noqa: E402
from pizero_native.ops import PZ_EPI_GEGLU, PZ_EPI_NONE  # noqa: E402
from tools.launch_floor import graph_us  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=50)
    ap.add_argument("--n", type=int, default=100)
    a = ap.parse_args()
    M = a.rows
    dev = "cuda"
    shapes = [("qkv", 2560, 1024, PZ_EPI_NONE), ("o", 1024, 2048, PZ_EPI_NONE), ("gate|up", 8192, 1024, PZ_EPI_GEGLU),
              ("down", 1024, 4096, PZ_EPI_NONE)]
    if a.rows > 64:  # B=1 SigLIP prefill shapes (256 rows / image): row-chunked skinny-64 vs the tile path
        shapes = [("sig qkv", 3456, 1152, PZ_EPI_NONE), ("sig o", 1152, 1152, PZ_EPI_NONE),
                  ("sig fc1", 4304, 1152, PZ_EPI_NONE), ("sig fc2", 1152, 4352, PZ_EPI_NONE),
                  ("vlm o", 2048, 2048, PZ_EPI_NONE), ("vlm qkv", 2560, 2048, PZ_EPI_NONE)]
        for name, N, K, epi in shapes:
            x = (torch.randn(M, K, device=dev)).to(torch.bfloat16)
            W = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
            out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            os.environ.pop("PZ_SK64_MAXM", None)
            t0 = graph_us(lambda: ops.linear(x, W, out), a.n)
            n0 = ops.gemm_kernel_name(M, N, K)
            os.environ["PZ_SK64_MAXM"] = str(M)
            t1 = graph_us(lambda: ops.linear(x, W, out), a.n)
            n1 = ops.gemm_kernel_name(M, N, K)
            os.environ.pop("PZ_SK64_MAXM")
            os.environ["PZ_GEMM_256_MINM"], os.environ["PZ_GEMM_256_MINUNITS"] = "1", "1"
            t2 = graph_us(lambda: ops.linear(x, W, out), a.n)
            n2 = ops.gemm_kernel_name(M, N, K)
            os.environ.pop("PZ_GEMM_256_MINM")
            os.environ.pop("PZ_GEMM_256_MINUNITS")
            print(f"{name:8s} M={M} N={N} K={K}: default {t0:7.2f} us ({n0})   row-chunked {t1:7.2f} us ({n1})   "
                  f"256-tile {t2:7.2f} us ({n2})")
        return
    for name, N, K, epi in shapes:
        x = (torch.randn(M, K, device=dev)).to(torch.bfloat16)
        W = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
        out = torch.empty(M, N // 2 if epi == PZ_EPI_GEGLU else N, device=dev, dtype=torch.bfloat16)
        s = ops.fp8_weight_scale(W)
        q = torch.empty(N, K, device=dev, dtype=torch.uint8)
        ops.fp8_quant_tensor(W, q, s)
        mb = N * K * 2 / 1e6
        for nc in ("4", "8", "16"):
            for w in ("4", "8"):
                os.environ["PZ_SK64_NC"], os.environ["PZ_SK64_W"] = nc, w
                t16 = graph_us(lambda: ops.linear(x, W, out, epi=epi), a.n)
                t8 = graph_us(lambda: ops.linear_fp8(x, q, s, out, epi=epi), a.n)
                print(f"{name:8s} M={M} N={N} K={K} NC={nc:2s} W={w}: bf16 {t16:7.2f} us ({mb * 1e3 / t16:6.0f} GB/s)"
                      f"  fp8 {t8:7.2f} us ({mb * 0.5e3 / t8:6.0f} GB/s)")
        os.environ.pop("PZ_SK64_NC")
        os.environ.pop("PZ_SK64_W")


if __name__ == "__main__":
    main()
