"""Memory-bound kernels of the training backward at micro-batch 256, hipGraph-timed per launch, with the
algorithmic HBM bytes and the rate: Gemma RMSNorm backward (70656 x 2048, residual gradient), SigLIP LayerNorm
backward (65536 x 1152, residual gradient, dw / db / dx column-sum partials), SigLIP fc1 GELU backward + bias
column sums (65536 x 4304), timed twice (round 5 measured the norm backward with one row ahead instead of two:
LayerNorm 138.1 vs 131.5 us, profiles/r05/norm_bench.log; that variant is no longer built).

    python tools/norm_bench.py [--n 20]
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

BF16, F32 = torch.bfloat16, torch.float32


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=20)
    a = ap.parse_args()
    dev = "cuda"
    rpp = ops.rows_per_part()
    cases = []

    R, D = 70656, 2048
    x, dy, dr = (torch.randn(R, D, device=dev).to(BF16) for _ in range(3))
    w = torch.randn(D, device=dev).to(BF16)
    rstd = torch.rand(R, device=dev) + 0.5
    dx = torch.empty(R, D, device=dev, dtype=BF16)
    part = torch.empty((R + rpp - 1) // rpp, D, device=dev, dtype=F32)
    cases.append(("rmsnorm_bwd 70656x2048", lambda: ops.rmsnorm_bwd(dy, x, w, rstd, dx, dres=dr, dw_part=part),
                  4 * R * D * 2 + part.numel() * 4))
    cases.append(("rmsnorm_fwd 70656x2048", lambda: ops.rmsnorm(x, w, dx, rstd, 1e-6), 2 * R * D * 2))

    R2, D2 = 65536, 1152
    x2, dy2, dr2 = (torch.randn(R2, D2, device=dev).to(BF16) for _ in range(3))
    w2, b2 = torch.randn(D2, device=dev).to(BF16), torch.randn(D2, device=dev).to(BF16)
    mean2, rstd2 = torch.randn(R2, device=dev), torch.rand(R2, device=dev) + 0.5
    dx2 = torch.empty(R2, D2, device=dev, dtype=BF16)
    P2 = (R2 + rpp - 1) // rpp
    pw, pb, px = (torch.empty(P2, D2, device=dev, dtype=F32) for _ in range(3))
    cases.append(("layernorm_bwd 65536x1152", lambda: ops.layernorm_bwd(dy2, x2, w2, mean2, rstd2, dx2, dres=dr2,
                                                                         dw_part=pw, db_part=pb, dx_part=px),
                  4 * R2 * D2 * 2 + 3 * P2 * D2 * 4))

    R3, N3 = 65536, 4304
    dh, pre = torch.randn(R3, N3, device=dev).to(BF16), torch.randn(R3, N3, device=dev).to(BF16)
    ws = torch.empty(1024, N3, device=dev, dtype=F32)
    db = torch.empty(N3, device=dev, dtype=BF16)
    cases.append(("gelu_bwd_colsum 65536x4304", lambda: ops.act_bwd_colsum(dh, pre, dh, ops.PZ_EPI_GELU, ws, db),
                  3 * R3 * N3 * 2))

    for name, fn, nbytes in cases:
        res = []
        for label, env in (("run 1", {}), ("run 2", {})):
            os.environ.update(env)
            try:
                t = graph_us(fn, a.n)
            finally:
                for k in env:
                    os.environ.pop(k)
            res.append(f"{label} {t:7.1f} us {nbytes / t / 1e6:5.2f} TB/s")
        print(f"{name:28s} {nbytes / 1e6:7.1f} MB: " + " | ".join(res), flush=True)


if __name__ == "__main__":
    main()
