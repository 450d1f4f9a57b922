"""Run one pz_gemm shape/layout a few times (for rocprofv3 counter passes).

    python tools/gemm_one.py --layout TN --M 17664 --N 2048 --K 2048 [--variant 8phase|2stage] [--iters 5]
M, N, K = the forward nn.Linear shape; layouts NT (fwd), NN (dgrad), TN (wgrad) as in tools/gemm_bench.py;
GEGLU = the vlm gate|up GEMM with the GeGLU epilogue and saved g|u (N = 2 * intermediate); DGEGLU = the down-proj
dgrad with the GeGLU derivative (M x N x K = tokens x hidden x intermediate, e.g. --M 70656 --N 2048 --K 16384).
"""

import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "open-pi-zero_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layout", default="NT")
    ap.add_argument("--M", type=int, default=17664)
    ap.add_argument("--N", type=int, default=2048)
    ap.add_argument("--K", type=int, default=2048)
    ap.add_argument("--variant", default="8phase")
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--notail", action="store_true", help="PZ_GEMM_TAIL=0: whole tiles only")
    a = ap.parse_args()
    os.environ["PZ_GEMM_BIG"] = a.variant
    if a.notail:
        os.environ["PZ_GEMM_TAIL"] = "0"
    from pizero_native import ops

    dev = "cuda"
    rnd = lambda *s: (torch.rand(*s, device=dev) * 2 - 1).to(torch.bfloat16)  # noqa: E731
    M, N, K = a.M, a.N, a.K  # forward shape: y[M,N] = x[M,K] W[N,K]^T
    x, w, dy = rnd(M, K), rnd(N, K), rnd(M, N)
    y = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    dx = torch.empty(M, K, device=dev, dtype=torch.bfloat16)
    dW = torch.empty(N, K, device=dev, dtype=torch.bfloat16)
    if a.layout == "DGEGLU":  # the vlm down-proj dgrad with the GeGLU derivative: reads g|u, writes d(g|u) in place
        gu = rnd(M, 2 * K)
        fn = lambda: ops.linear_dgrad(dy, w, gu, epi=ops.PZ_EPI_DGEGLU, aux=gu)  # noqa: E731
    elif a.layout == "GEGLU":  # the bench's dominant launch: gate|up GEMM + GeGLU, saved g|u (engine.py)
        hm = torch.empty(M, N // 2, device=dev, dtype=torch.bfloat16)
        fn = lambda: ops.linear(x, w, hm, epi=ops.PZ_EPI_GEGLU, aux=y)  # noqa: E731
    else:
        fn = {"NT": lambda: ops.linear(x, w, y), "NN": lambda: ops.linear_dgrad(dy, w, dx),
              "TN": lambda: ops.linear_wgrad(dy, x, dW)}[a.layout]
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(2):
        fn()
    e0.record()
    for _ in range(a.iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.iters
    print(f"{a.layout} {a.variant} M={M} N={N} K={K}: {ms:.3f} ms {2.0 * M * N * K / ms / 1e9:.1f} TF/s", flush=True)


if __name__ == "__main__":
    main()
