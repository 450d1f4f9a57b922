"""Microbenchmark: pz_gemm (all layouts; split tail on/off) vs torch.matmul (hipBLASLt) on the Pi0 training shapes.

    python tools/gemm_bench.py [--iters 20]
Random bf16 operands (uniform [-1,1)), interleaved A/B timing in one process.
"""

import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "open-pi-zero_amd"))

import torch  # noqa: E402

from pizero_native import ops  # noqa: E402

SHAPES = [  # (name, M, N, K)
    ("vlm_geglu_fwd", 17664, 32768, 2048),
    ("vlm_qkv_fwd", 17664, 2560, 2048),
    ("vlm_down_fwd", 17664, 2048, 16384),
    ("vlm_o_fwd", 17664, 2048, 2048),
    ("sig_fc1_fwd", 16384, 4304, 1152),
    ("sig_fc2_fwd", 16384, 1152, 4304),
    ("sig_qkv_fwd", 16384, 3456, 1152),
]


def timeit(fn, iters):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    dev = "cuda"
    rnd = lambda *s: (torch.rand(*s, device=dev) * 2 - 1).to(torch.bfloat16)  # noqa: E731
    print(f"{'shape':16s} {'layout':6s} {'M':>6} {'N':>6} {'K':>6} {'8ph TF/s':>9} {'notail':>9} {'torch TF/s':>10}")

    def ab(fn):
        """time fn with and without the 8-phase split tail (pz_gemm reads PZ_GEMM_TAIL per call)"""
        a = timeit(fn, args.iters)
        os.environ["PZ_GEMM_TAIL"] = "0"
        b = timeit(fn, args.iters)
        os.environ.pop("PZ_GEMM_TAIL")
        return a, b

    for name, M, N, K in SHAPES:
        fl = 2.0 * M * N * K
        x, w = rnd(M, K), rnd(N, K)
        out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
        if "geglu" in name:
            t, t2 = ab(lambda: ops.linear(x, w, out[:, : N // 2], epi=ops.PZ_EPI_GEGLU))
        else:
            t, t2 = ab(lambda: ops.linear(x, w, out))
        tt = timeit(lambda: torch.matmul(x, w.t()), args.iters)
        print(f"{name:16s} {'NT':6s} {M:6d} {N:6d} {K:6d} {fl / t / 1e9:9.1f} {fl / t2 / 1e9:9.1f} {fl / tt / 1e9:10.1f}")
        # dgrad: dx[M,K] = dy[M,N] W[N,K]
        dy = rnd(M, N)
        dx = torch.empty(M, K, device=dev, dtype=torch.bfloat16)
        t, t2 = ab(lambda: ops.linear_dgrad(dy, w, dx))
        tt = timeit(lambda: torch.matmul(dy, w), args.iters)
        print(f"{name:16s} {'NN':6s} {M:6d} {K:6d} {N:6d} {fl / t / 1e9:9.1f} {fl / t2 / 1e9:9.1f} {fl / tt / 1e9:10.1f}")
        dW = torch.empty(N, K, device=dev, dtype=torch.bfloat16)
        t, t2 = ab(lambda: ops.linear_wgrad(dy, x, dW))
        tt = timeit(lambda: torch.matmul(dy.t(), x), args.iters)
        print(f"{name:16s} {'TN':6s} {N:6d} {K:6d} {M:6d} {fl / t / 1e9:9.1f} {fl / t2 / 1e9:9.1f} {fl / tt / 1e9:10.1f}", flush=True)
        del x, w, out, dy, dx, dW
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
