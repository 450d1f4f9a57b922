"""Per-launch floor inside a hipGraph: N back-to-back launches of tiny kernels, replayed, timed with
HIP events (no profiler).  Compares the library's small kernels with a torch elementwise kernel.

    python tools/launch_floor.py [--n 500]
"""

import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "open-pi-zero_amd"))

import torch  # noqa: E402

from pizero_native import ops  # noqa: E402


def graph_us(fn, n, reps=5):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(n):
            fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (reps * n)


def eager_us(fn, n, reps=3):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps * n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (reps * n)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=500)
    a = ap.parse_args()
    dev = "cuda"
    x = torch.randn(4, 1024, device=dev).to(torch.bfloat16)
    y = torch.empty_like(x)
    t = torch.zeros(16, device=dev)
    res = {}
    res["torch add_ (16 fp32)"] = graph_us(lambda: t.add_(1.0), a.n)
    res["torch add_ (16 fp32), eager"] = eager_us(lambda: t.add_(1.0), a.n)
    res["pz_copy_rows 4x1024"] = graph_us(lambda: ops.copy_rows(x, 1024, 0, y, 1024, 0, 1, 4, 1024), a.n)
    tt = torch.rand(1, device=dev)
    te = torch.empty(1, 1024, device=dev, dtype=torch.bfloat16)
    res["pz_time_embed 1x1024"] = graph_us(lambda: ops.time_embed(tt, te, 100.0), a.n)
    res["pz_time_embed 1x1024, eager"] = eager_us(lambda: ops.time_embed(tt, te, 100.0), a.n)
    for (N, K) in ((1024, 2048), (1024, 4096), (2560, 1024), (8192, 1024)):
        W = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
        xa = torch.randn(4, K, device=dev).to(torch.bfloat16)
        out = torch.empty(4, N, device=dev, dtype=torch.bfloat16)
        us = graph_us(lambda: ops.linear(xa, W, out), a.n // 5)
        res[f"skinny 4x{N}x{K} ({N * K * 2 / 1e6:.1f} MB)"] = us
        res[f"  -> GB/s {N}x{K}"] = N * K * 2 / (us * 1e-6) / 1e9
    for k, v in res.items():
        print(f"{k:40s} {v:8.2f}")


if __name__ == "__main__":
    main()
