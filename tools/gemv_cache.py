"""Denoise GEMV launches (C4, B=1) with cache-resident vs HBM-streamed weights, inside a hipGraph
(measurement tool).

    python tools/gemv_cache.py [--reps 64]

A graph of --reps back-to-back launches of one action-expert projection is replayed; "warm" reuses ONE
weight tensor (it stays in L2 / the Infinity Cache after the first launch), "cold" cycles through --reps
distinct copies whose total exceeds the 256 MiB Infinity Cache, as in the real chunk where 18 layers x 35 MB
of action-expert weights stream through every denoise step.  Per-launch time = replay time / reps.  The
gap bounds what prefetching a kernel's weights (while the latency-bound attention runs) could save.
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
    ap.add_argument("--reps", type=int, default=64)
    a = ap.parse_args()
    from pizero_native import ops

    dev = "cuda"
    rnd = lambda *s: (torch.rand(*s, device=dev) * 2 - 1).to(torch.bfloat16)  # noqa: E731
    nw = rnd(1024)
    cases = {
        "o (2048->1024, +resid)": (2048, 1024, dict(resid=rnd(4, 1024)), 1024),
        "gate|up (1024->2x4096, norm+GeGLU)": (1024, 8192, dict(epi=ops.PZ_EPI_GEGLU, norm=(nw, 1e-6)), 4096),
        "down (4096->1024, +resid)": (4096, 1024, dict(resid=rnd(4, 1024)), 1024),
    }
    for name, (K, N, kw, n) in cases.items():
        x = rnd(4, K)
        out = torch.empty(4, n, device=dev, dtype=torch.bfloat16)
        mb = N * K * 2 / 1e6
        ncopy = max(1, int(300e6 / (N * K * 2)) + 1)
        Ws = [rnd(N, K) for _ in range(ncopy)]
        res = {}
        for mode in ("warm", "cold"):
            seq = [Ws[0]] * a.reps if mode == "warm" else [Ws[i % ncopy] for i in range(a.reps)]
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                for W in seq[:2]:
                    ops.linear(x, W, out, **kw)
            torch.cuda.current_stream().wait_stream(s)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                for W in seq:
                    ops.linear(x, W, out, **kw)
            for _ in range(3):
                g.replay()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(5):
                g.replay()
            e1.record()
            torch.cuda.synchronize()
            res[mode] = e0.elapsed_time(e1) / 5 / a.reps * 1e3
            del g
        print(f"{name:36s} {mb:5.1f} MB: HBM-streamed {res['cold']:6.2f} us ({mb / res['cold']:.2f} TB/s), "
              f"cache-resident {res['warm']:6.2f} us ({mb / res['warm']:.2f} TB/s)", flush=True)
        del Ws


if __name__ == "__main__":
    main()
