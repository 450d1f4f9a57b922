"""GeGLU backward of the Gemma MLP: down-proj dgrad with the derivative in its epilogue (PZ_EPI_DGEGLU) vs a
plain dgrad + the separate HBM-bound geglu_bwd pass (engine PZ_SPLIT_DACT=1, the default).  Measurement tool.

    python tools/dact_ab.py [--iters 20]
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
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    from pizero_native import ops

    dev = "cuda"
    rnd = lambda *s: (torch.rand(*s, device=dev) * 2 - 1).to(torch.bfloat16)  # noqa: E731

    def timed(fn):
        for _ in range(3):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / a.iters

    for name, M, H, I in (("vlm", 17664, 2048, 16384), ("action", 320, 1024, 4096)):
        dx, W = rnd(M, H), rnd(H, I) * 0.02
        gu0 = rnd(M, 2 * I)
        gu = gu0.clone()
        dh = torch.empty(M, I, device=dev, dtype=torch.bfloat16)

        def split():
            ops.linear_dgrad(dx, W, dh)
            ops.geglu_bwd(dh, gu, gu, None, M, I)

        def fused():
            ops.linear_dgrad(dx, W, gu, epi=ops.PZ_EPI_DGEGLU, aux=gu)

        def dgrad_only():
            ops.linear_dgrad(dx, W, dh)

        ts = timed(split)
        gu.copy_(gu0)
        tf = timed(fused)
        td = timed(dgrad_only)
        # one-shot numerics check from the same saved g|u
        gu.copy_(gu0)
        split()
        r1 = gu.clone()
        gu.copy_(gu0)
        fused()
        rel = float((gu.float() - r1.float()).norm() / r1.float().norm())
        print(f"{name:7s} M={M} H={H} I={I}: split {ts:.4f} ms (dgrad {td:.4f} + pass {ts - td:.4f}) | fused "
              f"{tf:.4f} ms | fused - split {tf - ts:+.4f} ms | rel-L2 {rel:.2e}", flush=True)


if __name__ == "__main__":
    main()
