"""A/B: SigLIP's 4304-wide operands with their natural row pitch (8608 B, not a multiple of the 128-B line) vs the
same values in buffers padded to a 4352-element pitch (8704 B = 68 lines), for the training GEMMs that read them.

    python tools/ld_pad_ab.py [--M 32768] [--iters 10]
Each case runs the identical math on identical values; outputs must match bitwise (the pitch changes only addresses).
"""

import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "open-pi-zero_amd"))

import torch  # noqa: E402

from pizero_native import ops  # noqa: E402


def padded(t, pitch):
    buf = torch.zeros(t.shape[0], pitch, device=t.device, dtype=t.dtype)
    buf[:, : t.shape[1]].copy_(t)
    return buf[:, : t.shape[1]]


def timeit(fn, iters):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", type=int, default=32768)
    ap.add_argument("--D", type=int, default=1152)
    ap.add_argument("--F", type=int, default=4304)
    ap.add_argument("--pitch", type=int, default=4352)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    rnd = lambda *s: (torch.rand(*s, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)  # noqa: E731
    M, D, F, P = a.M, a.D, a.F, a.pitch
    h, dh = rnd(M, F), rnd(M, F)          # fc1 output / its gradient (M x F)
    x, dy = rnd(M, D), rnd(M, D)          # fc1 input / fc2 output gradient (M x D)
    w1, w2 = rnd(F, D), rnd(D, F)         # fc1.weight [F, D], fc2.weight [D, F]
    hp, dhp, w2p = padded(h, P), padded(dh, P), padded(w2, P)

    cases = []
    y0, y1 = torch.empty(M, D, device=dev, dtype=torch.bfloat16), torch.empty(M, D, device=dev, dtype=torch.bfloat16)
    cases.append(("fc2 fwd   NT", 2.0 * M * D * F, lambda: ops.linear(h, w2, y0), lambda: ops.linear(hp, w2p, y1),
                  y0, y1))
    dx0, dx1 = torch.empty(M, D, device=dev, dtype=torch.bfloat16), torch.empty(M, D, device=dev, dtype=torch.bfloat16)
    cases.append(("fc1 dgrad NN", 2.0 * M * D * F, lambda: ops.linear_dgrad(dh, w1, dx0),
                  lambda: ops.linear_dgrad(dhp, w1, dx1), dx0, dx1))
    dh0 = torch.empty(M, F, device=dev, dtype=torch.bfloat16)
    dh1 = padded(torch.empty(M, F, device=dev, dtype=torch.bfloat16), P)
    cases.append(("fc2 dgrad NN", 2.0 * M * D * F, lambda: ops.linear_dgrad(dy, w2, dh0),
                  lambda: ops.linear_dgrad(dy, w2p, dh1), dh0, dh1))
    dw20 = torch.empty(D, F, device=dev, dtype=torch.bfloat16)
    dw21 = padded(torch.empty(D, F, device=dev, dtype=torch.bfloat16), P)
    cases.append(("fc2 wgrad TN", 2.0 * M * D * F, lambda: ops.linear_wgrad(dy, h, dw20),
                  lambda: ops.linear_wgrad(dy, hp, dw21), dw20, dw21))
    dw10 = torch.empty(F, D, device=dev, dtype=torch.bfloat16)
    dw11 = torch.empty(F, D, device=dev, dtype=torch.bfloat16)
    cases.append(("fc1 wgrad TN", 2.0 * M * D * F, lambda: ops.linear_wgrad(dh, x, dw10),
                  lambda: ops.linear_wgrad(dhp, x, dw11), dw10, dw11))
    h0 = torch.empty(M, F, device=dev, dtype=torch.bfloat16)
    h1 = padded(torch.empty(M, F, device=dev, dtype=torch.bfloat16), P)
    cases.append(("fc1 fwd   NT", 2.0 * M * D * F, lambda: ops.linear(x, w1, h0), lambda: ops.linear(x, w1, h1),
                  h0, h1))
    for name, flop, f0, f1, o0, o1 in cases:
        t0, t1 = timeit(f0, a.iters), timeit(f1, a.iters)
        t0b, t1b = timeit(f0, a.iters), timeit(f1, a.iters)
        t0, t1 = min(t0, t0b), min(t1, t1b)
        same = torch.equal(o0, o1)
        print(f"{name} M={M} D={D} F={F}: pitch {F}: {t0 * 1e3:8.1f} us ({flop / t0 / 1e9:6.1f} TF/s) | "
              f"pitch {P}: {t1 * 1e3:8.1f} us ({flop / t1 / 1e9:6.1f} TF/s) | {t0 / t1:5.3f}x | bitwise {same}",
              flush=True)


if __name__ == "__main__":
    main()
