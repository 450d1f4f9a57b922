"""8-bit AdamW step over a Pi0-sized parameter arena (SigLIP 27 layers + Gemma 18 + the action expert 18: 2.7 B
bf16 parameters in ~800 tensors, one contiguous run), HIP-event timed, with the algorithmic bytes (10 B / element:
p and g read, p written, two 1-byte state codes read and written) and the rate.

    python tools/optim_bench.py [--iters 10]
"""

import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "open-pi-zero_amd"))

import torch  # noqa: E402


def shapes():
    out = []
    for _ in range(27):  # SigLIP So400m/14 layer
        out += [(1152, 1152)] * 3 + [(1152,)] * 3 + [(1152, 1152), (1152,), (4304, 1152), (4304,), (1152, 4304),
                                                     (1152,), (1152,), (1152,), (1152,), (1152,)]
    for _ in range(18):  # Gemma-2B layer
        out += [(2048, 2048), (256, 2048), (256, 2048), (2048, 2048), (16384, 2048), (16384, 2048), (2048, 16384),
                (2048,), (2048,)]
    for _ in range(18):  # action expert layer
        out += [(2048, 1024), (256, 1024), (256, 1024), (1024, 2048), (4096, 1024), (4096, 1024), (1024, 4096),
                (1024,), (1024,)]
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    from pizero_native.optim import FusedAdamW

    sh = shapes()
    n = [int(torch.tensor(s).prod()) for s in sh]
    pad = [(k + 7) // 8 * 8 for k in n]
    total = sum(pad)
    dev = "cuda"
    w = (torch.rand(total, device=dev) * 0.2 - 0.1).to(torch.bfloat16)
    gbuf = (torch.randn(total, device=dev) * 1e-3).to(torch.bfloat16)
    params, o = [], 0
    for s, k, kp in zip(sh, n, pad):
        p = torch.nn.Parameter(w[o:o + k].view(s))
        p.grad = gbuf[o:o + k].view(s)
        params.append(p)
        o += kp
    opt = FusedAdamW(params, lr=1e-4, weight_decay=0.01, state_bits=8)
    for _ in range(2):
        opt.step()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        opt.step()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.iters
    elems = sum(n)
    print(f"adamw8 step: {len(sh)} tensors, {elems / 1e9:.3f} B elements: {ms:.3f} ms, "
          f"{elems * 10 / ms / 1e9:.2f} TB/s of 10 B / element", flush=True)


if __name__ == "__main__":
    main()
