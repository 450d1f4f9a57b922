"""A/B: the joint forward with the softmax export, one 16-row block per wave (flash_fwd_probs_kernel, 8 waves)
vs two per wave (flash_fwd_probs2_kernel, 4 waves; PZ_FLASH_PROBS2=1), at the bench's joint-attention shape.

    python tools/probs2_ab.py [--mb 256] [--iters 10] [--reps 3]
P, tanh(cap) and O are compared bitwise (same operands in the same order per row).
"""

import argparse
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "open-pi-zero_amd"))

import torch  # noqa: E402

from pizero_native import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=int, default=256)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    dev = "cuda"
    B, P, C, H, nh, hd = a.mb, 276, 1, 4, 8, 256
    L = P + C + H
    Lp = (L + 7) // 8 * 8
    g = torch.Generator(device=dev).manual_seed(0)
    Q = torch.randn(B, L * nh, hd, device=dev, generator=g).to(torch.bfloat16)
    K = torch.randn(B, Lp, hd, device=dev, generator=g).to(torch.bfloat16)
    V = torch.randn(B, Lp, hd, device=dev, generator=g).to(torch.bfloat16)
    # ragged prefixes (pad tokens -> dead rows) like the bench's synthetic batches
    cnt = torch.randint(P - 40, P + 1, (B,), device=dev, generator=g).to(torch.int32)
    outs = {}
    times = {"0": [], "1": []}
    for rep in range(a.reps):
        for v in ("0", "1"):
            os.environ["PZ_FLASH_PROBS2"] = v
            Ov = torch.zeros(B * P, nh * hd, device=dev, dtype=torch.bfloat16)
            Oe = torch.zeros(B * (C + H), nh * hd, device=dev, dtype=torch.bfloat16)
            Pm = torch.zeros(B, L * nh, Lp, device=dev, dtype=torch.bfloat16)
            tcm = torch.zeros_like(Pm)
            fa = ops.flash_args(B, 1, L * nh, L, hd, Q, (hd, L * nh * hd, 0), K, (hd, Lp * hd, 0), V,
                                (hd, Lp * hd, 0), [(0, Ov, P * nh * hd, hd), (P * nh, Oe, (C + H) * nh * hd, hd)], 0,
                                None, 1 / math.sqrt(hd), cap=50.0, mask_mode=1, cnt=cnt, prefix=P, cond=C,
                                rows_per_token=nh)
            fn = lambda: ops.flash_fwd_probs(fa, Pm, tcm, Lp)  # noqa: E731
            fn()
            torch.cuda.synchronize()
            if rep == 0:
                outs[v] = (Ov.clone(), Oe.clone(), Pm.clone(), tcm.clone())
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                fn()
            e1.record()
            torch.cuda.synchronize()
            times[v].append(e0.elapsed_time(e1) / a.iters)
    os.environ["PZ_FLASH_PROBS2"] = "0"
    same = [torch.equal(x, y) for x, y in zip(outs["0"], outs["1"])]
    fl = 4.0 * B * L * nh * L * hd
    for v, ts in times.items():
        t = min(ts)
        print(f"probs{'2' if v == '1' else ' '} B={B}: {t:.4f} ms ({fl / t / 1e9:.0f} TF/s) all {['%.4f' % q for q in ts]}",
              flush=True)
    print(f"bitwise O_vlm / O_expert / P / tanh: {same}", flush=True)
    if not all(same):
        for name, x, y in zip(("Ov", "Oe", "P", "tc"), outs["0"], outs["1"]):
            print(name, float((x.float() - y.float()).abs().max()), flush=True)


if __name__ == "__main__":
    main()
