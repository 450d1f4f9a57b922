"""CU-contention probe (VERDICT r5 "Next round" 6): how the persistent SigLIP attention kernels, the joint attention
kernels and the 8-phase GEMMs slow down when k CUs are held by another stream's kernel -- a stand-in for the RCCL
all-reduce kernels that share the CUs with the last micro-batch's backward under data parallelism.

For k in {0, 8, 32}: a side stream launches pz_debug_spin(k workgroups x 96 KiB LDS: one per CU, and no 160 KiB
workgroup fits beside it) for a few ms, then the main stream runs the kernel under test; the kernel's time is taken
with HIP events on the main stream (median over rounds).  The ideal slowdown with k CUs lost is 256 / (256 - k)
(1.03 at 8, 1.14 at 32); a kernel whose work is assigned statically per workgroup waits for the held CUs instead.

    python tools/contention_probe.py [--rounds 5] [--batch 256]
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


def timed(fn, k, side, hold_ticks):
    main = torch.cuda.current_stream()
    side.wait_stream(main)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if k:
        with torch.cuda.stream(side):
            ops.debug_spin(k, hold_ticks)
    e0.record()
    fn()
    e1.record()
    main.wait_stream(side)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--hold-ms", type=float, default=20.0)
    ap.add_argument("--sig-grids", default="1", help="PZ_SIG_GRID values to probe for the persistent SigLIP kernels")
    ap.add_argument("--only", default="", help="substring filter on the case names")
    a = ap.parse_args()
    dev = "cuda"
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    side = torch.cuda.Stream()
    # calibrate the spin (wall-clock ticks per ms) with one workgroup
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ops.debug_spin(1, 100000)
    e0.record()
    ops.debug_spin(1, 1000000)
    e1.record()
    torch.cuda.synchronize()
    per_ms = 1000000 / e0.elapsed_time(e1)
    ticks = int(a.hold_ms * per_ms)
    print(f"spin calibration: {per_ms:.0f} wall-clock ticks per ms", flush=True)
    B = a.batch
    # SigLIP attention (the persistent kernels): B images x 16 heads x 256 x 72
    nh, hd, N = 16, 72, 256
    qkv = torch.randn(B * N, 3 * nh * hd, device=dev).to(torch.bfloat16)
    O = torch.empty(B * N, nh * hd, device=dev, dtype=torch.bfloat16)
    dO = torch.randn_like(O)
    lse = torch.empty(B * nh, N, device=dev)
    delta = torch.empty_like(lse)
    dqkv = torch.empty_like(qkv)
    sa = ops.siglip_flash_args(qkv, O, lse, B, nh, hd, N, dO=dO, delta=delta, dqkv=dqkv)
    # joint attention (probs / dS): B x 281 x 8 heads, head 256
    P_, C_, H_, jnh, jhd = 276, 1, 4, 8, 256
    L = P_ + C_ + H_
    Lp = (L + 7) // 8 * 8
    Q = torch.randn(B, L * jnh, jhd, device=dev).to(torch.bfloat16)
    K = torch.randn(B, Lp, jhd, device=dev).to(torch.bfloat16)
    V = torch.randn(B, Lp, jhd, device=dev).to(torch.bfloat16)
    Ov = torch.empty(B * P_, jnh * jhd, device=dev, dtype=torch.bfloat16)
    Oe = torch.empty(B * (C_ + H_), jnh * jhd, device=dev, dtype=torch.bfloat16)
    cnt = torch.full((B,), P_, device=dev, dtype=torch.int32)
    fa = ops.flash_args(B, 1, L * jnh, L, jhd, Q, (jhd, L * jnh * jhd, 0), K, (jhd, Lp * jhd, 0), V, (jhd, Lp * jhd, 0),
                        [(0, Ov, P_ * jnh * jhd, jhd), (P_ * jnh, Oe, (C_ + H_) * jnh * jhd, jhd)], 0, None,
                        1 / math.sqrt(jhd), cap=50.0, mask_mode=1, cnt=cnt, prefix=P_, cond=C_, rows_per_token=jnh,
                        dgroups=[torch.randn_like(Ov), torch.randn_like(Oe)], dq=torch.empty_like(Q))
    Pm = torch.empty(B, L * jnh, Lp, device=dev, dtype=torch.bfloat16)
    tc = torch.empty_like(Pm)
    dS = torch.empty_like(Pm)
    ops.flash_fwd_probs(fa, Pm, tc, Lp)
    # 8-phase GEMMs at a quarter of the micro-batch-256 rows (vlm GeGLU gate|up and the SigLIP fc1 + GELU)
    M = B // 4 * 276
    x = torch.randn(M, 2048, device=dev).to(torch.bfloat16)
    Wgu = (torch.randn(32768, 2048, device=dev) * 0.02).to(torch.bfloat16)
    h = torch.empty(M, 16384, device=dev, dtype=torch.bfloat16)
    gu = torch.empty(M, 32768, device=dev, dtype=torch.bfloat16)
    Ms = B // 4 * 256
    xs = torch.randn(Ms, 1152, device=dev).to(torch.bfloat16)
    W1 = (torch.randn(4304, 1152, device=dev) * 0.02).to(torch.bfloat16)
    g1 = torch.empty(Ms, 4304, device=dev, dtype=torch.bfloat16)
    def sig(fn, grid):
        def run():
            os.environ["PZ_SIG_GRID"] = str(grid)
            fn()
        return run

    cases = {}
    for grid in a.sig_grids.split(","):
        cases[f"siglip fwd (persistent, {grid} x CUs wgs)"] = sig(lambda: ops.flash_fwd(sa), grid)
        cases[f"siglip bwd dQ + dK/dV (persistent, {grid} x CUs)"] = sig(lambda: ops.flash_bwd(sa), grid)
    cases.update({
        "joint fwd + probs": lambda: ops.flash_fwd_probs(fa, Pm, tc, Lp),
        "joint bwd dS + dQ": lambda: ops.flash_bwd_ds(fa, Pm, tc, dS, Lp),
        f"GEMM {M}x32768x2048 GeGLU (8-phase)": lambda: ops.linear(x, Wgu, h, epi=ops.PZ_EPI_GEGLU, aux=gu),
        f"GEMM {Ms}x4304x1152 GELU (8-phase)": lambda: ops.linear(xs, W1, g1, epi=ops.PZ_EPI_GELU),
    })
    ks = (0, 8, 32)
    print(f"{cus} CUs; side-stream spin holds k CUs for {a.hold_ms} ms; median of {a.rounds} rounds", flush=True)
    for name, fn in cases.items():
        if a.only and a.only not in name:
            continue
        for _ in range(2):
            fn()
        res = {k: [] for k in ks}
        for _ in range(a.rounds):
            for k in ks:
                res[k].append(timed(fn, k, side, ticks))
        med = {k: sorted(v)[len(v) // 2] for k, v in res.items()}
        line = "  ".join(f"k={k}: {med[k]:.3f} ms (x{med[k] / med[0]:.2f}, ideal x{cus / (cus - k):.2f})" for k in ks)
        print(f"{name:42s} {line}", flush=True)


if __name__ == "__main__":
    main()
