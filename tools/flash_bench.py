"""Microbenchmark of the fused attention kernels at the bench shapes (micro-batch 256).

    python tools/flash_bench.py [--iters 10] [--batch 256] [--default-only]
joint: B samples x (281 tokens x 8 heads) queries, 281 keys, head 256, soft-cap + block mask;
siglip: B x 16 heads x 256 x 256, head 72.  Prints fwd / bwd ms and TF/s (algorithmic
FLOP: fwd 4*nq*nk*hd per unit, bwd 2.5x fwd).

The non-default variants (PZ_PROBS_DMA=0, PZ_SIG_DELTA=pass, PZ_SIG_QB=2) exist only in a -DPZ_FLASH_AB build of the
library; in the product build those settings run the default kernels (use --default-only there).
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


def timeit(fn, iters):
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
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--default-only", action="store_true", help="only the training-default kernels (PMC passes)")
    ap.add_argument("--rounds", type=int, default=5, help="interleaved timing rounds per variant (median)")
    a = ap.parse_args()
    dev = "cuda"
    B, P, C, H, nh, hd = a.batch, 276, 1, 4, 8, 256
    L = P + C + H
    Lp = (L + 7) // 8 * 8
    Q = torch.randn(B, L * nh, hd, device=dev).to(torch.bfloat16)
    K = torch.randn(B, Lp, hd, device=dev).to(torch.bfloat16)
    V = torch.randn(B, Lp, hd, device=dev).to(torch.bfloat16)
    Ov = torch.empty(B * P, nh * hd, device=dev, dtype=torch.bfloat16)
    Oe = torch.empty(B * (C + H), nh * hd, device=dev, dtype=torch.bfloat16)
    dOv, dOe = torch.randn_like(Ov), torch.randn_like(Oe)
    lse = torch.empty(B, L * nh, device=dev)
    delta = torch.empty_like(lse)
    dQ, dK, dV = torch.empty_like(Q), torch.empty_like(K), torch.empty_like(V)
    cnt = torch.full((B,), P, device=dev, dtype=torch.int32)
    fa = ops.flash_args(B, 1, L * nh, L, hd, Q, (hd, L * nh * hd, 0), K, (hd, Lp * hd, 0), V, (hd, Lp * hd, 0),
                        [(0, Ov, P * nh * hd, hd), (P * nh, Oe, (C + H) * nh * hd, hd)], 0, lse, 1 / math.sqrt(hd),
                        cap=50.0, mask_mode=1, cnt=cnt, prefix=P, cond=C, rows_per_token=nh, dgroups=[dOv, dOe],
                        delta=delta, dq=dQ, dk=dK, dv=dV)
    fl = 4.0 * B * L * nh * L * hd
    Pm = torch.empty(B, L * nh, Lp, device=dev, dtype=torch.bfloat16)
    tcm = torch.empty_like(Pm)
    dSm = torch.empty_like(Pm)
    jt = {dma: ([], []) for dma in (("1",) if a.default_only else ("1", "0"))}  # PZ_PROBS_DMA: LDS-DMA ring / registers
    for _ in range(1 if a.default_only else a.rounds):
        for dma in jt:
            os.environ["PZ_PROBS_DMA"] = dma
            jt[dma][0].append(timeit(lambda: ops.flash_fwd_probs(fa, Pm, tcm, Lp), a.iters))
            jt[dma][1].append(timeit(lambda: ops.flash_bwd_ds(fa, Pm, tcm, dSm, Lp), a.iters))
    os.environ.pop("PZ_PROBS_DMA")
    for dma, (tps, tds) in jt.items():
        tp, td = sorted(tps)[len(tps) // 2], sorted(tds)[len(tds) // 2]
        print(f"joint(dma={dma})  fwd+probs {tp:.3f} ms {fl / tp / 1e9:.0f} TF/s (O + bf16 P / tanh(cap) export)   "
              f"bwd dS {td:.3f} ms (+ dQ)  (median of {len(tps)} rounds)", flush=True)
    for fast in () if a.default_only else ("1", "0"):  # PZ_FLASH_FAST: fast element-wise joint backward vs the generic kernels
        os.environ["PZ_FLASH_FAST"] = fast
        tf = timeit(lambda: ops.flash_fwd(fa), a.iters)
        tb = timeit(lambda: ops.flash_bwd(fa), a.iters)
        print(f"joint(fast={fast})  fwd {tf:.3f} ms {fl / tf / 1e9:.0f} TF/s   bwd {tb:.3f} ms "
              f"{2.5 * fl / tb / 1e9:.0f} TF/s", flush=True)
    os.environ.pop("PZ_FLASH_FAST", None)
    nh, hd, N = 16, 72, 256
    qkv = torch.randn(B * N, 3 * nh * hd, device=dev).to(torch.bfloat16)
    O = torch.empty(B * N, nh * hd, device=dev, dtype=torch.bfloat16)
    dO = torch.randn_like(O)
    lse = torch.empty(B * nh, N, device=dev)
    delta = torch.empty_like(lse)
    dqkv = torch.empty_like(qkv)
    sa = ops.siglip_flash_args(qkv, O, lse, B, nh, hd, N, dO=dO, delta=delta, dqkv=dqkv)
    fl = 4.0 * B * nh * N * N * hd
    # PZ_FLASH_SIG / PZ_FLASH_UNIT: the persistent pipelined kernels (default), one workgroup per (image, head)
    # unit, the 2-/4-workgroup resident kernels; "1p": the persistent kernels with the separate delta pass
    # (PZ_SIG_DELTA=pass); "1q": the forward with 8 waves of 32 rows (PZ_SIG_QB=2).  The variants are timed in
    # interleaved rounds (clock drift between back-to-back runs of the same kernel reaches ~10 %) and the median
    # of the rounds is printed.
    variants = [("1", "1")] if a.default_only else [("1", "1"), ("1q", "1"), ("1p", "1"), ("0", "1"), ("0", "0")]
    times = {v: ([], []) for v in variants}
    for _ in range(1 if a.default_only else a.rounds):
        for v in variants:
            sig, unit = v
            os.environ["PZ_FLASH_UNIT"], os.environ["PZ_FLASH_SIG"] = unit, sig[0]
            os.environ["PZ_SIG_DELTA"] = "pass" if sig == "1p" else "fused"
            os.environ["PZ_SIG_QB"] = "2" if sig == "1q" else "1"
            times[v][0].append(timeit(lambda: ops.flash_fwd(sa), a.iters))
            times[v][1].append(timeit(lambda: ops.flash_bwd(sa), a.iters))
    for (sig, unit), (tfs, tbs) in times.items():
        tf, tb = sorted(tfs)[len(tfs) // 2], sorted(tbs)[len(tbs) // 2]
        print(f"siglip(sig={sig},unit={unit}) fwd {tf:.3f} ms {fl / tf / 1e9:.0f} TF/s   bwd {tb:.3f} ms "
              f"{2.5 * fl / tb / 1e9:.0f} TF/s  (median of {len(tfs)} rounds)", flush=True)
    for k in ("PZ_FLASH_UNIT", "PZ_FLASH_SIG", "PZ_SIG_DELTA", "PZ_SIG_QB"):
        os.environ.pop(k)

if __name__ == "__main__":
    main()
