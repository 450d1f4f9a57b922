"""Microbenchmark of the fused attention kernels at the bench shapes (micro-batch 256).

    python tools/flash_bench.py [--iters 10] [--batch 256] [--default-only]
joint: B samples x (281 tokens x 8 heads) queries, 281 keys, head 256, soft-cap + block mask;
siglip: B x 16 heads x 256 x 256, head 72.  Prints fwd / bwd ms and TF/s (algorithmic
FLOP: fwd 4*nq*nk*hd per unit, bwd 2.5x fwd).
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
    ap.add_argument("--iters", type=int, default=30)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--default-only", action="store_true", help="only the training-default kernels (PMC passes)")
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
    for dma in ("1",) if a.default_only else ("1", "0"):  # PZ_PROBS_DMA: LDS-DMA ring (default) vs register staging
        os.environ["PZ_PROBS_DMA"] = dma
        tp = timeit(lambda: ops.flash_fwd_probs(fa, Pm, tcm, Lp), a.iters)
        print(f"joint  fwd+probs(dma={dma}) {tp:.3f} ms {fl / tp / 1e9:.0f} TF/s (O + bf16 P / tanh(cap) export)",
              flush=True)
    os.environ.pop("PZ_PROBS_DMA")
    dSm = torch.empty_like(Pm)
    td = timeit(lambda: ops.flash_bwd_ds(fa, Pm, tcm, dSm, Lp), a.iters)
    print(f"joint  bwd dS {td:.3f} ms (dP = dO V^T in registers + softmax backward from P / tanh(cap))", flush=True)
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
    # unit, the 2-/4-workgroup resident kernels
    for sig, unit in (("1", "1"),) if a.default_only else (("1", "1"), ("1q", "1"), ("1p", "1"), ("0", "1"), ("0", "0")):
        # "1p": the persistent kernels with the separate delta pass (PZ_SIG_DELTA=pass); "1q": the forward with 8 waves
        # of 32 rows (PZ_SIG_QB=2)
        os.environ["PZ_FLASH_UNIT"], os.environ["PZ_FLASH_SIG"] = unit, sig[0]
        os.environ["PZ_SIG_DELTA"] = "pass" if sig == "1p" else "fused"
        os.environ["PZ_SIG_QB"] = "2" if sig == "1q" else "1"
        tf = timeit(lambda: ops.flash_fwd(sa), a.iters)
        tb = timeit(lambda: ops.flash_bwd(sa), a.iters)
        print(f"siglip(sig={sig},unit={unit}) fwd {tf:.3f} ms {fl / tf / 1e9:.0f} TF/s   bwd {tb:.3f} ms "
              f"{2.5 * fl / tb / 1e9:.0f} TF/s", flush=True)
    os.environ.pop("PZ_FLASH_UNIT")
    os.environ.pop("PZ_FLASH_SIG")
    os.environ.pop("PZ_SIG_DELTA")
    os.environ.pop("PZ_SIG_QB")


if __name__ == "__main__":
    main()
