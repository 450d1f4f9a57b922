"""Microbenchmark of the fused attention kernels at the bench shapes (micro-batch 256).

    python tools/flash_bench.py [--iters 10] [--batch 256] [--default-only]
joint: B samples x (281 tokens x 8 heads) queries, 281 keys, head 256, soft-cap + block mask;
siglip: B x 16 heads x 256 x 256, head 72.  Prints fwd / bwd ms and TF/s (algorithmic
FLOP: fwd 4*nq*nk*hd per unit, bwd 2.5x fwd).

Non-default variants timed beside the defaults: the all-fused joint kernels (pz_flash_fwd / pz_flash_bwd, the
PZ_JOINT_ATTN=flash path) and the one-workgroup-per-unit / resident SigLIP kernels (PZ_FLASH_SIG=0, PZ_FLASH_UNIT=0).
(The round-4 register-staged joint kernels, the separate SigLIP delta pass and the 8 x 32-row SigLIP forward were
measured slower and removed in round 6: profiles/r05/flash_bench_r5l.log.)
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
    tps, tds = [], []
    for _ in range(1 if a.default_only else a.rounds):
        tps.append(timeit(lambda: ops.flash_fwd_probs(fa, Pm, tcm, Lp), a.iters))
        tds.append(timeit(lambda: ops.flash_bwd_ds(fa, Pm, tcm, dSm, Lp), a.iters))
    tp, td = sorted(tps)[len(tps) // 2], sorted(tds)[len(tds) // 2]
    print(f"joint(dma=1)  fwd+probs {tp:.3f} ms {fl / tp / 1e9:.0f} TF/s (O + bf16 P / tanh(cap) export)   "
          f"bwd dS {td:.3f} ms (+ dQ)  (median of {len(tps)} rounds)", flush=True)
    if not a.default_only:  # the all-fused joint kernels (PZ_JOINT_ATTN=flash)
        tf = timeit(lambda: ops.flash_fwd(fa), a.iters)
        tb = timeit(lambda: ops.flash_bwd(fa), a.iters)
        print(f"joint(fused)  fwd {tf:.3f} ms {fl / tf / 1e9:.0f} TF/s   bwd {tb:.3f} ms "
              f"{2.5 * fl / tb / 1e9:.0f} TF/s", flush=True)
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
    # unit, the 2-/4-workgroup resident kernels.  The variants are timed in interleaved rounds (clock drift between
    # back-to-back runs of the same kernel reaches ~10 %) and the median of the rounds is printed.
    variants = [("1", "1")] if a.default_only else [("1", "1"), ("0", "1"), ("0", "0")]
    times = {v: ([], []) for v in variants}
    for _ in range(1 if a.default_only else a.rounds):
        for v in variants:
            sig, unit = v
            os.environ["PZ_FLASH_UNIT"], os.environ["PZ_FLASH_SIG"] = unit, sig
            times[v][0].append(timeit(lambda: ops.flash_fwd(sa), a.iters))
            times[v][1].append(timeit(lambda: ops.flash_bwd(sa), a.iters))
    for (sig, unit), (tfs, tbs) in times.items():
        tf, tb = sorted(tfs)[len(tfs) // 2], sorted(tbs)[len(tbs) // 2]
        print(f"siglip(sig={sig},unit={unit}) fwd {tf:.3f} ms {fl / tf / 1e9:.0f} TF/s   bwd {tb:.3f} ms "
              f"{2.5 * fl / tb / 1e9:.0f} TF/s  (median of {len(tfs)} rounds)", flush=True)
    for k in ("PZ_FLASH_UNIT", "PZ_FLASH_SIG"):
        os.environ.pop(k)

if __name__ == "__main__":
    main()
