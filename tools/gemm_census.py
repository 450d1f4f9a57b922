"""Every pz_gemm launch of one bench micro-batch (fwd + bwd, micro-batch 64) with its shape, layout,
epilogue, kernel and HIP-event duration, aggregated per (layout, M, N, K, epilogue).  Single stream
(PZ_EXPERT_STREAM=0 unless set): events on the launching stream would otherwise time the action-expert
GEMMs while they share the chip with the vlm group's on the second stream.

    python tools/gemm_census.py [--micro-batch 64]
"""

import argparse
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "open-pi-zero_amd"))

import torch  # noqa: E402

os.environ.setdefault("PZ_EXPERT_STREAM", "0")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--micro-batch", type=int, default=64)
    a = ap.parse_args()
    from bench import synthetic_batch
    from pizero_native import ops
    from src.model.vla.pizero import PiZero
    from src.utils.config import load_config

    cfg = load_config(os.path.join(ROOT, "open-pi-zero_amd", "config", "train", "bridge.yaml"))
    dev = torch.device("cuda")
    m = PiZero(cfg, device=dev, dtype=torch.bfloat16, init="default")
    m.tie_action_proprio_weights()
    m.freeze_unused_weights()
    m.train()
    b = synthetic_batch(m, a.micro_batch, dev, torch.Generator().manual_seed(0))
    rec = []
    orig = ops._gemm

    def probe(M, N, K, A, lda, a_kc, B, ldb, b_kc, Cm, ldc, epi, alpha, beta, *rest):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        orig(M, N, K, A, lda, a_kc, B, ldb, b_kc, Cm, ldc, epi, alpha, beta, *rest)
        e1.record()
        batch = rest[6]
        name = ops.gemm_kernel_name(M, N, K, a_kc=a_kc, b_kc=b_kc, epi=epi, geglu_inter=rest[5], batch=batch,
                                    c_fp32=Cm.dtype == torch.float32)
        lay = ("N" if a_kc else "T") + ("T" if b_kc else "N")
        rec.append(((lay, M, N, K, int(epi), batch, bool(beta), Cm.dtype == torch.float32, name), e0, e1))

    for it in range(3):
        if it == 2:
            ops._gemm = probe
        m.zero_grad(set_to_none=True)
        loss = m(**b)
        loss.backward()
    torch.cuda.synchronize()
    ops._gemm = orig
    agg = collections.defaultdict(lambda: [0, 0.0])
    for key, e0, e1 in rec:
        agg[key][0] += 1
        agg[key][1] += e0.elapsed_time(e1)
    tot = sum(v[1] for v in agg.values())
    print(f"{len(rec)} GEMM launches, {tot:.1f} ms per micro-batch of {a.micro_batch}")
    print(f"{'lay':3s} {'M':>6s} {'N':>6s} {'K':>6s} epi bat beta f32 {'n':>4s} {'ms':>8s} {'%':>5s} {'TF/s':>7s}  kernel")
    for key, (n, ms) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        lay, M, N, K, epi, batch, beta, f32, name = key
        tf = 2.0 * M * N * K * batch * n / (ms * 1e-3) / 1e12
        print(f"{lay:3s} {M:6d} {N:6d} {K:6d} {epi:3d} {batch:3d} {int(beta):4d} {int(f32):3d} {n:4d} {ms:8.2f} "
              f"{100 * ms / tot:5.1f} {tf:7.1f}  {name}")


if __name__ == "__main__":
    main()
