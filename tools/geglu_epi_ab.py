"""GeGLU GEMM epilogue variants on the bench's dominant launch (vlm gate|up, M = 276 x micro-batch, N = 32768,
K = 2048), HIP-event timed over --iters back-to-back launches per variant, variants interleaved over --reps rounds:
PZ_GEMM_DBG 0 = shipped (h, g and u staged through LDS images in two passes), 1 = no epilogue stores (main loop
only), 4 = every output stored straight from the accumulators (8 B per lane), 5 = h and g staged, u stored
straight from the accumulators (one image pass).  Outputs of 4 / 5 are compared with 0 (bitwise).

    python tools/geglu_epi_ab.py [--mb 128] [--iters 10] [--reps 3]
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
    ap.add_argument("--mb", type=int, default=128)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    from pizero_native import ops

    dev = "cuda"
    M, N, K = 276 * a.mb, 32768, 2048
    x = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
    w = ((torch.rand(N, K, device=dev) * 2 - 1) * K ** -0.5).to(torch.bfloat16)
    h = torch.empty(M, N // 2, device=dev, dtype=torch.bfloat16)
    gu = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    print(ops.gemm_kernel_name(M, N, K, epi=ops.PZ_EPI_GEGLU, geglu_inter=N // 2), flush=True)
    outs = {}
    times = {v: [] for v in ("0", "1", "4", "5")}
    for rep in range(a.reps):
        for v in times:
            os.environ["PZ_GEMM_DBG"] = v
            for _ in range(2):
                ops.linear(x, w, h, epi=ops.PZ_EPI_GEGLU, aux=gu)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.iters):
                ops.linear(x, w, h, epi=ops.PZ_EPI_GEGLU, aux=gu)
            e1.record()
            torch.cuda.synchronize()
            times[v].append(e0.elapsed_time(e1) / a.iters)
            if rep == 0 and v != "1":
                outs[v] = (h.clone(), gu.clone())
    os.environ["PZ_GEMM_DBG"] = "0"
    fl = 2.0 * M * N * K
    for v, ts in times.items():
        t = min(ts)
        same = "" if v in ("0", "1") else f"  bitwise {'==' if all(torch.equal(p, q) for p, q in zip(outs[v], outs['0'])) else '!='} shipped"
        print(f"dbg {v}: {t:.4f} ms ({fl / t / 1e9:.0f} TF/s)  all {['%.4f' % q for q in ts]}{same}", flush=True)


if __name__ == "__main__":
    main()
