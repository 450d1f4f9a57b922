"""A/B: first-round phase offsets (PZ_GEMM_DESYNC="sleeps,groups[,all]") on the 8-phase launches whose epilogue
moves the most bytes: the vlm down-proj dgrad with the GeGLU derivative (reads g|u, writes d(g|u): 512 KiB per tile,
all CUs of a round at once) and the gate|up + GeGLU forward (h + g|u written).

    python tools/desync_ab.py [--mb 256] [--iters 10] [--reps 3]
Outputs are compared bitwise with the undelayed launch (the offsets change only timing).
"""

import argparse
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
    g = torch.Generator(device=dev).manual_seed(0)
    rnd = lambda *s: (torch.rand(*s, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)  # noqa: E731
    M, H, I = 276 * a.mb, 2048, 16384
    dy, wd = rnd(M, H), rnd(H, I)          # down-proj output gradient, down_proj.weight [H, I]
    gu = rnd(M, 2 * I)                     # saved g | u
    dgu = torch.empty(M, 2 * I, device=dev, dtype=torch.bfloat16)
    x, wgu = rnd(M, H), rnd(2 * I, H)      # gate|up input and weights
    h = torch.empty(M, I, device=dev, dtype=torch.bfloat16)
    gu_out = torch.empty(M, 2 * I, device=dev, dtype=torch.bfloat16)
    cases = {
        "dgeglu": (lambda: ops.linear_dgrad(dy, wd, dgu, epi=ops.PZ_EPI_DGEGLU, aux=gu), 2.0 * M * I * H, [dgu]),
        "geglu": (lambda: ops.linear(x, wgu, h, epi=ops.PZ_EPI_GEGLU, aux=gu_out), 2.0 * M * 2 * I * H, [h, gu_out]),
    }
    settings = {"dgeglu": ["", "1,8", "2,8", "1,16", "2,16", "3,16"],
                "geglu": ["", "1,16,all", "2,16,all"]}
    for name, (fn, flop, outs) in cases.items():
        times = {s: [] for s in settings[name]}
        ref = None
        for _ in range(a.reps):
            for s in settings[name]:
                os.environ["PZ_GEMM_DESYNC"] = s
                fn()
                torch.cuda.synchronize()
                if s == "" and ref is None:
                    ref = [o.clone() for o in outs]
                same = ref is None or all(torch.equal(o, r) for o, r in zip(outs, ref))
                assert same, (name, s)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                times[s].append(e0.elapsed_time(e1) / a.iters)
        os.environ["PZ_GEMM_DESYNC"] = ""
        for s, ts in times.items():
            t = min(ts)
            print(f"{name} M={M}: desync '{s or 'off'}': {t:.4f} ms ({flop / t / 1e9:.0f} TF/s) all "
                  f"{['%.4f' % q for q in ts]} bitwise == off", flush=True)
        del ref


if __name__ == "__main__":
    main()
