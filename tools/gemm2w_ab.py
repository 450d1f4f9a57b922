"""A/B of the two-resident-workgroup NT GEMM (PZ_GEMM_2W=1) against the 8-phase kernel on the bench's
forward shapes (measurement tool, not product code).

    python tools/gemm2w_ab.py [--iters 20]

Random bf16 inputs; HIP-event timing on the launch stream; per shape: the 8-phase plan as shipped, the
two-workgroup kernel, and the two-workgroup kernel with its epilogue stores skipped (PZ_GEMM_DBG=1).
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
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--desync", type=int, nargs="*", default=[], help="PZ_GEMM_DBG values >= 2 to time (2w)")
    ap.add_argument("--only", default="", help="comma-separated case names")
    a = ap.parse_args()
    from pizero_native import ops

    dev = "cuda"
    rnd = lambda *s: (torch.rand(*s, device=dev) * 2 - 1).to(torch.bfloat16)  # noqa: E731

    def timed(fn):
        for _ in range(3):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / a.iters

    def case(name, M, N, K, geglu=False, bias=False, act=None, resid=False):
        if a.only and name not in a.only.split(","):
            return
        x, w = rnd(M, K), rnd(N, K)
        b = rnd(N) if bias else None
        r = rnd(M, N) if resid else None
        if geglu:
            out = torch.empty(M, N // 2, device=dev, dtype=torch.bfloat16)
            aux = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            fn = lambda: ops.linear(x, w, out, epi=ops.PZ_EPI_GEGLU, aux=aux)  # noqa: E731
            kn = lambda: ops.gemm_kernel_name(M, N, K, epi=ops.PZ_EPI_GEGLU, geglu_inter=N // 2)  # noqa: E731
        else:
            out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            aux = torch.empty(M, N, device=dev, dtype=torch.bfloat16) if act else None
            epi = {None: ops.PZ_EPI_NONE, "gelu": ops.PZ_EPI_GELU}[act]
            fn = lambda: ops.linear(x, w, out, bias=b, resid=r, epi=epi, aux=aux)  # noqa: E731
            kn = lambda: ops.gemm_kernel_name(M, N, K, epi=epi)  # noqa: E731
        res, names = {}, {}
        for mode in ("0", "1"):
            os.environ["PZ_GEMM_2W"] = mode
            names[mode] = kn()
            ref = None
            res[mode] = timed(fn)
            if mode == "0":
                ref = out.clone()
            else:
                torch.cuda.synchronize()
        os.environ["PZ_GEMM_DBG"] = "1"
        res["1ns"] = timed(fn)
        desync = []
        for d in a.desync:  # first-round upper-slot workgroups delayed by d - 2 x s_sleep(127)
            os.environ["PZ_GEMM_DBG"] = str(d)
            desync.append(f"{d - 2}: {timed(fn):.4f}")
        os.environ["PZ_GEMM_DBG"] = "0"
        os.environ["PZ_GEMM_2W"] = "0"
        del ref
        tf = lambda ms: 2.0 * M * N * K / ms / 1e9  # noqa: E731
        print(f"{name:10s} {M}x{N}x{K}: 8-phase {res['0']:.4f} ms ({tf(res['0']):.0f} TF/s) [{names['0']}] | "
              f"2w {res['1']:.4f} ms ({tf(res['1']):.0f}) [{names['1']}] | 2w no stores {res['1ns']:.4f} ms "
              f"({tf(res['1ns']):.0f})" + (f" | desync {', '.join(desync)}" if desync else ""), flush=True)

    case("geglu", 17664, 32768, 2048, geglu=True)
    case("plainNT", 17664, 32768, 2048)
    case("qkv", 17664, 2560, 2048)
    case("o_proj", 17664, 2048, 2048, resid=True)
    case("down", 17664, 2048, 16384, resid=True)
    case("sig_out", 16384, 1152, 1152, bias=True, resid=True)
    case("sig_qkv", 16384, 3456, 1152, bias=True)
    case("sig_fc1", 16384, 4304, 1152, bias=True, act="gelu")
    case("sig_fc2", 16384, 1152, 4304, bias=True, resid=True)


if __name__ == "__main__":
    main()
