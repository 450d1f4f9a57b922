"""How much of an 8-phase GEMM launch is its epilogue / tail?  (measurement tool, not product code)

    python tools/epi_probe.py [--iters 20]

For the forward (NT) shapes of the bench it times each launch with the epilogue as shipped and with
PZ_GEMM_DBG=1 (the kernel skips its output stores: main loop + prologue only), with and without the
split tail (PZ_GEMM_TAIL=0).  Inputs are random bf16; HIP-event timing on the launch stream.
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
    a = ap.parse_args()
    from pizero_native import ops

    dev = "cuda"
    rnd = lambda *s: (torch.rand(*s, device=dev) * 2 - 1).to(torch.bfloat16)  # noqa: E731

    def case(name, M, N, K, geglu=False, bias=False, act=None, resid=False):
        x, w = rnd(M, K), rnd(N, K)
        b = rnd(N) if bias else None
        r = rnd(M, N) if resid else None
        if geglu:
            out = torch.empty(M, N // 2, device=dev, dtype=torch.bfloat16)
            aux = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            fn = lambda: ops.linear(x, w, out, epi=ops.PZ_EPI_GEGLU, aux=aux)  # noqa: E731
            kname = ops.gemm_kernel_name(M, N, K, epi=ops.PZ_EPI_GEGLU, geglu_inter=N // 2)
        else:
            out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
            aux = torch.empty(M, N, device=dev, dtype=torch.bfloat16) if act else None
            epi = {None: ops.PZ_EPI_NONE, "gelu": ops.PZ_EPI_GELU}[act]
            fn = lambda: ops.linear(x, w, out, bias=b, resid=r, epi=epi, aux=aux)  # noqa: E731
            kname = ops.gemm_kernel_name(M, N, K, epi=epi)
        res = {}
        for tail in ("1", "0"):
            for dbg in ("0", "1"):
                os.environ["PZ_GEMM_TAIL"] = tail
                os.environ["PZ_GEMM_DBG"] = dbg
                for _ in range(3):
                    fn()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.iters):
                    fn()
                e1.record()
                torch.cuda.synchronize()
                res[(tail, dbg)] = e0.elapsed_time(e1) / a.iters
        os.environ["PZ_GEMM_TAIL"] = "1"
        os.environ["PZ_GEMM_DBG"] = "0"
        os.environ["PZ_GEMM_NT"] = "1"
        for _ in range(3):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        res["nt"] = e0.elapsed_time(e1) / a.iters
        os.environ["PZ_GEMM_NT"] = "0"
        tf = lambda ms: 2.0 * M * N * K / ms / 1e9  # noqa: E731
        print(f"{name:10s} {M}x{N}x{K} [{kname}]\n"
              f"   shipped {res[('1', '0')]:.3f} ms ({tf(res[('1', '0')]):.0f} TF/s) | no stores "
              f"{res[('1', '1')]:.3f} ms ({tf(res[('1', '1')]):.0f}) | no tail {res[('0', '0')]:.3f} ms "
              f"({tf(res[('0', '0')]):.0f}) | no tail, no stores {res[('0', '1')]:.3f} ms ({tf(res[('0', '1')]):.0f})\n"
              f"   non-temporal 16-B epilogue stores: {res['nt']:.3f} ms", flush=True)

    case("geglu", 17664, 32768, 2048, geglu=True)
    case("plainNT", 17664, 32768, 2048)
    case("qkv", 17664, 2560, 2048)
    case("o_proj", 17664, 2048, 2048, resid=True)
    case("sig_out", 16384, 1152, 1152, bias=True, resid=True)
    case("sig_qkv", 16384, 3456, 1152, bias=True)
    case("sig_fc1", 16384, 4304, 1152, bias=True, act="gelu")
    case("sig_fc2", 16384, 1152, 4304, bias=True, resid=True)


if __name__ == "__main__":
    main()
