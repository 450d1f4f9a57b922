"""Action-chunk inference latency (B=1 default): eager native path and hipGraph replay.

    python tools/infer_bench.py [--bsz 1] [--iters 20]
"""

import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "open-pi-zero_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bsz", type=int, default=1)
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    from bench import synthetic_batch
    from pizero_native.graph import InferenceGraph
    from src.model.vla.pizero import PiZero
    from src.utils.config import load_config

    cfg = load_config(os.path.join(ROOT, "open-pi-zero_amd", "config", "train", "bridge.yaml"))
    dev = torch.device("cuda")
    m = PiZero(cfg, device=dev, dtype=torch.bfloat16, init="default")
    m.tie_action_proprio_weights()
    m.freeze_all_weights()
    m.eval()
    d = m._engine().d
    gi = synthetic_batch(m, args.bsz, dev, torch.Generator().manual_seed(7))
    itp, amask = m.split_full_mask_into_submasks(gi["causal_mask"])
    noise = torch.randn(args.bsz, d.H, d.A, device=dev)

    def eager():
        return m.infer_action(gi["input_ids"], gi["pixel_values"], itp, amask, gi["vlm_position_ids"],
                              gi["proprio_position_ids"], gi["action_position_ids"], gi["proprios"], noise=noise)

    for _ in range(3):
        a0 = eager()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(5):
        eager()
    torch.cuda.synchronize()
    eager_ms = (time.perf_counter() - t) / 5 * 1e3
    g = InferenceGraph(m, args.bsz)
    g.load(gi["input_ids"], gi["pixel_values"], m._prefix_counts(itp), gi["vlm_position_ids"],
           gi["proprio_position_ids"], gi["action_position_ids"], gi["proprios"], noise)
    g.capture()
    out = g.replay()
    torch.cuda.synchronize()
    diff = (out.float() - a0.float()).abs().max().item()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.iters):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    print(f"bsz={args.bsz} eager {eager_ms:.2f} ms  graph {e0.elapsed_time(e1) / args.iters:.2f} ms  "
          f"|graph-eager|max {diff:.2e}")


if __name__ == "__main__":
    main()
