"""Config C5 inference (3 images = 768 image tokens + 20 text + 1 proprio, chunk 50, B=1) in one
hipGraph, timed over --iters replays -- the bench.py c5 leg on its own, for rocprofv3 splits.

    python tools/c5_bench.py [--iters 20]
"""

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "open-pi-zero_amd"))

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    from src.utils.config import load_config

    cfg = load_config(os.path.join(ROOT, "open-pi-zero_amd", "config", "train", "bridge.yaml"))
    print(json.dumps(bench.c5_inference(cfg, "cuda", a.iters)))


if __name__ == "__main__":
    torch.manual_seed(0)
    main()
