"""Launcher (scripts/run.py:34-76 equivalent without hydra): load a config, instantiate its agent, run.

    python open-pi-zero_amd/scripts/run.py --config-name=bridge [key=value ...]
    torchrun --nproc-per-node N --master-addr 127.0.0.1 open-pi-zero_amd/scripts/run.py --config-name=bridge
"""

import argparse
import logging
import os
import random
import sys

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from src.utils.config import cfg_get, instantiate, load_config  # noqa: E402


def _parse_value(v):
    for cast in (int, float):
        try:
            return cast(v)
        except ValueError:
            pass
    return {"true": True, "false": False, "null": None, "none": None}.get(v.lower(), v)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--config-name", default="bridge")
    ap.add_argument("--config-path", default=os.path.join(HERE, "config", "train"))
    ap.add_argument("overrides", nargs="*")
    args = ap.parse_args(argv)
    ov = dict(o.split("=", 1) for o in args.overrides)
    cfg = load_config(os.path.join(args.config_path, args.config_name + ".yaml"),
                      {k: _parse_value(v) for k, v in ov.items()})
    logging.basicConfig(level=logging.INFO, format="[%(asctime)s][%(name)s] %(message)s")
    seed = int(cfg_get(cfg, "seed", 42)) + int(os.environ.get("RANK", "0"))
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    agent = instantiate({"_target_": cfg_get(cfg, "_target_")}, cfg=cfg)
    agent.run()
    if torch.distributed.is_initialized():
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
