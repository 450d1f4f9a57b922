"""Data-parallel gradient reduction on CPU: world_size 2, gloo, 127.0.0.1.

Exercises pizero_native.ddp (bucketed all-reduce of the flat gradient arena
driven by the engine's per-layer notifications, no_sync) with the tiny model's
real arena layout; the RCCL path on MI355X is the same code with backend nccl.
"""

import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    try:
        import sys

        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        sys.path.insert(0, root)
        sys.path.insert(0, os.path.join(root, "open-pi-zero_amd"))
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from oracle.pizero_oracle import TINY_DIMS
        from pizero_native.ddp import GradReducer, region_marks
        from src.model.vla.pizero import PiZero
        from tests.golden.make_golden import ref_cfg

        m = PiZero(ref_cfg(TINY_DIMS))
        m.tie_action_proprio_weights()
        ar = m._arena
        g = ar.ensure_grad()
        g.fill_(float(rank + 1))
        red = GradReducer(ar, region_marks(m), bucket_bytes=4096)
        nL = m.joint_model.num_hidden_layers
        vL = len(m.vision_tower.vision_model.encoder.layers)
        order = [("joint", l) for l in reversed(range(nL))] + [("encoders", -1)]
        order += [("vision", i) for i in reversed(range(vL))] + [("vision", -1)]
        launched = []
        orig = red._launch
        red._launch = lambda region, lo, hi, streams=(): (launched.append((region, lo, hi)), orig(region, lo, hi, streams))
        for st, l in order:
            red.notify(st, l)
        red.finish()
        ok = True
        for region in ("action", "vlm"):
            lo, hi = ar.region_range[region]
            ok &= bool(torch.allclose(g[lo:hi], torch.full_like(g[lo:hi], 1.5)))
        lo, hi = ar.region_range["frozen"]
        ok &= bool(torch.all(g[lo:hi] == rank + 1))
        # buckets are disjoint, ordered, and the early ones were launched before finish()
        spans = sorted((lo, hi) for _, lo, hi in launched)
        ok &= all(a[1] <= b[0] for a, b in zip(spans, spans[1:]))
        q.put((rank, ok, len(launched)))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover
        q.put((rank, False, repr(e)))


@pytest.mark.timeout(300)
def test_grad_reducer_two_ranks_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = [q.get(timeout=240) for _ in ps]
    for p in ps:
        p.join(timeout=60)
    assert all(ok for _, ok, _ in res), res
    assert all(n > 2 for _, _, n in res), res
