"""The RCCL branch of the data-parallel reducer, executed on the MI355X.

A one-rank ``nccl`` (= RCCL on ROCm) process group on the single GPU, with PiZeroDDP forced on
(``force_reduce=True``: AVG over one rank is the identity).  This runs exactly the code an 8-GPU job
runs in its last micro-batch (reference train.py:114-128, 350-368): the engine's per-layer hook
records an event on the compute stream and enqueues ``all_reduce(AVG)`` of each newly final
gradient-arena slice on the communication stream while the backward continues; ``finish()`` flushes
the rest and makes the compute stream wait.  Asserts: the RCCL (async) branch ran, buckets were
enqueued during the backward (before the flush), every slice of the trainable arena was reduced once,
and the gradient arena is BITWISE equal to the same backward without the wrapper.  ``no_sync`` leaves
the reducer idle.  A third step delays the engine's expert side stream and snapshots every bucket on the
communication stream after its collective: each snapshot equals the final gradients.
"""

import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(port, q):
    try:
        import sys

        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        sys.path.insert(0, root)
        sys.path.insert(0, os.path.join(root, "open-pi-zero_amd"))
        import torch.distributed as dist

        torch.cuda.set_device(0)
        dev = torch.device("cuda:0")
        dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)
        from oracle.pizero_oracle import TINY_DIMS
        from pizero_native.ddp import PiZeroDDP
        from tests.pizero_gpu_helpers import build_gpu_model, gpu_inputs

        d = TINY_DIMS
        m = build_gpu_model(d)
        gi = gpu_inputs(m, d, 3)
        kw = dict(input_ids=gi["input_ids"], pixel_values=gi["pixel_values"], causal_mask=gi["causal_mask"],
                  vlm_position_ids=gi["vpos"], proprio_position_ids=gi["ppos"], action_position_ids=gi["apos"],
                  proprios=gi["proprios"], actions=gi["actions32"], t=gi["t32"], noise=gi["x0"])
        res = {"backend": dist.get_backend()}
        # reference gradients: plain backward, no wrapper
        m.zero_grad(set_to_none=True)
        m(**kw).backward()
        torch.cuda.synchronize()
        gref = m._arena.grad.clone()

        w = PiZeroDDP(m, bucket_bytes=1 << 16, force_reduce=True)
        red = w.reducer
        phase = {"flushing": False, "during": 0}
        orig_launch, orig_finish = red._launch, red.finish

        def launch(region, lo, hi, streams=()):
            if not phase["flushing"]:
                phase["during"] += 1
            return orig_launch(region, lo, hi, streams)

        def finish():
            phase["flushing"] = True
            orig_finish()
            phase["flushing"] = False

        red._launch = launch
        eng = m._engine()
        eng.post_backward = None  # rebound by the wrapper's forward
        # no_sync: the reducer stays idle
        m.zero_grad(set_to_none=True)
        with w.no_sync():
            w(**kw).backward()
        torch.cuda.synchronize()
        res["no_sync_launches"] = len(red.log)
        res["no_sync_equal"] = torch.equal(m._arena.grad, gref)
        # synced step: hooks -> RCCL buckets on the comm stream during the backward
        m.zero_grad(set_to_none=True)
        loss = w(**kw)
        red.finish = finish
        eng.post_backward = red.finish
        loss.backward()
        torch.cuda.synchronize()
        res["launches"] = len(red.log)
        res["async_launches"] = sum(1 for a, _ in red.log if a)
        res["during_backward"] = phase["during"]
        res["reduced_elems"] = sum(n for _, n in red.log)
        ar = m._arena
        res["trainable_elems"] = sum((ar.region_range[r][1] + 7) // 8 * 8 - ar.region_range[r][0]
                                     for r in ("action", "vlm") if r in ar.region_range)
        res["bitwise_equal"] = torch.equal(ar.grad, gref)
        res["max_abs_diff"] = float((ar.grad.float() - gref.float()).abs().max())
        # the communication stream must wait for the expert side stream before each bucket.  Delay the
        # side stream (a ~20 ms spin before every layer's expert q|k|v backward) and snapshot each bucket's slice
        # on the communication stream right after its all_reduce: every snapshot must equal the final gradients
        # (a bucket that read its slice before the side stream's wgrads landed would differ)
        snaps = []
        red.finish = orig_finish
        eng.post_backward = None

        def launch_snap(region, lo, hi, streams=()):
            orig_launch(region, lo, hi, streams)
            with torch.cuda.stream(red.stream):
                snaps.append((lo, hi, m._arena.grad[lo:hi].clone()))

        red._launch = launch_snap
        orig_qkv = eng._qkv_backward
        main_stream = torch.cuda.current_stream()
        delayed = {"n": 0}

        def qkv_delayed(*a, **k):
            if torch.cuda.current_stream() != main_stream:
                torch.cuda._sleep(40_000_000)
                delayed["n"] += 1
            return orig_qkv(*a, **k)

        eng._qkv_backward = qkv_delayed
        m.zero_grad(set_to_none=True)
        loss = w(**kw)
        eng.post_backward = red.finish
        loss.backward()
        torch.cuda.synchronize()
        eng._qkv_backward = orig_qkv
        res["side_delays"] = delayed["n"]
        res["snapshots"] = len(snaps)
        res["snapshots_final"] = all(torch.equal(sn, m._arena.grad[lo:hi]) for lo, hi, sn in snaps)
        res["delayed_bitwise_equal"] = torch.equal(m._arena.grad, gref)
        dist.destroy_process_group()
        q.put(res)
    except Exception as e:  # pragma: no cover
        import traceback

        q.put({"error": repr(e), "tb": traceback.format_exc()})


@pytest.mark.timeout(300)
def test_rccl_reducer_branch_world1_bitwise():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_worker, args=(_free_port(), q))
    p.start()
    res = q.get(timeout=280)
    p.join(timeout=60)
    print("RCCL world-1 reducer:", res)
    assert "error" not in res, res
    assert res["backend"] == "nccl", res
    assert res["no_sync_launches"] == 0 and res["no_sync_equal"], res
    assert res["async_launches"] == res["launches"] >= 3, res  # every bucket took the RCCL branch
    assert res["during_backward"] >= 2, res  # enqueued while the backward was still running
    assert res["reduced_elems"] == res["trainable_elems"], res  # each final slice reduced exactly once
    assert res["bitwise_equal"], res
    assert res["side_delays"] >= 1 and res["snapshots"] >= 3, res  # the side stream ran (and was delayed)
    assert res["snapshots_final"], res  # every collective read the finished slice, side-stream wgrads included
    assert res["delayed_bitwise_equal"], res
