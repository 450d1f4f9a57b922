"""PiZeroDDP through the real engine hooks on the MI355X: 2 ranks on one GPU (gloo, 127.0.0.1).

Rank r trains on samples {2r, 2r+1} of a 4-sample tiny batch as 2 micro-batches (the first under
no_sync, the second synced: train.py:350-368).  The averaged gradient arena must equal one process's
gradients on the whole 4-sample batch (bf16 accumulation-order noise only), the no_sync micro-batch
must leave ranks' gradients unreduced, and buckets must be launched during the backward (before the
flush).  Wrapping the model in torch DistributedDataParallel instead fails loudly (the native
backward fires no per-parameter hooks).  RCCL cannot put 2 ranks on one GPU, so the collective here
is gloo; the RCCL/xGMI path is the same code with backend "nccl" (bench.py --gpus N).
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


def _worker(rank, world, port, q):
    try:
        import sys

        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        sys.path.insert(0, root)
        sys.path.insert(0, os.path.join(root, "open-pi-zero_amd"))
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        import torch.distributed as dist

        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from oracle.pizero_oracle import TINY_DIMS
        from pizero_native.ddp import PiZeroDDP
        from tests.pizero_gpu_helpers import build_gpu_model, gpu_inputs

        d = TINY_DIMS
        m = build_gpu_model(d)
        gi = gpu_inputs(m, d, 4)
        res = {}

        def mb(idx):
            sl = slice(idx, idx + 1)
            return dict(input_ids=gi["input_ids"][sl], pixel_values=gi["pixel_values"][sl],
                        causal_mask=gi["causal_mask"][sl], vlm_position_ids=gi["vpos"][sl],
                        proprio_position_ids=gi["ppos"][sl], action_position_ids=gi["apos"][sl],
                        proprios=gi["proprios"][sl], actions=gi["actions32"][sl], t=gi["t32"][sl],
                        noise=gi["x0"][sl])

        # torch DDP cannot drive the native backward: loud error, not a silent un-reduced step
        try:
            ddp = torch.nn.parallel.DistributedDataParallel(m)
            ddp(**mb(0))
            res["torch_ddp"] = "no error"
        except RuntimeError as e:
            res["torch_ddp"] = "PiZeroDDP" in str(e)
        m.zero_grad(set_to_none=True)

        w = PiZeroDDP(m, bucket_bytes=1 << 16)
        launched = []
        orig_launch, orig_finish = w.reducer._launch, w.reducer.finish
        phase = {"flushing": False}

        def launch(region, lo, hi, streams=()):
            launched.append(phase["flushing"])
            return orig_launch(region, lo, hi, streams)

        def finish():
            phase["flushing"] = True
            orig_finish()
            phase["flushing"] = False

        w.reducer._launch = launch
        eng = m._engine()
        m.zero_grad(set_to_none=True)
        with w.no_sync():
            (w(**mb(2 * rank)) / 2).backward()
        g1 = m._arena.grad.float().clone()
        gl = [torch.empty_like(g1) for _ in range(world)]
        dist.all_gather(gl, g1)
        res["no_sync_unreduced"] = not torch.equal(gl[0], gl[1])
        (w(**mb(2 * rank + 1)) / 2).backward()
        torch.cuda.synchronize()
        res["buckets_during_backward"] = sum(1 for f in launched if not f)
        gavg = m._arena.grad.float().clone()
        gl = [torch.empty_like(gavg) for _ in range(world)]
        dist.all_gather(gl, gavg)
        res["ranks_equal"] = torch.equal(gl[0], gl[1])
        w.reducer.finish = orig_finish
        if rank == 0:
            # one process, the whole 4-sample batch
            eng.hook = eng.post_backward = None
            m._ddp_wrapper = None
            dist.destroy_process_group()
            m.zero_grad(set_to_none=True)
            loss = m(input_ids=gi["input_ids"], pixel_values=gi["pixel_values"], causal_mask=gi["causal_mask"],
                     vlm_position_ids=gi["vpos"], proprio_position_ids=gi["ppos"], action_position_ids=gi["apos"],
                     proprios=gi["proprios"], actions=gi["actions32"], t=gi["t32"], noise=gi["x0"])
            loss.backward()
            torch.cuda.synchronize()
            ar = m._arena
            gref = ar.grad.float()
            worst = 0.0
            for n in ar.order:
                if not m._requires_grad(n):
                    continue
                if n.startswith("vision_tower") and n.endswith("self_attn.k_proj.bias"):
                    continue  # exact gradient 0 (softmax shift invariance): both sides are rounding noise
                a, b = ar.view(n, gavg), ar.view(n, gref)
                nb = float(b.norm())
                if nb > 0:
                    worst = max(worst, float((a - b).norm()) / nb)
            res["worst_rel"] = worst
        else:
            dist.destroy_process_group()
        q.put((rank, res))
    except Exception as e:  # pragma: no cover
        import traceback

        q.put((rank, {"error": repr(e), "tb": traceback.format_exc()}))


@pytest.mark.timeout(600)
def test_pizero_ddp_two_ranks_one_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=540) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    for r in (0, 1):
        assert "error" not in res[r], res[r]
        assert res[r]["torch_ddp"] is True, res[r]
        assert res[r]["no_sync_unreduced"], res[r]
        assert res[r]["ranks_equal"], res[r]
        assert res[r]["buckets_during_backward"] >= 2, res[r]
    print("DDP vs single-process worst per-tensor rel-L2:", res[0]["worst_rel"])
    assert res[0]["worst_rel"] < 2e-2, res[0]
