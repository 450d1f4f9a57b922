"""Data-parallel PiZero: bucketed RCCL all-reduce of the flat gradient arena,
overlapped with the native backward (train.py:114-128 used torch DDP).

The arena stores parameters in backward-completion order, so the gradient of
each region becomes final as a growing prefix: after joint layer l of the
last micro-batch, the action-expert and VLM regions are final up to the end
of layer l.  The engine reports each finished layer; the reducer records an
event on the compute stream and enqueues ``all_reduce(AVG)`` of every newly
final slice that reached the bucket size on a dedicated communication stream
(RCCL over xGMI on MI355X; one process per GPU).  Slices are views of the
arena: no bucket copies.  ``no_sync()`` skips communication for gradient
accumulation micro-batches, like DistributedDataParallel.no_sync.
"""

from __future__ import annotations

import contextlib

import torch
import torch.distributed as dist


class GradReducer:
    def __init__(self, arena, region_marks, bucket_bytes=256 << 20, group=None):
        """region_marks: {(stage, layer): {region: end_offset}} -> prefix ends that are final."""
        self.arena = arena
        self.marks = region_marks
        self.bucket = bucket_bytes
        self.group = group
        self.enabled = True
        self.stream = torch.cuda.Stream() if arena.data.is_cuda else None
        # (async, elements) per launched bucket since construction: "async" = the RCCL branch (event on the
        # compute stream, all_reduce(AVG) enqueued on the communication stream)
        self.log = []
        # timing=True: HIP events around every bucket on the communication stream (RCCL time) and around the
        # compute stream's wait for the last bucket in finish() (the exposed, un-overlapped part); read with
        # timing_summary() after a synchronize
        self.timing = False
        self._comm_ev, self._wait_ev = [], []
        self._reset()

    def _reset(self):
        self.done = {r: self.arena.region_range[r][0] for r in ("action", "vlm") if r in self.arena.region_range}
        self.final = dict(self.done)
        self.handles = []

    def _launch(self, region, lo, hi, streams=()):
        g = self.arena.grad[lo:hi]
        if self.stream is None or dist.get_backend(self.group) != "nccl":
            # gloo (CPU tests / single-GPU rehearsal): synchronous SUM then scale, after the side streams' work
            for s in streams:
                torch.cuda.current_stream().wait_stream(s)
            dist.all_reduce(g, op=dist.ReduceOp.SUM, group=self.group)
            g.mul_(1.0 / dist.get_world_size(self.group))
            self.log.append((False, hi - lo))
            return
        ev = torch.cuda.Event()
        ev.record()
        with torch.cuda.stream(self.stream):
            self.stream.wait_event(ev)
            for s in streams:  # gradients of this slice also produced there (the engine's expert stream)
                self.stream.wait_stream(s)
            if self.timing:
                e0 = torch.cuda.Event(enable_timing=True)
                e0.record()
            dist.all_reduce(g, op=dist.ReduceOp.AVG, group=self.group)
            if self.timing:
                e1 = torch.cuda.Event(enable_timing=True)
                e1.record()  # the collective's completion (all_reduce made this stream wait on RCCL's)
                self._comm_ev.append((e0, e1))
            # the arena slice is produced on the compute stream and consumed here: keep the caching
            # allocator from recycling it before the collective ran
            g.record_stream(self.stream)
        self.log.append((True, hi - lo))

    def notify(self, stage, layer, streams=()):
        if not self.enabled:
            return
        ends = self.marks.get((stage, layer))
        if not ends:
            return
        elt = self.arena.grad.element_size()
        for region, end in ends.items():
            self.final[region] = max(self.final[region], end)
            if (self.final[region] - self.done[region]) * elt >= self.bucket:
                self._launch(region, self.done[region], self.final[region], streams)
                self.done[region] = self.final[region]

    def finish(self):
        """Flush every remaining final slice and make the compute stream wait for the reduction."""
        if not self.enabled:
            return
        for region, (lo, hi) in self.arena.region_range.items():
            if region not in self.done:
                continue
            hi8 = (hi + 7) // 8 * 8
            if hi8 > self.done[region]:
                self._launch(region, self.done[region], hi8)
        if self.stream is not None:
            if self.timing:
                w0, w1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                w0.record()  # the compute stream finished its backward
                torch.cuda.current_stream().wait_stream(self.stream)
                w1.record()  # ... and the last bucket landed: w1 - w0 = communication NOT hidden by compute
                self._wait_ev.append((w0, w1))
            else:
                torch.cuda.current_stream().wait_stream(self.stream)
        self._reset()

    def timing_summary(self, steps):
        """{comm_ms_per_step, exposed_ms_per_step, overlap_frac} over the events recorded since the last call
        (the caller synchronizes first); None without timed buckets."""
        if not self._comm_ev:
            return None
        comm = sum(a.elapsed_time(b) for a, b in self._comm_ev)
        exposed = sum(max(0.0, a.elapsed_time(b)) for a, b in self._wait_ev)
        self._comm_ev, self._wait_ev = [], []
        steps = max(1, steps)
        return {"comm_ms_per_step": comm / steps, "exposed_ms_per_step": exposed / steps,
                "overlap_frac": 1.0 - exposed / comm if comm > 0 else None}


def region_marks(model):
    """Map engine notifications to the arena prefix that is final after them."""
    ar = model._arena
    marks = {}

    def end_of(names):
        return max(ar.slots[n].offset + ar.slots[n].numel for n in names if n in ar.slots)

    nL = model.joint_model.num_hidden_layers
    head = ["action_decoder.weight", "action_decoder.bias", "joint_model.mixtures.action.norm.weight"]
    for l in range(nL):
        e = {}
        an = [n for n in ar.order if n.startswith(f"joint_model.mixtures.action.layers.{l}.")
              or n.startswith(f"joint_model.mixtures.proprio.layers.{l}.")]
        vn = [n for n in ar.order if n.startswith(f"joint_model.mixtures.vlm.layers.{l}.")]
        if an:
            e["action"] = max(end_of(an), end_of(head))
        if vn:
            e["vlm"] = end_of(vn)
        marks[("joint", l)] = e
    marks[("encoders", -1)] = {"action": ar.region_range["action"][1]}
    vL = len(model.vision_tower.vision_model.encoder.layers)
    for i in range(vL):
        vn = [n for n in ar.order if n.startswith(f"vision_tower.vision_model.encoder.layers.{i}.")]
        marks[("vision", i)] = {"vlm": end_of(vn)}
    marks[("vision", -1)] = {"vlm": ar.region_range["vlm"][1]}
    return marks


class PiZeroDDP(torch.nn.Module):
    """DistributedDataParallel-compatible wrapper (``.module``, ``no_sync()``, forward -> loss)."""

    def __init__(self, module, bucket_bytes=256 << 20, group=None, broadcast=True, force_reduce=False):
        """force_reduce: reduce even in a world of one rank (an RCCL world_size=1 group exercises the
        overlapped communication-stream path on a single GPU; AVG over one rank is the identity)."""
        super().__init__()
        self.force_reduce = force_reduce
        self.module = module
        # a plain attribute, not a registered submodule (module -> wrapper -> module would make
        # .train() / .eval() / .modules() recurse forever)
        module.__dict__["_ddp_wrapper"] = self
        module.use_ddp = True
        self._sync = True
        ar = module._arena
        ar.ensure_grad()
        if broadcast and dist.is_initialized():
            dist.broadcast(ar.data, src=0, group=group)
        self.reducer = GradReducer(ar, region_marks(module), bucket_bytes, group)

    @contextlib.contextmanager
    def no_sync(self):
        old = self._sync
        self._sync = False
        try:
            yield
        finally:
            self._sync = old

    def forward(self, *args, **kwargs):
        eng = self.module._engine()
        if self._sync and dist.is_initialized() and (dist.get_world_size(self.reducer.group) > 1 or self.force_reduce):
            self.reducer.enabled = True
            eng.hook = self.reducer.notify
            eng.post_backward = self.reducer.finish
        else:
            self.reducer.enabled = False
            eng.hook = None
            eng.post_backward = None
        return self.module(*args, **kwargs)
