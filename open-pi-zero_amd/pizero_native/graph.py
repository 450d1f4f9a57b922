"""hipGraph-captured action-chunk inference (pizero.py:416-490 as ONE graph replay).

The whole chunk -- SigLIP, prefix prefill writing the static KV cache, and the
10 Euler denoise steps through the action expert -- is recorded once into a
torch.cuda.CUDAGraph (= hipGraph on ROCm).  Every kernel of the path is a
libpizero_hip.so launch on the capture stream; all buffers come from the
graph's private pool; inputs are copied into static tensors before replay.
Replay removes the ~1.7k host launches per chunk (the reference's
eager path is launch-bound).
"""

from __future__ import annotations

import torch


class InferenceGraph:
    def __init__(self, model, bsz, clip=True):
        self.m = model
        self.B = bsz
        self.clip = clip
        e = model._engine()
        d = e.d
        dev = model._dev()
        self.static = dict(
            ids=torch.zeros(bsz, d.P, device=dev, dtype=torch.int64),
            pix=torch.zeros(bsz * d.n_images, 3, d.img, d.img, device=dev, dtype=torch.bfloat16),
            cnt=torch.full((bsz,), d.P, device=dev, dtype=torch.int32),
            vpos=torch.arange(1, d.P + 1, device=dev).repeat(bsz, 1),
            ppos=torch.arange(1, d.C + 1, device=dev).repeat(bsz, 1),
            apos=torch.arange(d.C + 1, d.C + d.H + 1, device=dev).repeat(bsz, 1),
            proprios=torch.zeros(bsz, d.C, d.Pd, device=dev, dtype=torch.float32),
            noise=torch.zeros(bsz, d.H, d.A, device=dev, dtype=torch.float32),
        )
        self.k, self.v = model._kv_buffers(bsz)
        self.graph = None
        self.out = None
        self._f8 = None

    def _run(self):
        s = self.static
        return self.m._engine().infer_action(s["ids"], s["pix"], s["cnt"], s["vpos"], s["ppos"], s["apos"],
                                              s["proprios"], s["noise"], self.k, self.v, clip=self.clip)

    def load(self, input_ids, pixel_values, cnt, vpos, ppos, apos, proprios, noise):
        s = self.static
        s["ids"].copy_(input_ids)
        s["pix"].copy_(pixel_values.reshape(s["pix"].shape))
        s["cnt"].copy_(cnt)
        s["vpos"].copy_(vpos)
        s["ppos"].copy_(ppos)
        s["apos"].copy_(apos)
        s["proprios"].copy_(proprios.reshape(s["proprios"].shape))
        s["noise"].copy_(noise.reshape(s["noise"].shape))

    def capture(self):
        # re-quantise stale fp8 codes first, so the codes recorded here are the ones the captured launches read
        # (the warm-up's infer_action would otherwise replace them and force a needless re-capture)
        e = self.m._engine()
        e.fp8_refresh()
        self._f8 = e.f8
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(2):  # warm-up: kernel attributes, rope tables, allocator
                self._run()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.out = self._run()
        torch.cuda.synchronize()
        return self

    def replay(self):
        # bf16 weights are read in place (an optimizer step / checkpoint load is seen by the next replay);
        # fp8 codes and their per-tensor scales are baked into the captured launches, so a weight change
        # since the capture re-quantises them (Engine.fp8_refresh) and re-captures the graph
        e = self.m._engine()
        e.derived_refresh()  # in place: the captured launches keep their pointers
        if e.f8 is not self._f8 or e.fp8_refresh():
            self.capture()
        self.graph.replay()
        return self.out
