"""ad-hoc check: gradients of a 4-sample tiny batch in one micro-batch vs 4 accumulated single-sample
micro-batches (the DDP test's comparison without the collective); prints the worst tensors."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "open-pi-zero_amd"))

import torch  # noqa: E402

from oracle.pizero_oracle import TINY_DIMS  # noqa: E402
from tests.pizero_gpu_helpers import build_gpu_model, gpu_inputs  # noqa: E402


def main():
    d = TINY_DIMS
    m = build_gpu_model(d)
    gi = gpu_inputs(m, d, 4)

    def kw(sl):
        return dict(input_ids=gi["input_ids"][sl], pixel_values=gi["pixel_values"][sl], causal_mask=gi["causal_mask"][sl],
                    vlm_position_ids=gi["vpos"][sl], proprio_position_ids=gi["ppos"][sl],
                    action_position_ids=gi["apos"][sl], proprios=gi["proprios"][sl], actions=gi["actions32"][sl],
                    t=gi["t32"][sl], noise=gi["x0"][sl])

    m.zero_grad(set_to_none=True)
    m(**kw(slice(0, 4))).backward()
    torch.cuda.synchronize()
    gref = m._arena.grad.float().clone()
    m.zero_grad(set_to_none=True)
    for i in range(4):
        (m(**kw(slice(i, i + 1))) / 4).backward()
    torch.cuda.synchronize()
    gacc = m._arena.grad.float().clone()
    ar = m._arena
    rows = []
    for n in ar.order:
        if not m._requires_grad(n):
            continue
        a, b = ar.view(n, gacc), ar.view(n, gref)
        nb = float(b.norm())
        if nb > 0:
            rows.append((float((a - b).norm()) / nb, n))
    rows.sort(reverse=True)
    for r, n in rows[:12]:
        print(f"{r:.4g}  {n}")


if __name__ == "__main__":
    main()
