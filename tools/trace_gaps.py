"""GPU idle time in a rocprofv3 kernel trace: union of the kernel intervals (all streams) over the traced
window, total idle time, a histogram of the gaps and the largest gaps with the kernels on either side.

    python tools/trace_gaps.py <kernel_trace.csv> [--after-ms T] [--top 20]

--after-ms skips the first T ms of the trace (model build, warm-up), --last-ms keeps only the last T ms, so the
numbers describe the timed steps.
"""

from __future__ import annotations

import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--after-ms", type=float, default=0.0)
    ap.add_argument("--last-ms", type=float, default=0.0, help="only the last T ms of the trace (0: all)")
    ap.add_argument("--top", type=int, default=20)
    a = ap.parse_args()
    ev = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:90]))
    ev.sort()
    if not ev:
        print("empty trace")
        return
    t0 = ev[0][0] + int(a.after_ms * 1e6)
    if a.last_ms > 0:
        t0 = max(t0, max(e[1] for e in ev) - int(a.last_ms * 1e6))
    ev = [e for e in ev if e[0] >= t0]
    span0, span1 = ev[0][0], max(e[1] for e in ev)
    busy = 0
    gaps = []
    cur_s, cur_e, cur_n = ev[0][0], ev[0][1], ev[0][2]
    for s, e, n in ev[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            gaps.append((s - cur_e, cur_n, n, cur_e - span0))
            cur_s, cur_e, cur_n = s, e, n
        elif e > cur_e:
            cur_e, cur_n = e, n
    busy += cur_e - cur_s
    span = span1 - span0
    idle = span - busy
    print(f"kernels {len(ev)}  span {span / 1e6:.2f} ms  busy {busy / 1e6:.2f} ms  idle {idle / 1e6:.2f} ms "
          f"({100.0 * idle / max(1, span):.2f} %)")
    edges = [1e3, 2e3, 5e3, 1e4, 5e4, 1e5, 1e6, 1e12]
    hist = [[0, 0] for _ in edges]
    for g, *_ in gaps:
        for i, e in enumerate(edges):
            if g < e:
                hist[i][0] += 1
                hist[i][1] += g
                break
    lo = 0
    for (c, tot), e in zip(hist, edges):
        print(f"  gaps {lo / 1e3:>8.0f}-{e / 1e3:<8.0f} us: {c:6d}  total {tot / 1e6:8.3f} ms")
        lo = e
    for g, n0, n1, at in sorted(gaps, reverse=True)[: a.top]:
        print(f"  {g / 1e3:9.1f} us at {at / 1e6:9.2f} ms  after {n0}  before {n1}")


if __name__ == "__main__":
    main()
