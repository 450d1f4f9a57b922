"""Split one hipGraph action chunk of an infer_bench kernel trace into prefill / denoise kernel time.

    python tools/infer_trace_split.py gpurun_out/<tag>/infprof/infer_kernel_trace.csv
"""
import collections
import csv
import sys


def _step_start(r):
    """first kernel of a denoise step: the time embedding (separate glue) or pz_action_in (fused glue, ABI 20)"""
    return "time_embed" in r["Kernel_Name"] or "action_in_kernel" in r["Kernel_Name"]


def main():
    rows = [r for r in csv.DictReader(open(sys.argv[1])) if r.get("Start_Timestamp") and r.get("End_Timestamp")]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    idx = [i for i, r in enumerate(rows) if "patchify" in r["Kernel_Name"]]  # first kernel of a chunk
    # the last whole chunk: a patchify-to-patchify segment with exactly 10 denoise steps (bench.c5_inference also
    # replays prefill-only and denoise-only graphs after the chunk timing)
    ch = None
    for k in range(len(idx) - 2, -1, -1):
        seg = rows[idx[k]:idx[k + 1]]
        if sum(_step_start(r) for r in seg) == 10:
            ch = seg
            break
    if ch is None:
        ch = rows[idx[-2]:idx[-1]]
    t0 = int(ch[0]["Start_Timestamp"])
    te = [i for i, r in enumerate(ch) if _step_start(r) or "denoise" in r["Kernel_Name"]]
    dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3  # noqa: E731
    print(f"chunk: {len(ch)} kernels, wall {(int(ch[-1]['End_Timestamp']) - t0) / 1e3:.1f} us, "
          f"busy {sum(map(dur, ch)):.1f} us; prefill {te[0]} kernels, "
          f"{(int(ch[te[0]]['Start_Timestamp']) - t0) / 1e3:.1f} us")
    for name, seg in (("prefill", ch[:te[0]]), ("denoise (10 steps)", ch[te[0]:])):
        d = collections.defaultdict(lambda: [0, 0.0])
        for r in seg:
            n = r["Kernel_Name"].replace("void (anonymous namespace)::", "").replace("(anonymous namespace)::", "").split("(")[0][:50]
            d[n][0] += 1
            d[n][1] += dur(r)
        print(f"{name}: {len(seg)} kernels, {sum(v[1] for v in d.values()):.1f} us")
        for k, v in sorted(d.items(), key=lambda x: -x[1][1])[:14]:
            print(f"   {k:50s} {v[0]:5d} {v[1]:8.1f}")


if __name__ == "__main__":
    main()
