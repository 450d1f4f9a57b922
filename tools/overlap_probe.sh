# Which kernels run concurrently with the SigLIP forward attention inside the training step (kernel trace of
# 1 warm-up + 1 timed step, no inference legs): for every flash_fwd_sig dispatch, its duration, queue and the
# kernels on other queues that overlap it.  usage (gpurun): bash tools/overlap_probe.sh OUTDIR
set -e
OUT=${1:-gpurun_out/ovl}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d "$OUT" -o ovl \
  -- python3 bench.py --steps 1 --warmup 1 --no-infer --no-cpu-baseline > "$OUT.log" 2>&1
python3 - "$OUT" <<'PY' > "$OUT.txt"
import csv, glob, sys
rows = []
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
for r in rows:
    r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
rows.sort(key=lambda r: r["s"])
sig = [r for r in rows if "flash_fwd_sig" in r["Kernel_Name"]]
print(len(rows), "dispatches;", len(sig), "flash_fwd_sig")
keys = [k for k in rows[0] if "Queue" in k or "Stream" in k]
print("queue/stream columns:", keys)
# every kernel's longest dispatch against its median (a stalled dispatch stands out), and same-queue overlaps:
# dispatch n + 1 starting before dispatch n ends on one queue (in-order streams: a timestamp artefact or a real race)
import statistics
by = {}
for r in rows:
    by.setdefault(r["Kernel_Name"][:80], []).append(r["e"] - r["s"])
print("longest dispatch / median per kernel (top 8 by ratio):")
rat = sorted(((max(v) / max(1, statistics.median(v)), k, max(v), statistics.median(v), len(v)) for k, v in by.items()),
             reverse=True)
for q, k, mx, md, n in rat[:8]:
    print(f"    x{q:8.1f}  max {mx / 1e6:9.3f} ms  median {md / 1e6:8.3f} ms  n {n:5d}  {k}")
byq = {}
for r in rows:
    byq.setdefault((r.get("Queue_Id"), r.get("Stream_Id")), []).append(r)
for q, lst in byq.items():
    lst.sort(key=lambda r: r["s"])
    ov = [(a["e"] - b["s"]) for a, b in zip(lst, lst[1:]) if b["s"] < a["e"]]
    print(f"queue/stream {q}: {len(lst)} dispatches, {len(ov)} start before the previous one ends"
          + (f" (overlap max {max(ov) / 1e3:.1f} us, median {statistics.median(ov) / 1e3:.1f} us)" if ov else ""))
for r in sig[:6] + sig[-3:]:
    d = (r["e"] - r["s"]) / 1e6
    ov = [o for o in rows if o is not r and o["s"] < r["e"] and o["e"] > r["s"]]
    print(f"sig dispatch {d:.3f} ms", {k: r[k] for k in keys}, "grid", r.get("Grid_Size", r.get("Grid_Size_X")),
          "wg", r.get("Workgroup_Size", r.get("Workgroup_Size_X")), "lds", r.get("LDS_Block_Size", r.get("Lds_Size")),
          "scratch", r.get("Scratch_Size", r.get("Private_Segment_Size")), "vgpr", r.get("VGPR_Count", r.get("Arch_VGPR_Count")))
    for o in ov[:8]:
        print(f"    overlaps {(o['e'] - o['s']) / 1e6:.3f} ms", {k: o[k] for k in keys}, o["Kernel_Name"][:70])
PY
rm -rf "$OUT"
echo overlap ok
