"""Per-kernel PMC summary of the fused attention kernels (tools/pmc_flash.sh passes over tools/flash_bench.py).

    python tools/pmc_attn.py OUTDIR [out.json]

Per kernel, the mean over dispatches of every counter, and the derived figures:
  - HBM traffic: FETCH_SIZE x2 (gfx950 streaming-read correction, MI355X_MICROARCH.md "HBM") + WRITE_SIZE;
  - issue / wait fractions of SQ_WAVE_CYCLES (quad-cycle units cancel): WAIT_ANY (parked at s_waitcnt /
    barrier), WAIT_INST_ANY (issue stall), ACTIVE_INST_* (issuing);
  - MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / 1024 SIMDs / (GRBM_GUI_ACTIVE / 8 XCDs);
  - LDS bank-conflict share = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE; effective clock GRBM / 8 / duration.
"""
import collections
import csv
import glob
import json
import os
import sys


def load(root):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    for path in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        per = collections.defaultdict(float)
        names, d = {}, {}
        for r in csv.DictReader(open(path)):
            k = (r["Dispatch_Id"], r["Counter_Name"])
            per[k] += float(r["Counter_Value"])
            names[r["Dispatch_Id"]] = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]
            if "Start_Timestamp" in r and r["Start_Timestamp"]:
                d[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6
        for (disp, c), v in per.items():
            agg[names[disp]][c].append(v)
        if "fetch" in os.path.basename(path):
            for disp, ms in d.items():
                dur[names[disp]].append(ms)
    return agg, dur


def main():
    agg, dur = load(sys.argv[1])
    out = {}
    for kern, cs in sorted(agg.items()):
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        r = {"dispatches": max(len(v) for v in cs.values()), "counters": m}
        if dur.get(kern):
            r["avg_duration_ms_profiled"] = sum(dur[kern]) / len(dur[kern])
        if "FETCH_SIZE" in m:
            r["fetch_bytes_corrected_x2"] = 2 * 1024 * m["FETCH_SIZE"]
        if "WRITE_SIZE" in m:
            r["write_bytes"] = 1024 * m["WRITE_SIZE"]
        if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
            r["traffic_bytes"] = r["fetch_bytes_corrected_x2"] + r["write_bytes"]
        wc = m.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS",
                      "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_MISC", "SQ_WAIT_INST_LDS"):
                if c in m:
                    r[c[3:].lower() + "_frac"] = m[c] / wc
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m and "GRBM_GUI_ACTIVE" in m:
            r["mfma_busy_frac"] = m["SQ_VALU_MFMA_BUSY_CYCLES"] / 1024 / (m["GRBM_GUI_ACTIVE"] / 8)
        if "SQ_LDS_BANK_CONFLICT" in m and m.get("SQ_LDS_IDX_ACTIVE"):
            r["lds_bank_conflict_frac"] = m["SQ_LDS_BANK_CONFLICT"] / m["SQ_LDS_IDX_ACTIVE"]
        if "GRBM_GUI_ACTIVE" in m and r.get("avg_duration_ms_profiled"):
            r["effective_clock_ghz"] = m["GRBM_GUI_ACTIVE"] / 8 / (r["avg_duration_ms_profiled"] * 1e-3) / 1e9
        if m.get("SQ_INSTS_MFMA"):
            for c in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU"):
                if c in m:
                    r[c[9:].lower() + "_per_mfma"] = m[c] / m["SQ_INSTS_MFMA"]
        out[kern] = r
        show = {k: (round(v, 3) if isinstance(v, float) else v) for k, v in r.items() if k != "counters"}
        print(kern[:60], json.dumps(show))
    if len(sys.argv) > 2:
        os.makedirs(os.path.dirname(sys.argv[2]) or ".", exist_ok=True)
        json.dump({"source": "rocprofv3 --pmc passes of tools/pmc_flash.sh over tools/flash_bench.py --default-only",
                   "kernels": out}, open(sys.argv[2], "w"), indent=1)


if __name__ == "__main__":
    main()
