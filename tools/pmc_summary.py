"""Summarise the PMC passes of tools/pmc_dominant.sh into profiles/<round>/pmc_dominant.json.

    python tools/pmc_summary.py gpurun_out/<tag>/pmc profiles/r01/pmc_dominant.json

HBM traffic per launch of the bench's dominant kernel (vlm gate|up GeGLU GEMM), corrected as
/opt/skills/guides/MI355X_MICROARCH.md "HBM" prescribes: FETCH_SIZE (KiB) reports half of the
bytes of wide coalesced streaming reads on gfx950 -> x2; WRITE_SIZE (KiB) is exact for 16-B
stores (this kernel's epilogue stores 8 B per lane: uncalibrated, reported as measured).
bench.py reads the JSON and reports `traffic` when its kernel name and shape match.
"""

import collections
import csv
import json
import os
import sys


def per_dispatch(path, kern):
    agg = collections.defaultdict(float)
    dur = {}
    name = None
    for r in csv.DictReader(open(path)):
        if kern not in r["Kernel_Name"]:
            continue
        name = r["Kernel_Name"]
        agg[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        dur[r["Dispatch_Id"]] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6
    out = collections.defaultdict(list)
    for (d, c), v in agg.items():
        out[c].append(v)
    return name, out, list(dur.values())


def mean(x):
    return sum(x) / max(1, len(x))


def main():
    src, dst = sys.argv[1], sys.argv[2]
    dgeglu = os.environ.get("PMC_LAYOUT") == "DGEGLU"  # the down-proj dgrad + GeGLU derivative (pmcdgeglu passes)
    if dgeglu:  # d(g|u)[M, 2I] from dy[M, H] W_down[H, I]: reads dy, W, g|u; writes d(g|u)
        M, N, K = int(os.environ.get("PMC_M", "70656")), 16384, 2048
    else:
        M, N, K = int(os.environ.get("PMC_M", "70656")), 32768, 2048
    kern = sys.argv[3] if len(sys.argv) > 3 else ("gemm8p_kernel<true, false" if dgeglu else "gemm8p_kernel<true, true, true")
    name, fetch, d1 = per_dispatch(os.path.join(src, "fetch", "fetch_counter_collection.csv"), kern)
    _, write, d2 = per_dispatch(os.path.join(src, "write", "write_counter_collection.csv"), kern)
    _, sq, d3 = per_dispatch(os.path.join(src, "sq", "sq_counter_collection.csv"), kern)
    fetch_raw = mean(fetch["FETCH_SIZE"]) * 1024
    write_b = mean(write["WRITE_SIZE"]) * 1024
    if dgeglu:
        algo = 2 * (M * K + N * K) + 2 * (2 * M * 2 * N)  # dy + W read, g|u read and d(g|u) written
    else:
        algo = 2 * (M * K + N * K) + 2 * M * (N // 2) + 2 * M * N  # A + B read, h + saved g|u written
    mfma_cyc = mean(sq["SQ_VALU_MFMA_BUSY_CYCLES"])
    gui = mean(fetch["GRBM_GUI_ACTIVE"])
    ms = mean(d1)
    out = {
        "kernel": name.replace("void (anonymous namespace)::", "").split("(")[0],
        "shape_MNK": [M, N, K],
        "dispatches": len(d1),
        "avg_duration_ms_profiled": ms,
        "fetch_size_bytes_raw": fetch_raw,
        "fetch_bytes_corrected_x2": 2 * fetch_raw,
        "write_size_bytes": write_b,
        "traffic_bytes": 2 * fetch_raw + write_b,
        "algorithmic_bytes": algo,
        "traffic_over_algorithmic": (2 * fetch_raw + write_b) / algo,
        "effective_clock_ghz": gui / 8 / (ms * 1e-3) / 1e9 if ms else None,
        "mfma_busy_frac": mfma_cyc / 1024 / (gui / 8) if gui else None,  # per-SIMD MFMA cycles / wall cycles
        "sq_wait_any_frac": mean(sq["SQ_WAIT_ANY"]) / mean(sq["SQ_WAVE_CYCLES"]),
        "sq_wait_inst_any_frac": mean(sq["SQ_WAIT_INST_ANY"]) / mean(sq["SQ_WAVE_CYCLES"]),
        "sq_active_inst_frac": mean(sq["SQ_ACTIVE_INST_ANY"]) / mean(sq["SQ_WAVE_CYCLES"]),
        "source": "rocprofv3 --pmc passes of tools/pmc_dominant.sh (FETCH_SIZE+GRBM_GUI_ACTIVE, WRITE_SIZE, SQ_*)",
    }
    os.makedirs(os.path.dirname(dst), exist_ok=True)
    json.dump(out, open(dst, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
