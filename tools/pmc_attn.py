"""Per-kernel PMC ratios of the fused attention kernels (tools/flash_bench.py workload).

    bash: rocprofv3 --pmc <group> -d OUT/<pass> ... -- python3 tools/flash_bench.py --iters 2  (one pass per group)
    python tools/pmc_attn.py OUT

Prints, per kernel, the mean over dispatches of each counter and the issue/wait fractions of
SQ_WAVE_CYCLES (quad-cycle units cancel), MFMA busy vs GRBM_GUI_ACTIVE / 8 XCDs.
"""
import collections
import csv
import glob
import os
import sys


def main():
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for path in glob.glob(os.path.join(sys.argv[1], "**", "*counter_collection.csv"), recursive=True):
        per = collections.defaultdict(float)
        names = {}
        for r in csv.DictReader(open(path)):
            k = (r["Dispatch_Id"], r["Counter_Name"])
            per[k] += float(r["Counter_Value"])
            names[r["Dispatch_Id"]] = r["Kernel_Name"].replace("void (anonymous namespace)::", "").split("(")[0]
        for (d, c), v in per.items():
            agg[names[d]][c].append(v)
    for kern, cs in sorted(agg.items()):
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        line = [kern[:48]]
        wc = m.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS",
                      "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_SCA", "SQ_WAIT_INST_LDS"):
                if c in m:
                    line.append(f"{c[3:]}={m[c] / wc:.2f}")
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m and "GRBM_GUI_ACTIVE" in m:
            line.append(f"mfma_busy={m['SQ_VALU_MFMA_BUSY_CYCLES'] / 1024 / (m['GRBM_GUI_ACTIVE'] / 8):.3f}")
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_MFMA", "SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT",
                  "SQ_LDS_IDX_ACTIVE", "SQ_LDS_DATA_FIFO_FULL", "SQ_LDS_CMD_FIFO_FULL", "SQ_INST_LEVEL_LDS",
                  "SQ_INST_LEVEL_VMEM", "SQ_INSTS_VMEM_RD", "SQ_BUSY_CYCLES", "SQ_WAVES"):
            if c in m:
                line.append(f"{c[3:]}={m[c]:.3g}")
        print("  ".join(line))


if __name__ == "__main__":
    main()
