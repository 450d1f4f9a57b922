#!/bin/bash
# LDS counters of the dominant launch (vlm gate|up GeGLU GEMM, micro-batch 256): bank-conflict cycles against all
# LDS-array cycles, LDS instructions, per dispatch of the 8-phase kernel.  usage (gpurun): bash tools/pmc_lds.sh OUTDIR
set -e
OUT=${1:-gpurun_out/pmcl}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
CMD=${PMC_CMD:-"python3 tools/gemm_one.py --layout GEGLU --M 70656 --N 32768 --K 2048 --iters 3"}
timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d "$OUT/lds" -o lds \
  --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_LDS_ADDR_CONFLICT GRBM_GUI_ACTIVE -- $CMD > "$OUT.lds.log" 2>&1
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
tot, n = collections.defaultdict(float), collections.Counter()
for f in glob.glob(sys.argv[1] + "/lds/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "gemm8" in r.get("Kernel_Name", ""):
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
            n[r["Counter_Name"]] += 1
for k in sorted(tot):
    print(f"{k}: {tot[k] / max(n[k], 1):.4g} per dispatch-row ({n[k]} rows)")
PY
echo pmc lds ok
