#!/bin/bash
# PMC passes (SQ wait/LDS counters, then HBM fetch) for one GEMM layout under both large-GEMM variants.
# usage (on the GPU box, from the repo root): bash tools/pmc_gemm.sh LAYOUT M N K OUTDIR
set -e
L=$1; M=$2; N=$3; K=$4; OUT=$5
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for V in 8phase 2stage; do
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "$OUT/${L}_${V}_sq" -o sq \
    --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES \
    -- python3 tools/gemm_one.py --layout "$L" --M "$M" --N "$N" --K "$K" --variant "$V" --iters 3
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "$OUT/${L}_${V}_fetch" -o fetch \
    --pmc FETCH_SIZE GRBM_GUI_ACTIVE \
    -- python3 tools/gemm_one.py --layout "$L" --M "$M" --N "$N" --K "$K" --variant "$V" --iters 3
done
