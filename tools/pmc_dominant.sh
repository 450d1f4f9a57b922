#!/bin/bash
# HBM traffic of the bench's dominant launch (vlm gate|up GeGLU GEMM, M=276*micro-batch N=32768 K=2048; PMC_M, default
# 70656 = micro-batch 256),
# one counter group per rocprofv3 pass (MI355X_MICROARCH.md "HBM": FETCH_SIZE and WRITE_SIZE cannot share a pass).
# usage (gpurun, repo root): bash tools/pmc_dominant.sh OUTDIR
set -e
OUT=${1:-gpurun_out/pmc}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
CMD=${PMC_CMD:-"python3 tools/gemm_one.py --layout GEGLU --M ${PMC_M:-70656} --N 32768 --K 2048 --iters 3"}
timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d "$OUT/fetch" -o fetch \
  --pmc FETCH_SIZE GRBM_GUI_ACTIVE -- $CMD > "$OUT.fetch.log" 2>&1
timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d "$OUT/write" -o write \
  --pmc WRITE_SIZE -- $CMD > "$OUT.write.log" 2>&1
timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d "$OUT/sq" -o sq \
  --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  -- $CMD > "$OUT.sq.log" 2>&1
echo pmc ok
