#!/bin/bash
# PMC of the fused attention kernels at the bench shape (tools/flash_bench.py), one counter group per pass.
# usage (gpurun, repo root): bash tools/pmc_flash.sh OUTDIR
set -e
OUT=${1:-gpurun_out/pmcf}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
CMD="python3 tools/flash_bench.py --iters 2"
timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d "$OUT/lds" -o lds \
  --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_WAVE_CYCLES -- $CMD > "$OUT.lds.log" 2>&1
timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d "$OUT/busy" -o busy \
  --pmc SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_WAIT_ANY GRBM_GUI_ACTIVE -- $CMD > "$OUT.busy.log" 2>&1
echo pmc ok
