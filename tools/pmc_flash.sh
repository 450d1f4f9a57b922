#!/bin/bash
# PMC passes over tools/flash_bench.py (one counter group per rocprofv3 run)
set -e
OUT=${1:-gpurun_out/pmcf}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p "$OUT"
timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d "$OUT/a" -o a \
  --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS \
  -- python3 tools/flash_bench.py --iters 2 > "$OUT/a.log" 2>&1
timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d "$OUT/b" -o b \
  --pmc FETCH_SIZE GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_INSTS_VMEM_RD \
  -- python3 tools/flash_bench.py --iters 2 > "$OUT/b.log" 2>&1
echo pmc ok
