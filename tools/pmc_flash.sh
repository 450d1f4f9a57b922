#!/bin/bash
# PMC of the training-default fused attention kernels at micro-batch 256 (tools/flash_bench.py --default-only):
# joint flash_fwd_probs / flash_bwd_ds <256>, SigLIP flash_{fwd,bwd_q,bwd_kv}_unit <72>.  One counter group per
# rocprofv3 pass (MI355X_MICROARCH.md "rocprofv3 PMC slots": 8 SQ, FETCH_SIZE and WRITE_SIZE in separate passes).
# usage (gpurun, repo root): bash tools/pmc_flash.sh OUTDIR ; python3 tools/pmc_attn.py OUTDIR [json]
set -e
OUT=${1:-gpurun_out/pmcf}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
CMD=${PMC_CMD:-"python3 tools/flash_bench.py --iters 2 --default-only --batch ${PMC_B:-256}"}
pass() {  # name counters...
  local n=$1; shift
  timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d "$OUT/$n" -o "$n" --pmc "$@" -- $CMD \
    > "$OUT/$n.log" 2>&1
}
pass fetch FETCH_SIZE GRBM_GUI_ACTIVE
pass write WRITE_SIZE
pass lds SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAVES SQ_WAVE_CYCLES \
  SQ_BUSY_CYCLES
pass busy SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU \
  SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES GRBM_GUI_ACTIVE
pass occ SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM \
  SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES
echo pmc ok
