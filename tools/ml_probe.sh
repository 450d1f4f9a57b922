set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ml; mkdir -p $O
for L in NT NN TN; do for V in quad khalf; do for K in 16384 2048; do
  PZ_GEMM_MAIN=$V timeout -k 10 60 python3 tools/gemm_one.py --layout $L --M 4096 --N 4096 --K $K --iters 10 | sed "s/^/$V /" >> $O/ml.log
done; done; done
for V in quad khalf; do
  PZ_GEMM_MAIN=$V timeout -s KILL 60 rocprofv3 --kernel-trace --output-format csv -d $O/pmc_$V -o p --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS GRBM_GUI_ACTIVE -- python3 tools/gemm_one.py --layout NT --M 4096 --N 4096 --K 16384 --iters 3 > $O/pmc_$V.log 2>&1
done
echo done
