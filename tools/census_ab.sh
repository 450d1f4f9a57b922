# same-box A/B of the micro-batch GEMM census (tools/gemm_census.py): the default build against the in-tree
# alternate build named by CENSUS_ALT (e.g. libpz_nnk.so), interleaved twice; the per-class lines of each run.
set -e
mkdir -p gpurun_out
O=gpurun_out/census_ab.log
: > $O
for rep in 1 2; do
  for v in base alt; do
    if [ $v = base ]; then L=; else L=$CENSUS_ALT; fi
    echo "== $v" >> $O
    PZ_LIB_PATH=$L timeout -k 10 300 python3 -u tools/gemm_census.py --micro-batch ${CENSUS_MB:-256} >> $O 2>> gpurun_out/census_err.log
  done
done
