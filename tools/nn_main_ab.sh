# NN dgrad main-loop A/B (PZ_GEMM_MAIN=khalf | quad) on the micro-batch's NN shapes, interleaved twice;
# NN_SHAPES = "M N K;..." in tools/gemm_one.py's NN convention (reduction N, output K).
O=gpurun_out/nn_ab.log; : > $O
IFS=';' read -ra SPECS <<< "${NN_SHAPES:-70656 2048 16384;70656 16384 2048;65536 4304 1152;65536 1152 4304;70656 2048 2048}"
for rep in 1 2; do for mode in khalf quad; do
for spec in "${SPECS[@]}"; do
  set -- $spec; echo -n "$mode " >> $O
  PZ_GEMM_MAIN=$mode timeout -k 10 120 python3 -u tools/gemm_one.py --layout NN --M $1 --N $2 --K $3 --iters 10 >> $O 2>> gpurun_out/nn_err.log || exit 1
done; done; done
