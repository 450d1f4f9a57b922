# operand-feed probe of the 8-phase GEMM: the default build against two -DPZ_FEED_TEST builds of pz_gemm.hip
# (1: every K-tile's operands re-read from the tile's first two K-tiles, L2-resident; 2: B operand DMA skipped after
# the first two K-tiles; 3: fragment LDS reads skipped after K-tile 0; 4: the barrier after each phase's MFMAs
# removed; 5: 3 + 4).  The variants compute wrong products -- timing only.  FEED_VARIANTS picks them
# (quad4: the round-5 four-phase main loop, -DPZ_GEMM_QUAD4, a correct build).
set -e
mkdir -p gpurun_out
O=gpurun_out/feed_ab.log
: > $O
for rep in 1 2; do
for v in ${FEED_VARIANTS:-base feed1 feed2}; do
  if [ $v = base ]; then L=; else L=libpz_$v.so; fi
  IFS=';' read -ra SPECS <<< "${FEED_SHAPES:-GEGLU 70656 32768 2048;NT 70656 2048 2048;TN 70656 2048 2048;NN 70656 2048 16384}"
  for spec in "${SPECS[@]}"; do
    set -- $spec
    echo -n "$v " >> $O
    PZ_LIB_PATH=$L timeout -k 10 120 python3 -u tools/gemm_one.py --layout $1 --M $2 --N $3 --K $4 --iters 10 >> $O 2>> gpurun_out/feed_err.log
  done
done
done
