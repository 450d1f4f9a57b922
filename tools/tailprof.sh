set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/tailprof; mkdir -p $O
for cfg in "GEGLU 17664 32768 2048" "NT 17664 2048 2048" "NN 17664 2048 32768"; do
  set -- $cfg
  for t in "" "--notail"; do
    timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$1$t -o k -- python3 tools/gemm_one.py --layout $1 --M $2 --N $3 --K $4 --iters 10 $t >> $O/log.txt 2>&1
  done
done
