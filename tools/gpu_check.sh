#!/bin/bash
# One GPU-box pass: parity tests, default bench line, rocprofv3 kernel stats of the bench.
# usage (gpurun, from the repo root): bash tools/gpu_check.sh TAG [tests|bench|prof ...]
# Every GPU step has its own time limit; the first failing step ends the script.
set -e
TAG=${1:-run}; shift || true
STEPS=${*:-tests bench prof}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for s in $STEPS; do
  case $s in
    tests)
      timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 300 --timeout-method thread \
        > "$OUT/tests.log" 2>&1 ;;
    bench)
      timeout -k 10 600 python -u bench.py > "$OUT/bench.log" 2>&1 ;;
    prof)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o bench \
        -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > "$OUT/prof.log" 2>&1
      # the full trace (~100 MB) exceeds what gpurun copies back; keep the per-dispatch rows of the
      # dominant GEMM only (grid split / duration check) and the stats summary
      python3 - "$OUT/prof" <<'PY'
import csv, glob, os, sys
import subprocess
for f in glob.glob(os.path.join(sys.argv[1], "*kernel_trace.csv")):
    with open(f.replace("kernel_trace.csv", "gaps.txt"), "w") as g:
        subprocess.run([sys.executable, "tools/trace_gaps.py", f, "--after-ms", os.environ.get("GAPS_AFTER_MS", "0")],
                       stdout=g, stderr=subprocess.STDOUT)
    with open(f) as fi, open(f.replace("kernel_trace", "dominant_trace"), "w", newline="") as fo:
        r = csv.DictReader(fi)
        w = csv.DictWriter(fo, fieldnames=r.fieldnames)
        w.writeheader()
        for row in r:
            if "gemm8p_kernel<true, true, true, false>" in row.get("Kernel_Name", ""):
                w.writerow(row)
    os.remove(f)
PY
      ;;
    infprof)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/infprof" -o infer \
        -- python3 tools/infer_bench.py --iters 20 > "$OUT/infprof.log" 2>&1 ;;
    c5prof)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c5prof" -o c5 \
        -- python3 tools/c5_bench.py --iters 20 > "$OUT/c5prof.log" 2>&1 ;;
    ddpab)  # same box, same build: plain vs the forced world-1 DDP path (RCCL bucket all-reduce on the comm stream)
      timeout -k 10 400 python -u bench.py --steps ${AB_STEPS:-5} --warmup 1 --no-infer --no-cpu-baseline \
        > "$OUT/ab_plain.log" 2>&1
      timeout -k 10 400 python -u bench.py --steps ${AB_STEPS:-5} --warmup 1 --no-infer --no-cpu-baseline --force-ddp \
        > "$OUT/ab_ddp.log" 2>&1
      timeout -k 10 400 python -u bench.py --steps ${AB_STEPS:-5} --warmup 1 --no-infer --no-cpu-baseline \
        > "$OUT/ab_plain2.log" 2>&1 ;;
    ddpprof)  # kernel trace of the forced-DDP step (compare with prof's plain-step stats)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/ddpprof" -o ddp \
        -- python3 bench.py --steps 1 --warmup 1 --no-infer --no-cpu-baseline --force-ddp > "$OUT/ddpprof.log" 2>&1
      for f in "$OUT"/ddpprof/*kernel_trace.csv "$OUT"/ddpprof/*/*kernel_trace.csv; do
        if [ -f "$f" ]; then python3 tools/trace_gaps.py "$f" > "${f%kernel_trace.csv}gaps.txt" 2>&1; rm -f "$f"; fi
      done ;;
    mbab)  # the default micro-batch (256 x 4) against 128 x 8, same box
      timeout -k 10 500 python -u bench.py --steps ${AB_STEPS:-3} --warmup 1 --no-infer --no-cpu-baseline \
        > "$OUT/ab_mb256.log" 2>&1
      timeout -k 10 500 python -u bench.py --steps ${AB_STEPS:-3} --warmup 1 --no-infer --no-cpu-baseline \
        --micro-batch 128 > "$OUT/ab_mb128.log" 2>&1 ;;
    knobab)  # engine knobs at the default micro-batch, same box: one bench line each (--no-infer)
      for kv in ${KNOBS:-base PZ_SPLIT_DGEGLU=1 PZ_SPLIT_DACT=0 PZ_EXPERT_STREAM=0 PZ_JOINT_ATTN=gemm base}; do
        if [ "$kv" = base ]; then envs=(); else envs=("$kv"); fi
        env "${envs[@]}" timeout -k 10 400 python -u bench.py --steps 3 --warmup 1 --no-infer --no-cpu-baseline \
          > "$OUT/knob.tmp" 2>&1
        echo "$kv $(grep -o '"value": [0-9.]*' "$OUT/knob.tmp")" >> "$OUT/knobab.log"
      done
      rm -f "$OUT/knob.tmp" ;;
    trainprof)  # kernel stats of the training step alone (1 warm-up + 1 timed step, no inference legs)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trainprof" -o train \
        -- python3 bench.py --steps 1 --warmup 1 --no-infer --no-cpu-baseline > "$OUT/trainprof.log" 2>&1
      rm -f "$OUT"/trainprof/*kernel_trace.csv "$OUT"/trainprof/*/*kernel_trace.csv ;;
    tallbench)
      timeout -k 10 300 python -u tools/tall_bench.py > "$OUT/tall_bench.log" 2>&1 ;;
    ldpad)  # SigLIP 4304-wide operands: natural 8608-B row pitch vs padded to 4352 elements
      timeout -k 10 300 python -u tools/ld_pad_ab.py > "$OUT/ld_pad_ab.log" 2>&1 ;;
    gaps)  # GPU idle time inside the training step (plain run, no inference legs): the last ~2 steps' kernels
      timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d "$OUT/gaps" -o gaps \
        -- python3 bench.py --steps 2 --warmup 1 --no-infer --no-cpu-baseline > "$OUT/gaps.log" 2>&1
      for f in "$OUT"/gaps/*kernel_trace.csv "$OUT"/gaps/*/*kernel_trace.csv; do
        if [ -f "$f" ]; then python3 tools/trace_gaps.py "$f" --last-ms ${GAPS_LAST_MS:-8000} --top 40 \
          > "$OUT/gaps.txt" 2>&1; rm -f "$f"; fi
      done ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 ;;
    flashbench)
      timeout -k 10 300 python -u tools/flash_bench.py > "$OUT/flash_bench.log" 2>&1 ;;
    gemmbench)
      timeout -k 10 400 python -u tools/gemm_bench.py --iters 10 > "$OUT/gemm_bench.log" 2>&1 ;;
    pmc)
      bash tools/pmc_dominant.sh "$OUT/pmc" ;;
    pmcdgeglu)  # the same counter passes on the DGEGLU dgrad (down-proj dgrad + GeGLU derivative, micro-batch 256)
      PMC_CMD="python3 tools/gemm_one.py --layout DGEGLU --M 70656 --N 2048 --K 16384 --iters 3" \
        bash tools/pmc_dominant.sh "$OUT/pmcd" ;;
    flashprof)  # per-kernel times of the attention microbenchmark (every variant)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/flashprof" -o flash \
        -- python3 tools/flash_bench.py --iters 5 > "$OUT/flashprof.log" 2>&1
      rm -f "$OUT"/flashprof/*kernel_trace.csv "$OUT"/flashprof/*/*kernel_trace.csv ;;
    pmcattn)  # counter passes of the training-default attention kernels at micro-batch 256
      bash tools/pmc_flash.sh "$OUT/pmca" && python3 tools/pmc_attn.py "$OUT/pmca" "$OUT/pmc_attn.json" \
        > "$OUT/pmc_attn.txt" 2>&1
      rm -f "$OUT"/pmca/*/*kernel_trace.csv ;;
    launcher)  # bench.py --gpus 2 rehearsal: 2 gloo ranks on this card
      timeout -k 10 900 python -u -m pytest tests/test_bench_launcher.py -m gpu -x -v --timeout 880 \
        --timeout-method thread > "$OUT/launcher.log" 2>&1 ;;
    normbench)  # memory-bound backward kernels (norms, GELU backward + column sums) under their A/B knobs
      timeout -k 10 300 python -u tools/norm_bench.py > "$OUT/norm_bench.log" 2>&1 ;;
    attngemm)  # planner A/B on the joint attention's batched dK / dV and the action expert's 1280-row GEMMs
      timeout -k 10 300 python -u tools/attn_gemm_ab.py > "$OUT/attn_gemm_ab.log" 2>&1 ;;
    infab)  # inference knobs on the C4 / C5 graphs, interleaved (KNOBS: "base" = defaults, or VAR=value each)
      for kv in ${KNOBS:-base base}; do
        if [ "$kv" = base ]; then envs=(); else envs=("$kv"); fi
        env "${envs[@]}" timeout -k 10 300 python -u tools/infer_bench.py --iters 50 > "$OUT/ab.tmp" 2>&1
        echo "$kv C4 $(grep -o 'graph [0-9.]* ms' "$OUT/ab.tmp")" >> "$OUT/infab.log"
        env "${envs[@]}" timeout -k 10 300 python -u tools/c5_bench.py --iters 20 > "$OUT/ab.tmp" 2>&1
        echo "$kv C5 $(grep -o '"graph_ms": [0-9.]*\|"fp8_graph_ms": [0-9.]*' "$OUT/ab.tmp" | tr '\n' ' ')" >> "$OUT/infab.log"
      done
      rm -f "$OUT/ab.tmp" ;;
    optbench)  # the 8-bit AdamW step over a Pi0-sized arena
      timeout -k 10 300 python -u tools/optim_bench.py > "$OUT/optim_bench.log" 2>&1 ;;
    optprof)  # kernel times of the 8-bit AdamW step (this build, and the build in ab_old/ when present)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/optprof" -o opt \
        -- python3 tools/optim_bench.py > "$OUT/optprof.log" 2>&1
      if [ -f ab_old/libpizero_hip.so ]; then
        PZ_LIB_PATH=$PWD/ab_old/libpizero_hip.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
          -d "$OUT/optprof_old" -o opt -- python3 tools/optim_bench.py > "$OUT/optprof_old.log" 2>&1
      fi
      rm -f "$OUT"/optprof*/*kernel_trace.csv "$OUT"/optprof*/*/*kernel_trace.csv ;;
    census)
      timeout -k 10 300 python -u tools/gemm_census.py --micro-batch ${CENSUS_MB:-256} > "$OUT/gemm_census.log" 2>&1 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
  echo "step $s ok"
done
