#!/bin/bash
# Short GPU experiments: bench variants only.  bash tools/gpu_exp.sh tag "args1" "args2" ...
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p "$OUT"; export TMPDIR=/tmp
i=0
for a in "$@"; do
  i=$((i+1))
  echo "[gpu_exp] $a"
  timeout -k 10 300 python bench.py --no-cpu-baseline $a > "$OUT/bench_exp$i.log" 2>&1 || { echo "[gpu_exp] failed: $a"; exit 1; }
done
