#!/bin/bash
# Bench lines for a set of argument strings (each its own time limit), one
# JSON line each into gpurun_out/TAG/lines.jsonl, summarised with
# tools/benchline.py.   bash tools/probe/bench_set.sh TAG "bench args" ...
set -o pipefail
OUT=gpurun_out/$1; shift; mkdir -p $OUT; export TMPDIR=/tmp
i=0
for a in "$@"; do
  i=$((i+1))
  echo "[bench_set] $(date +%T) $a"
  timeout -k 10 300 python bench.py $a > $OUT/b$i.log 2>&1 || { echo "[bench_set] failed: $a"; tail -20 $OUT/b$i.log; exit 1; }
  grep -h '^{' $OUT/b$i.log | tee -a $OUT/lines.jsonl | python3 tools/benchline.py "$a" || true
done
