#!/bin/bash
# HBM byte counters of the executor kernel: one rocprofv3 --pmc pass for
# FETCH_SIZE and one for WRITE_SIZE (they do not fit one pass on gfx950),
# kernel trace only.  bash tools/gpu_pmc_bytes.sh TAG "bench args"
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  echo "[pmc-bytes] $(date +%T) $c: $1"
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c --output-format csv -d "$OUT/$c" -o p -- python3 bench.py $1 > "$OUT/$c.log" 2>&1 || { echo "[pmc-bytes] failed $c"; tail -5 "$OUT/$c.log"; exit 1; }
done
echo "[pmc-bytes] done"
