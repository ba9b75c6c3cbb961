#!/bin/bash
# rocprofv3 kernel-trace summaries for a list of bench configs, one run each,
# every run under its own time limit; the chain stops at the first failure.
#   bash tools/gpu_profiles.sh TAG CONFIG [CONFIG ...]
# Writes gpurun_out/TAG/prof_<config>/ (kernel_stats.csv etc.) and
# gpurun_out/TAG/bench_<config>.json (the bench line of the profiled run).
set -o pipefail
TAG=${1:-prof}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for c in "$@"; do
  echo "[gpu_profiles] $(date +%T) $c"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_$c" -o "$c" \
    -- python bench.py --config "$c" --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/prof_$c.log" 2>&1 \
    || { echo "[gpu_profiles] failed: $c"; tail -20 "$OUT/prof_$c.log"; exit 1; }
  grep -h '^{' "$OUT/prof_$c.log" > "$OUT/bench_$c.json" || true
  python3 tools/benchline.py "$c" < "$OUT/bench_$c.json" || true
done
echo "[gpu_profiles] done"
