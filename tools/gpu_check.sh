#!/bin/bash
# GPU-box check run: parity tests, bench (both tiers) and a rocprofv3 kernel
# trace.  Every GPU step has its own time limit; the chain stops at the first
# failure.  Usage (from the repo root): bash tools/gpu_check.sh [tag]
set -o pipefail
TAG=${1:-run}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { local t=$1; shift; echo "[gpu_check] $(date +%T) $*" ; timeout -k 10 "$t" "$@"; }
step 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 &&
step 300 python bench.py --steps 20 --warmup 3 --cpu-seconds 10 > "$OUT/bench_c2.log" 2>&1 &&
step 300 python bench.py --steps 5 --warmup 1 --interp --no-cpu-baseline > "$OUT/bench_c2_interp.log" 2>&1 &&
step 300 python bench.py --config c3 --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/bench_c3.log" 2>&1 &&
step 300 python bench.py --config c5 --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/bench_c5.log" 2>&1 &&
step 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c2" -o c2 -- python bench.py --steps 20 --warmup 3 --no-cpu-baseline > "$OUT/prof_c2.log" 2>&1
rc=$?
echo "[gpu_check] done rc=$rc"
exit $rc
