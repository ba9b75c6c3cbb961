#!/bin/bash
# One GPU-box pass: parity tests, then a bench per config (+ optional extra
# bench argument sets), every GPU step under its own time limit, chained so
# that the first failure ends the call.
#   bash tools/gpu_round.sh TAG [--no-tests] [-- "bench args" ...]
set -o pipefail
TAG=${1:-run}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
TESTS=1
if [ "$1" = "--no-tests" ]; then TESTS=0; shift; fi
[ "$1" = "--" ] && shift
step() { local t=$1; shift; echo "[gpu_round] $(date +%T) $*"; timeout -k 10 "$t" "$@"; }
if [ $TESTS = 1 ]; then
  step 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
  tail -2 "$OUT/pytest_gpu.log"
fi
i=0
for a in "$@"; do
  i=$((i+1))
  step 300 env $a > "$OUT/bench$i.log" 2>&1 || { echo "[gpu_round] failed: $a"; tail -20 "$OUT/bench$i.log"; exit 1; }
  grep -h '^{' "$OUT/bench$i.log" | python3 tools/benchline.py "$a" || true
done
echo "[gpu_round] done"
