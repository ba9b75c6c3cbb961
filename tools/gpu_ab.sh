#!/bin/bash
# One GPU-box pass for an experiment: optional GPU tests (a -k selection),
# then bench lines for labelled argument sets, each under its own time limit;
# the first failure ends the call.
#   bash tools/gpu_ab.sh TAG [-k "pytest -k expr"] -- "label: ENV=.. --config c5 ..." ...
# A set is "label: [VAR=value ...] bench args"; every bench runs with
# --steps 10 --warmup 2 --no-cpu-baseline unless the set overrides them.
# Results: gpurun_out/TAG/{pytest.log,bench_<label>.log} and one summary line
# per set (tools/benchline.py).  Replaces the per-run gpu_r02*.sh scripts of
# round 2 (in git history).
set -o pipefail
TAG=${1:-ab}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { local t=$1; shift; echo "[gpu_ab] $(date +%T) $*"; timeout -k 10 "$t" "$@"; }
if [ "$1" = "-k" ]; then
  step 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$2" \
    > "$OUT/pytest.log" 2>&1 || { tail -c 3000 "$OUT/pytest.log"; exit 1; }
  tail -2 "$OUT/pytest.log"
  shift 2
fi
[ "$1" = "--" ] && shift
for set in "$@"; do
  label=${set%%:*}
  rest=${set#*:}
  envs=(); args=()
  for w in $rest; do
    if [[ "$w" == *=* && ${#args[@]} -eq 0 ]]; then envs+=("$w"); else args+=("$w"); fi
  done
  step 300 env "${envs[@]}" python bench.py --steps 10 --warmup 2 --no-cpu-baseline "${args[@]}" \
    > "$OUT/bench_$label.log" 2>&1 || { echo "[gpu_ab] failed: $set"; tail -20 "$OUT/bench_$label.log"; exit 1; }
  grep -h '^{' "$OUT/bench_$label.log" | python3 tools/benchline.py "$label" || true
done
echo "[gpu_ab] done"
