#!/bin/bash
# One GPU-box pass: optional crash-at-exit probe, parity tests, smoke, then a
# bench line per argument set, every GPU step under its own time limit and
# chained so that the first failure ends the call.  Replaces the per-session
# gpu_r0*.sh scripts of rounds 2 and 3 (in git history).
#   bash tools/gpu_round.sh TAG [--probe] [--no-tests] [--smoke] [--all-configs] [-- "bench args" ...]
#   --probe        tools/probe/dyn_stack_probe.py under PyTorch, defaults (exit status must be 0)
#   --all-configs  every BASELINE config's bench line (C2 with the CPU baseline, C3, C4 d64/d256/d1024,
#                  C5, the sessions leg), before the argument sets given after --
set -o pipefail
TAG=${1:-run}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
TESTS=1; SMOKE=0; PROBE=0; ALL=0
while [ $# -gt 0 ] && [ "$1" != "--" ]; do
  case "$1" in
    --no-tests) TESTS=0 ;;
    --smoke) SMOKE=1 ;;
    --probe) PROBE=1 ;;
    --all-configs) ALL=1 ;;
    *) echo "unknown option $1"; exit 2 ;;
  esac
  shift
done
[ "$1" = "--" ] && shift
step() { local t=$1; shift; echo "[gpu_round] $(date +%T) $*"; timeout -k 10 "$t" "$@"; }
if [ $PROBE = 1 ]; then
  step 400 python -u tools/probe/dyn_stack_probe.py torch > "$OUT/probe.log" 2>&1
  rc=$?; echo "probe rc=$rc" | tee -a "$OUT/probe.log"; tail -2 "$OUT/probe.log"
  [ $rc = 0 ] || exit 1
fi
if [ $TESTS = 1 ]; then
  step 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
    > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
  tail -1 "$OUT/pytest_gpu.log"
fi
if [ $SMOKE = 1 ]; then
  step 120 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { cat "$OUT/smoke.log"; exit 1; }
  tail -1 "$OUT/smoke.log"
fi
SETS=()
if [ $ALL = 1 ]; then
  SETS+=("python bench.py --steps 20 --warmup 3 --cpu-seconds 10"
         "python bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline"
         "python bench.py --config c4 --steps 20 --warmup 3 --no-cpu-baseline"
         "python bench.py --config c4d256 --steps 10 --warmup 2 --no-cpu-baseline"
         "python bench.py --config c4d1024 --steps 5 --warmup 1 --no-cpu-baseline"
         "python bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline"
         "python bench.py --steps 5 --warmup 1 --no-cpu-baseline --sessions 1048576")
fi
SETS+=("$@")
i=0
for a in "${SETS[@]}"; do
  i=$((i+1))
  step 300 env $a > "$OUT/bench$i.log" 2>&1 || { echo "[gpu_round] failed: $a"; tail -20 "$OUT/bench$i.log"; exit 1; }
  grep -h '^{' "$OUT/bench$i.log" | python3 tools/benchline.py "$a" || true
done
echo "[gpu_round] done"
