#!/bin/bash
# r02m: in-line side exits (BRX) for dynamic POP checks: tests, A/B.
set -o pipefail
OUT=gpurun_out/r02m; mkdir -p $OUT; export TMPDIR=/tmp
step() { local t=$1; shift; echo "[r02m] $(date +%T) $*"; timeout -k 10 "$t" "$@"; }
step 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "input_order or dynamic or machine_shape or loop_phases or random_networks" > $OUT/pytest_first.log 2>&1; rc=$?
tail -c 1500 $OUT/pytest_first.log; [ $rc -eq 0 ] || exit 1
b() { local tag=$1; shift; step 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline "$@" > $OUT/bench_$tag.log 2>&1 || { tail -5 $OUT/bench_$tag.log; return 1; }
  grep -h '^{' $OUT/bench_$tag.log | python3 tools/benchline.py $tag; }
for c in t2_dyn_depth t1_two_stacks; do
  b ${c}_brx --config $c && MK_SCHED_SIDE_EXITS=0 b ${c}_br --config $c || exit 1
done
b c5 --config c5
