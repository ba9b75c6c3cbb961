#!/bin/bash
# r02i: dynamic stacks (data-dependent depths on tiers 2 and 3): the new GPU
# tests first, then the whole suite, then the census-class and config benches.
set -o pipefail
OUT=gpurun_out/r02i; mkdir -p $OUT; export TMPDIR=/tmp
step() { local t=$1; shift; echo "[r02i] $(date +%T) $*"; timeout -k 10 "$t" "$@"; }
step 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "dynamic or configs_bit_exact or machine_shape or loop_phases" > $OUT/pytest_first.log 2>&1; rc=$?
tail -c 2500 $OUT/pytest_first.log; [ $rc -eq 0 ] || exit 1
step 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -c 1500 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit 1
for c in t2_dyn_depth t1_two_stacks c5 c2 c4; do
  step 300 python bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline > $OUT/bench_$c.log 2>&1 \
    || { tail -20 $OUT/bench_$c.log; exit 1; }
  grep -h '^{' $OUT/bench_$c.log | python3 tools/benchline.py $c
done
for c in t2_dyn_depth t1_two_stacks; do
  MK_JIT=0 step 300 python bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline > $OUT/bench_${c}_tier2.log 2>&1 \
    || { tail -20 $OUT/bench_${c}_tier2.log; exit 1; }
  grep -h '^{' $OUT/bench_${c}_tier2.log | python3 tools/benchline.py ${c}_tier2
done
