#!/bin/bash
# r02a: GPU suite after the budget-exit lookup + bounded compile, then the C4 configs.
set -o pipefail
OUT=gpurun_out/r02a; mkdir -p $OUT; export TMPDIR=/tmp
step() { local t=$1; shift; echo "[r02a] $(date +%T) $*"; timeout -k 10 "$t" "$@"; }
step 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
step 300 python bench.py --config c4 --steps 5 --warmup 1 --no-cpu-baseline > $OUT/bench_c4.log 2>&1 &&
step 300 python bench.py --config c4d1024 --steps 5 --warmup 1 --no-cpu-baseline > $OUT/bench_c4d1024.log 2>&1 &&
MK_JIT_SHAPE=machine step 300 python bench.py --config c4d256 --steps 5 --warmup 1 --no-cpu-baseline > $OUT/bench_c4d256_machine.log 2>&1 &&
step 300 python bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_c5.log 2>&1 &&
step 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench_c2.log 2>&1
rc=$?; grep -h '^{' $OUT/bench_*.log | cut -c1-400; exit $rc
