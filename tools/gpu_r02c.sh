#!/bin/bash
# r02c: the lane-pool (compaction) kernel of the machine shape: its tests
# first (short limit), then the whole suite, C5 pool vs pool-less, PMC
# passes for every workload, default bench with CPU baselines + HTTP leg.
set -o pipefail
OUT=gpurun_out/r02c; mkdir -p $OUT; export TMPDIR=/tmp
step() { local t=$1; shift; echo "[r02c] $(date +%T) $*"; timeout -k 10 "$t" "$@"; }
step 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "machine_shape or loop_phases or c5 or pipelined_pops" > $OUT/pytest_pool.log 2>&1; rc=$?
tail -3 $OUT/pytest_pool.log; [ $rc -le 1 ] || exit 1
step 300 python bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_c5_pool.log 2>&1 || exit 1
MK_JIT_COMPACT=0 step 300 python bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_c5_nopool.log 2>&1 || exit 1
for m in 128 192; do MK_JIT_POOL=$m step 300 python bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_c5_pool$m.log 2>&1 || exit 1; done
grep -h '^{' $OUT/bench_c5_*.log | python3 -c "
import json,sys
for l in sys.stdin: d=json.loads(l); print(d['config']['executor'][-60:], round(d['value']/1e12,2), 'T', round(d['roofline']['launch_us'],1), 'us')"
[ $rc -eq 0 ] || exit 1
step 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -3 $OUT/pytest_gpu.log; [ $rc -le 1 ] || exit 1
step 1200 bash tools/gpu_pmc_all.sh r02c/pmc c2 c3 c4 c4d256 c4d1024 c5 > $OUT/pmc.log 2>&1 || { tail -20 $OUT/pmc.log; exit 1; }
step 300 python bench.py --steps 20 --warmup 3 --cpu-seconds 10 --http 64 > $OUT/bench_c2.log 2>&1 || { tail -20 $OUT/bench_c2.log; exit 1; }
grep -h '^{' $OUT/bench_c2.log | cut -c1-300
echo "[r02c] done"
