#!/bin/bash
# r02g: input ordering (machine shape), host API paths, tier-1 pick for
# exploded schedules; whole GPU suite; A/B of the machine-shape knobs.
set -o pipefail
OUT=gpurun_out/r02g; mkdir -p $OUT; export TMPDIR=/tmp
step() { local t=$1; shift; echo "[r02g] $(date +%T) $*"; timeout -k 10 "$t" "$@"; }
step 300 python -u -m pytest tests/test_gpu_parity.py tests/test_tier_census.py -m gpu -x -q \
  --timeout 120 --timeout-method thread -k "order or host_api or device_mask or census or machine" \
  > $OUT/pytest_first.log 2>&1; rc=$?
tail -c 2500 $OUT/pytest_first.log; [ $rc -eq 0 ] || exit 1
step 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -c 1500 $OUT/pytest_gpu.log; [ $rc -le 1 ] || exit 1
b() { local tag=$1; shift; step 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline "$@" > $OUT/bench_$tag.log 2>&1 || { tail -5 $OUT/bench_$tag.log; return 1; }
  grep -h '^{' $OUT/bench_$tag.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); r=d['roofline']; print('$tag', d['config']['executor'][:40], round(d['value']/1e12,4), 'T', round(r['launch_us'],1), 'us', r['bound'], round(r['frac'],4))"; }
b c5_order --config c5 && MK_JIT_ORDER=0 b c5_noorder --config c5 && \
b c4d256 --config c4d256 && MK_JIT_SHAPE=machine b c4d256_machine --config c4d256 && \
b c4d1024 --config c4d1024 && MK_JIT_SHAPE=machine b c4d1024_machine --config c4d1024 && \
b t2_dyn --config t2_dyn_depth && b t1_two --config t1_two_stacks && b c2 --config c2 && b c3 --config c3 && b c4 --config c4
exit 0
