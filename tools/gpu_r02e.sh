#!/bin/bash
# r02e: new GPU tests (lane trace, interleaved streams), then tier-1/tier-2
# rates: census classes and C2/C5 forced onto tiers 1 and 2.
set -o pipefail
OUT=gpurun_out/r02e; mkdir -p $OUT; export TMPDIR=/tmp
step() { local t=$1; shift; echo "[r02e] $(date +%T) $*"; timeout -k 10 "$t" "$@"; }
step 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "lane_trace or interleaved" > $OUT/pytest_new.log 2>&1; rc=$?
tail -3 $OUT/pytest_new.log; [ $rc -le 1 ] || exit 1
b() { local tag=$1; shift; step 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline "$@" > $OUT/bench_$tag.log 2>&1 || { tail -5 $OUT/bench_$tag.log; return 1; }
  grep -h '^{' $OUT/bench_$tag.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); r=d['roofline']; print('$tag', d['config']['executor'][:40], round(d['value']/1e12,4), 'T', round(r['launch_us'],1), 'us', r['bound'], round(r['frac'],4))"; }
b t2_dyn --config t2_dyn_depth && b t1_two --config t1_two_stacks && b c2_interp --config c2 --mode interp && \
b c2_tile --config c2 --mode tile && b c5_interp --config c5 --mode interp && b c5_tile --config c5 --mode tile && \
b c4_tile --config c4 --mode tile && b c4_interp --config c4 --mode interp
step 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_t1 -o t1 -- python3 bench.py --config t1_two_stacks --steps 5 --warmup 1 --no-cpu-baseline > $OUT/prof_t1.log 2>&1
exit 0
