#!/bin/bash
# r02f: new/changed paths first (mixed deployments, HTTP, sessions, the
# tier-1 rewrite, lane trace, host API chunks), then the whole GPU suite,
# then tier-1/2 rates.
set -o pipefail
OUT=gpurun_out/r02f; mkdir -p $OUT; export TMPDIR=/tmp
step() { local t=$1; shift; echo "[r02f] $(date +%T) $*"; timeout -k 10 "$t" "$@"; }
step 400 python -u -m pytest tests/test_mixed.py tests/test_master.py tests/test_gpu_parity.py -m gpu -x -q \
  --timeout 120 --timeout-method thread \
  -k "mixed or http or session or interp or trace or host_api or c5 or random_networks" > $OUT/pytest_first.log 2>&1; rc=$?
tail -c 2500 $OUT/pytest_first.log; [ $rc -le 1 ] || exit 1; [ $rc -eq 0 ] || exit 1
step 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -c 1500 $OUT/pytest_gpu.log; [ $rc -le 1 ] || exit 1
b() { local tag=$1; shift; step 300 python bench.py --steps 5 --warmup 1 --no-cpu-baseline "$@" > $OUT/bench_$tag.log 2>&1 || { tail -5 $OUT/bench_$tag.log; return 1; }
  grep -h '^{' $OUT/bench_$tag.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); r=d['roofline']; print('$tag', d['config']['executor'][:40], round(d['value']/1e12,4), 'T', round(r['launch_us'],1), 'us', r['bound'], round(r['frac'],4))"; }
b t1_two --config t1_two_stacks && b c2_interp --config c2 --mode interp && b c5_interp --config c5 --mode interp && \
b c4_interp --config c4 --mode interp && b t2_dyn_interp --config t2_dyn_depth --mode interp && \
b c2_host --config c2 --host-io
exit 0
