#!/bin/bash
# r02d: K-lanes-per-thread machine kernel: its tests, then C5 across kernel variants.
set -o pipefail
OUT=gpurun_out/r02d; mkdir -p $OUT; export TMPDIR=/tmp
step() { local t=$1; shift; echo "[r02d] $(date +%T) $*"; timeout -k 10 "$t" "$@"; }
step 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "machine_shape or loop_phases or c5 or pipelined_pops" > $OUT/pytest_machine.log 2>&1; rc=$?
tail -3 $OUT/pytest_machine.log; [ $rc -le 1 ] || exit 1
for v in "MK_JIT_COMPACT=0" "MK_JIT_POOL=2" "MK_JIT_POOL=3" "MK_JIT_POOL=4" "MK_JIT_POOL=256"; do
  env $v timeout -k 10 300 python bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_c5_${v#MK_JIT_}.log 2>&1 || { echo "failed $v"; exit 1; }
  grep -h '^{' $OUT/bench_c5_${v#MK_JIT_}.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); print('$v', d['config']['executor'].split('shape=')[1][:20], round(d['value']/1e12,2), 'T', round(d['roofline']['launch_us'],1), 'us')"
done
exit $rc
