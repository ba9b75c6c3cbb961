#!/bin/bash
# r02h: restored-tree check after the container was re-created -- whole GPU
# suite, smoke(), the default bench line (with the CPU baselines), every
# config, and rocprofv3 kernel stats for C2 / C5 / C4 d1024.
set -o pipefail
OUT=gpurun_out/r02h; mkdir -p $OUT; export TMPDIR=/tmp
step() { local t=$1; shift; echo "[r02h] $(date +%T) $*"; timeout -k 10 "$t" "$@"; }
step 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 \
  || { tail -c 3000 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
step 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
step 400 python bench.py > $OUT/bench_default.log 2>&1 || { tail -20 $OUT/bench_default.log; exit 1; }
grep -h '^{' $OUT/bench_default.log | python3 tools/benchline.py default
for c in c3 c4 c4d256 c4d1024 c5 t2_dyn_depth t1_two_stacks; do
  step 300 python bench.py --config $c --steps 5 --warmup 1 --no-cpu-baseline > $OUT/bench_$c.log 2>&1 \
    || { tail -20 $OUT/bench_$c.log; exit 1; }
  grep -h '^{' $OUT/bench_$c.log | python3 tools/benchline.py $c
done
bash tools/gpu_profiles.sh r02h c2 c5 c4d1024
