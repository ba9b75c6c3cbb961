# r03l: code object v5 modules -- the crash-at-exit probe (native tier,
# dynamic-stack parity tests; four variants concurrently), then smoke and
# C2/C4/C5 bench lines (the modules' register allocation is unchanged: the
# version is the container format)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03l; mkdir -p $OUT
run() { local tag=$1; shift; env "$@" PYTHONFAULTHANDLER=1 timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py -m gpu -k "$K" > $OUT/pytest_$tag.log 2>&1; echo "$tag rc=$?" >> $OUT/rcs.txt; }
K="dynamic_stack_networks and auto" run dyn_auto MK_NONE=1 &
K="c4 or stack or slot or lds or sign or pipelin or heavy or countdown or c5" run c4subset MK_NONE=1 &
K="dynamic_stack_networks and auto" run dyn_notsort MK_JIT_TILE_SORT=0 &
wait
cat $OUT/rcs.txt
for t in dyn_auto c4subset dyn_notsort; do echo "== $t"; tail -2 $OUT/pytest_$t.log | cut -c1-160; done
grep -q "rc=0" $OUT/rcs.txt && ! grep -qv "rc=0" $OUT/rcs.txt || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
i=0
for a in "python bench.py --steps 20 --warmup 3 --no-cpu-baseline" "python bench.py --config c4 --steps 20 --warmup 3 --no-cpu-baseline" \
         "python bench.py --config c4d256 --steps 10 --warmup 2 --no-cpu-baseline" "python bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline"; do
  i=$((i+1)); echo "[r03l] $a"
  timeout -k 10 300 env $a > $OUT/bench$i.log 2>&1 || { echo "failed: $a"; tail -20 $OUT/bench$i.log; exit 1; }
  grep -h '^{' $OUT/bench$i.log | python3 tools/benchline.py "$a" || true
done
echo done
