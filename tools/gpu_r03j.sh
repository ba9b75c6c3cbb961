# r03j: every config's bench line with the committed PMC profiles, then the
# crash-at-exit probe split by tier: four concurrent pytest processes (one
# per mode of the dynamic-stack parity tests), all started together
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03j; mkdir -p $OUT
i=0
for a in "python bench.py --steps 20 --warmup 3 --cpu-seconds 10" "python bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline" \
         "python bench.py --config c4 --steps 20 --warmup 3 --no-cpu-baseline" "python bench.py --config c4d256 --steps 10 --warmup 2 --no-cpu-baseline" \
         "python bench.py --config c4d1024 --steps 5 --warmup 1 --no-cpu-baseline" "python bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline" ; do
  i=$((i+1)); echo "[r03j] $a"
  timeout -k 10 300 env $a > $OUT/bench$i.log 2>&1 || { echo "failed: $a"; tail -20 $OUT/bench$i.log; exit 1; }
  grep -h '^{' $OUT/bench$i.log | python3 tools/benchline.py "$a" || true
done
pids=""
for m in auto tile refill interp; do
  PYTHONFAULTHANDLER=1 timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py -m gpu -k "dynamic_stack_networks and $m" > $OUT/pytest_$m.log 2>&1 &
  pids="$pids $!"
done
rcs=""
for p in $pids; do wait $p; rcs="$rcs $?"; done
for m in auto tile refill interp; do echo "== $m"; tail -3 $OUT/pytest_$m.log | cut -c1-160; done
echo "rcs:$rcs"
