# r03s: final tree after the prelude change (saturating helpers only where
# used): full GPU suite, smoke, C2 / C4 d64 / C5 bench lines (the committed
# PMC profiles must match their modules again: roofline_issue present)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03s; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
i=0
for a in "python bench.py" "python bench.py --config c4 --steps 20 --warmup 3 --no-cpu-baseline" "python bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline"; do
  i=$((i+1)); echo "[r03s] $a"
  timeout -k 10 300 env $a > $OUT/bench$i.log 2>&1 || { echo "failed: $a"; tail -20 $OUT/bench$i.log; exit 1; }
  grep -h '^{' $OUT/bench$i.log | python3 tools/benchline.py "$a" || true
done
echo done
