# r03n: native library (this ROCm's runtime + hiprtc) loaded before PyTorch --
# the crash-at-exit subsets first (concurrent, started together), then the
# full GPU suite, smoke and the C2 / C4 / C5 bench lines
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03n; mkdir -p $OUT
run() { local tag=$1; PYTHONFAULTHANDLER=1 timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py -m gpu -k "$K" > $OUT/pytest_$tag.log 2>&1; echo "$tag rc=$?" >> $OUT/rcs.txt; }
K="dynamic_stack_networks and auto" run dyn_auto &
K="c4 or stack or slot or lds or sign or pipelin or heavy or countdown or c5" run c4subset &
ARG=torch PYTHONFAULTHANDLER=1 timeout -k 10 400 python -u tools/probe/dyn_stack_probe.py torch > $OUT/probe_torch.log 2>&1; echo "probe_torch_after rc=$?" >> $OUT/rcs.txt &
wait
cat $OUT/rcs.txt
for t in dyn_auto c4subset; do echo "== $t"; tail -2 $OUT/pytest_$t.log | cut -c1-160; done
tail -2 $OUT/probe_torch.log
if grep -qv "rc=0" $OUT/rcs.txt; then echo "a probe failed"; exit 1; fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
i=0
for a in "python bench.py --steps 20 --warmup 3 --cpu-seconds 10" "python bench.py --config c4 --steps 20 --warmup 3 --no-cpu-baseline" \
         "python bench.py --config c4d256 --steps 10 --warmup 2 --no-cpu-baseline" "python bench.py --config c4d1024 --steps 5 --warmup 1 --no-cpu-baseline" \
         "python bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline" "python bench.py --steps 5 --warmup 1 --no-cpu-baseline --sessions 1048576"; do
  i=$((i+1)); echo "[r03n] $a"
  timeout -k 10 300 env $a > $OUT/bench$i.log 2>&1 || { echo "failed: $a"; tail -20 $OUT/bench$i.log; exit 1; }
  grep -h '^{' $OUT/bench$i.log | python3 tools/benchline.py "$a" || true
done
echo done
