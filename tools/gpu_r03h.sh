# r03h: C4 d1024 launch-chunk sweep (slot blocks sized for the 256 MB
# Infinity Cache), the GPU suite on the final tree, then the r03c-g
# crash-at-exit subset (last: an abort ends the call)
set -o pipefail
OUT=gpurun_out/r03h; mkdir -p $OUT; export TMPDIR=/tmp
i=0
for mb in 128 160 192 224 256 320; do
  a="MK_JIT_SLOT_BYTES=$((mb << 20)) python bench.py --config c4d1024 --steps 5 --warmup 1 --no-cpu-baseline"
  i=$((i+1)); echo "[r03h] $a"
  timeout -k 10 200 env $a > $OUT/bench$i.log 2>&1 || { echo "failed: $a"; tail -20 $OUT/bench$i.log; exit 1; }
  grep -h '^{' $OUT/bench$i.log | python3 tools/benchline.py "$a" || true
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
PYTHONFAULTHANDLER=1 timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py -m gpu -k "c4 or stack or slot or lds or sign or pipelin or heavy or countdown or c5" > $OUT/pytest_c4.log 2>&1
rc=$?; tail -4 $OUT/pytest_c4.log | cut -c1-200; echo "rc=$rc"; exit $rc
