# r03g: C4 slot-placement A/B (d256: all slots in LDS at three waves vs the
# split at four; d1024: launch chunks small enough for the slot blocks to
# stay in the Infinity Cache, LDS split) and the PMC byte calibration probe
set -o pipefail
OUT=gpurun_out/r03g; mkdir -p $OUT; export TMPDIR=/tmp
i=0
for a in "python bench.py --config c4d256 --steps 10 --warmup 2 --no-cpu-baseline" \
         "MK_JIT_LDS_SLOTS=51200 python bench.py --config c4d256 --steps 10 --warmup 2 --no-cpu-baseline" \
         "MK_JIT_LDS_SLOTS=40960 MK_JIT_LDS_SPLIT=50 python bench.py --config c4d256 --steps 10 --warmup 2 --no-cpu-baseline" \
         "python bench.py --config c4d1024 --steps 5 --warmup 1 --no-cpu-baseline" \
         "MK_JIT_SLOT_BYTES=201326592 python bench.py --config c4d1024 --steps 5 --warmup 1 --no-cpu-baseline" \
         "MK_JIT_SLOT_BYTES=100663296 python bench.py --config c4d1024 --steps 5 --warmup 1 --no-cpu-baseline" \
         "MK_JIT_SLOT_BYTES=50331648 python bench.py --config c4d1024 --steps 5 --warmup 1 --no-cpu-baseline" \
         "MK_JIT_LDS_SPLIT=25 python bench.py --config c4d1024 --steps 5 --warmup 1 --no-cpu-baseline" ; do
  i=$((i+1)); echo "[r03g] $a"
  timeout -k 10 200 env $a > $OUT/bench$i.log 2>&1 || { echo "failed: $a"; tail -20 $OUT/bench$i.log; exit 1; }
  grep -h '^{' $OUT/bench$i.log | python3 tools/benchline.py "$a" || true
done
bash tools/gpu_pmc_calib.sh r03g_calib 4096 || exit 1
# the r03c-f crash at exit: glibc checks on every free (no tcache), freed
# memory perturbed, verbose test names, so the corruption surfaces in the test
# that causes it (last step: an abort ends the call)
GLIBC_TUNABLES=glibc.malloc.tcache_count=0:glibc.malloc.perturb=165 PYTHONFAULTHANDLER=1 timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py -m gpu -k "c4 or stack or slot or lds or sign or pipelin or heavy or countdown or c5" > $OUT/pytest_c4.log 2>&1
rc=$?; tail -40 $OUT/pytest_c4.log | cut -c1-200; echo "rc=$rc"; exit $rc
