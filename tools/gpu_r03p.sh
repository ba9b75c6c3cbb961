# r03p: A/B -- C5's countdown loops as one saturating decrement per iteration
# (MK_JIT_SAT_DEC 1 = asm, 2 = plain usub.sat, 0 = sub + min_u32), the loop
# parity subset under mode 2; C4 d256 with fewer LDS slots per wave
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03p; mkdir -p $OUT
MK_JIT_SAT_DEC=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "c5 or loop or dynamic_stack or random" > $OUT/pytest_satdec2.log 2>&1 || { tail -30 $OUT/pytest_satdec2.log; exit 1; }
tail -1 $OUT/pytest_satdec2.log
i=0
for a in "python bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline" \
         "MK_JIT_SAT_DEC=0 python bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline" \
         "MK_JIT_SAT_DEC=2 python bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline" \
         "MK_JIT_SAT_DEC=2 MK_JIT_TS_DYN=1 python bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline" \
         "MK_JIT_SAT_DEC=2 MK_JIT_TS_ROUNDS=8 python bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline" \
         "MK_JIT_TS_DYN=1 python bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline" \
         "MK_JIT_LDS_SLOTS=32768 MK_JIT_LDS_SPLIT=50 python bench.py --config c4d256 --steps 10 --warmup 2 --no-cpu-baseline" \
         "MK_JIT_LDS_SLOTS=20480 MK_JIT_LDS_SPLIT=40 python bench.py --config c4d256 --steps 10 --warmup 2 --no-cpu-baseline" ; do
  i=$((i+1)); echo "[r03p] $a"
  timeout -k 10 300 env $a > $OUT/bench$i.log 2>&1 || { echo "failed: $a"; tail -20 $OUT/bench$i.log; exit 1; }
  grep -h '^{' $OUT/bench$i.log | python3 tools/benchline.py "$a" || true
done
echo done
