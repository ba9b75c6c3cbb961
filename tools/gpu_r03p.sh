# r03p: A/B -- C4 d256 with fewer LDS slots per wave and more waves per CU
# (the rest of the 193 slots in the wave's HBM block), C5 tile knobs
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03p; mkdir -p $OUT
i=0
for a in "python bench.py --config c4d256 --steps 10 --warmup 2 --no-cpu-baseline" \
         "MK_JIT_LDS_SLOTS=32768 MK_JIT_LDS_SPLIT=50 python bench.py --config c4d256 --steps 10 --warmup 2 --no-cpu-baseline" \
         "MK_JIT_LDS_SLOTS=26624 MK_JIT_LDS_SPLIT=50 python bench.py --config c4d256 --steps 10 --warmup 2 --no-cpu-baseline" \
         "MK_JIT_LDS_SLOTS=20480 MK_JIT_LDS_SPLIT=40 python bench.py --config c4d256 --steps 10 --warmup 2 --no-cpu-baseline" \
         "MK_JIT_LDS_SLOTS=0 python bench.py --config c4d256 --steps 10 --warmup 2 --no-cpu-baseline" \
         "python bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline" \
         "MK_JIT_TS_ROUNDS=8 python bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline" \
         "MK_JIT_TS_DYN=1 python bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline" \
         "MK_JIT_TS_DYN=1 MK_JIT_TS_ROUNDS=8 python bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline" ; do
  i=$((i+1)); echo "[r03p] $a"
  timeout -k 10 300 env $a > $OUT/bench$i.log 2>&1 || { echo "failed: $a"; tail -20 $OUT/bench$i.log; exit 1; }
  grep -h '^{' $OUT/bench$i.log | python3 tools/benchline.py "$a" || true
done
echo done
