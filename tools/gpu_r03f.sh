# r03f: benches (C client, quad / flag-min / narrow A/B, sessions burst), then
# the subset whose pytest process crashed at exit in r03c-e (last: an abort ends the call)
set -o pipefail
OUT=gpurun_out/r03f; mkdir -p $OUT; export TMPDIR=/tmp; export PYTHONFAULTHANDLER=1
gcc -std=c99 -O2 -D__HIP_PLATFORM_AMD__ -I include -I /opt/rocm/include integration/c/mk_bench.c -L misaka-net_amd/lib -lmisaka_amd -L /opt/rocm/lib -lamdhip64 -Wl,-rpath,$PWD/misaka-net_amd/lib -Wl,-rpath,/opt/rocm/lib -o /tmp/mk_bench
for a in "c2 20 3" "c4:64 20 3" "c4:256 10 2"; do timeout -k 10 120 /tmp/mk_bench $a | tee -a $OUT/cbench.jsonl || exit 1; done
i=0
for a in "MK_JIT_LDS_QUAD=1 python bench.py --config c4 --steps 20 --warmup 3 --no-cpu-baseline" \
         "MK_JIT_LDS_QUAD=0 python bench.py --config c4 --steps 20 --warmup 3 --no-cpu-baseline" \
         "MK_JIT_LDS_QUAD=1 python bench.py --config c4d256 --steps 10 --warmup 2 --no-cpu-baseline" \
         "MK_JIT_LDS_QUAD=0 python bench.py --config c4d256 --steps 10 --warmup 2 --no-cpu-baseline" \
         "MK_JIT_FLAG_MIN=1 python bench.py --config c5 --steps 5 --warmup 1 --no-cpu-baseline" \
         "MK_JIT_FLAG_MIN=0 python bench.py --config c5 --steps 5 --warmup 1 --no-cpu-baseline" \
         "MK_JIT_NARROW=0 python bench.py --config c5 --steps 5 --warmup 1 --no-cpu-baseline" \
         "MK_JIT_NARROW=0 python bench.py --config c4 --steps 20 --warmup 3 --no-cpu-baseline" \
         "python bench.py --steps 5 --warmup 1 --no-cpu-baseline --sessions 1048576" ; do
  i=$((i+1)); echo "[r03f] $a"
  timeout -k 10 200 env $a > $OUT/bench$i.log 2>&1 || { echo "failed: $a"; tail -20 $OUT/bench$i.log; exit 1; }
  grep -h '^{' $OUT/bench$i.log | python3 tools/benchline.py "$a" || true
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py -m gpu -k "session" > $OUT/pytest_sess.log 2>&1 || { tail -30 $OUT/pytest_sess.log; exit 1; }
tail -1 $OUT/pytest_sess.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py -m gpu -k "c4 or stack or slot or lds or sign or pipelin or heavy or countdown or c5" > $OUT/pytest_c4.log 2>&1
rc=$?; tail -3 $OUT/pytest_c4.log; echo "rc=$rc"; exit $rc
