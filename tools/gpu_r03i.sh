# r03i: final-tree profiles (rocprofv3 kernel stats, PMC FETCH / WRITE / SQ /
# LDS passes, stall counters), the C client, smoke; then a bisect probe of
# the r03c-h crash at exit (last: an abort ends the call)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03i; mkdir -p $OUT
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
gcc -std=c99 -O2 -D__HIP_PLATFORM_AMD__ -I include -I /opt/rocm/include integration/c/mk_bench.c -L misaka-net_amd/lib -lmisaka_amd -L /opt/rocm/lib -lamdhip64 -Wl,-rpath,$PWD/misaka-net_amd/lib -Wl,-rpath,/opt/rocm/lib -o /tmp/mk_bench
for a in "c2 20 3" "c4:64 20 3" "c4:256 10 2" "c4:1024 5 1"; do timeout -k 10 120 /tmp/mk_bench $a | tee -a $OUT/cbench.jsonl || exit 1; done
bash tools/gpu_profiles.sh r03i c2 c4 c4d256 c4d1024 c5 || exit 1
bash tools/gpu_pmc_all.sh r03i_pmc c2 c4 c4d256 c4d1024 c5 || exit 1
for c in c4d256 c5 c4 c4d1024; do bash tools/gpu_pmc_stall.sh r03i_stall $c || exit 1; done
PYTHONFAULTHANDLER=1 timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py -m gpu -k "dynamic_stack_networks" > $OUT/pytest_dyn.log 2>&1
rc=$?; tail -4 $OUT/pytest_dyn.log | cut -c1-200; echo "rc=$rc"; exit $rc
