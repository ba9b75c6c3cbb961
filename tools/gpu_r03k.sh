# r03k: the native-tier crash-at-exit probe (dynamic-stack parity tests,
# mode auto), four variants as concurrent processes started together
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03k; mkdir -p $OUT
run() { local tag=$1; shift; env "$@" PYTHONFAULTHANDLER=1 timeout -k 10 400 python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py -m gpu -k "dynamic_stack_networks and auto" > $OUT/pytest_$tag.log 2>&1; echo "$tag rc=$?" >> $OUT/rcs.txt; }
run default MK_NONE=1 &
run linked MK_HIPRTC=linked &
run notsort MK_JIT_TILE_SORT=0 &
run jit_off MK_JIT=0 &
wait
cat $OUT/rcs.txt
for t in default linked notsort jit_off; do echo "== $t"; tail -2 $OUT/pytest_$t.log | cut -c1-160; done
