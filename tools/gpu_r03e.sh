# r03e: the r03d crash-at-exit subset with the quad LDS layout off
set -o pipefail
OUT=gpurun_out/r03e; mkdir -p $OUT; export TMPDIR=/tmp; export PYTHONFAULTHANDLER=1
MK_JIT_LDS_QUAD=0 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -p no:cacheprovider tests/test_gpu_parity.py -m gpu -k "c4 or stack or slot or lds or sign or pipelin or heavy or countdown or c5" > $OUT/pytest_c4.log 2>&1
rc=$?; tail -3 $OUT/pytest_c4.log; echo "rc=$rc"; exit $rc
