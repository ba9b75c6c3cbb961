#!/bin/bash
# r02f: mixed-deployment tests first, then the whole GPU suite.
set -o pipefail
OUT=gpurun_out/r02f; mkdir -p $OUT; export TMPDIR=/tmp
step() { local t=$1; shift; echo "[r02f] $(date +%T) $*"; timeout -k 10 "$t" "$@"; }
step 300 python -u -m pytest tests/test_mixed.py tests/test_master.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "mixed or http or session or interp or trace or c5 or random_networks" > $OUT/pytest_mixed.log 2>&1; rc=$?
tail -c 3000 $OUT/pytest_mixed.log; [ $rc -le 1 ] || exit 1
step 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -5 $OUT/pytest_gpu.log; exit $rc
