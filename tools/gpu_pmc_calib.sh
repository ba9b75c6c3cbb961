#!/bin/bash
# Byte-count calibration of FETCH_SIZE / WRITE_SIZE for the stack-slot access
# pattern (tools/probe/pmc_calib.hip): one rocprofv3 --pmc pass per counter
# and mode, kernel trace only, each under its own time limit.
#   bash tools/gpu_pmc_calib.sh TAG [MIB]
set -o pipefail
TAG=${1:-calib}; MIB=${2:-4096}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for m in st4 ld4 ld16; do
  timeout -k 10 60 ./tools/probe/pmc_calib $m $MIB > "$OUT/$m.json" || { echo "[calib] $m failed"; exit 1; }
  mkdir -p "$OUT/$m"
  for c in FETCH_SIZE WRITE_SIZE; do
    echo "[calib] $(date +%T) $m $c"
    timeout -s KILL 60 rocprofv3 --kernel-trace --pmc $c --output-format csv -d "$OUT/$m/$c" -o p -- ./tools/probe/pmc_calib $m $MIB > "$OUT/$m/$c.log" 2>&1 || { echo "[calib] failed $m $c"; tail -5 "$OUT/$m/$c.log"; exit 1; }
  done
done
python3 tools/pmc_calib_fold.py "$OUT"
