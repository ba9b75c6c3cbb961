#!/bin/bash
# Stateful sessions on the GPU box: for each launch kind
# (one call per launch, a burst of 8 calls per launch) a rocprofv3 kernel
# trace with stats, then PMC passes (FETCH_SIZE | WRITE_SIZE | SQ group), each
# its own run under its own time limit.  tools/sess_roofline.py folds them.
#   bash tools/gpu_sessprof.sh TAG [instances]
set -o pipefail
TAG=${1:-sess}; N=${2:-1048576}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_ANY GRBM_GUI_ACTIVE"
step() { local t=$1; shift; echo "[sessprof] $(date +%T) $*"; timeout -k 10 "$t" "$@"; }
for mode in percall burst; do
  mkdir -p "$OUT/$mode"
  step 150 python3 tools/probe/session_prof.py $mode $N 10 > "$OUT/$mode.json" 2> "$OUT/$mode.err" || { tail -5 "$OUT/$mode.err"; exit 1; }
  step 150 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/$mode/stats" -o s -- \
    python3 tools/probe/session_prof.py $mode $N 10 > "$OUT/$mode/stats.log" 2>&1 || { tail -5 "$OUT/$mode/stats.log"; exit 1; }
  for pass in FETCH_SIZE WRITE_SIZE SQ; do
    case $pass in SQ) ctr=$SQ ;; *) ctr=$pass ;; esac
    timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $ctr --output-format csv -d "$OUT/$mode/$pass" -o p -- \
      python3 tools/probe/session_prof.py $mode $N 10 > "$OUT/$mode/$pass.log" 2>&1 || { echo "[sessprof] $mode $pass failed"; tail -5 "$OUT/$mode/$pass.log"; exit 1; }
  done
done
echo "[sessprof] done"
