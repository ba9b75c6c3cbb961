#!/bin/bash
# SQ instruction/cycle counters (two rocprofv3 --pmc passes, kernel trace only)
# for each bench argument set.  bash tools/gpu_pmc_sq.sh TAG "ENV=.. args" ...
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
G1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"
G2="SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE"
# lane utilisation of VALU issue (rocprof's VALUUtilization) and the integer VALU mix
G3="SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU SQ_WAVES"
i=0
for a in "$@"; do
  i=$((i+1))
  envs=""; args=""
  for w in $a; do case $w in *=*) envs="$envs $w";; *) args="$args $w";; esac; done
  j=0
  for grp in "$G1" "$G2" "$G3"; do
    j=$((j+1))
    echo "[pmc] $(date +%T) set $i pass $j: $a"
    mkdir -p "$OUT/set$i"
    ( [ -n "$envs" ] && export $envs; timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d "$OUT/set$i/pmc$j" -o p -- python3 $args ) > "$OUT/set$i/pmc$j.log" 2>&1 || { echo "[pmc] failed set $i pass $j"; tail -5 "$OUT/set$i/pmc$j.log"; exit 1; }
  done
done
echo "[pmc] done"
