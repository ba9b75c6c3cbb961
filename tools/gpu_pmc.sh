#!/bin/bash
# PMC passes for the bench kernel (one rocprofv3 run per counter group; no
# trace domains are combined with --pmc).  Usage: bash tools/gpu_pmc.sh tag [bench args]
set -o pipefail
TAG=${1:-pmc}; shift
ARGS=${@:---steps 3 --warmup 1 --no-cpu-baseline}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { local t=$1; shift; echo "[gpu_pmc] $(date +%T) $*"; timeout -k 10 "$t" "$@"; }
step 120 rocprofv3 -L > "$OUT/counters_list.txt" 2>&1
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY" \
           "SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  step 300 rocprofv3 --kernel-trace --pmc $grp --output-format csv -d "$OUT/pmc$i" -o p -- python bench.py $ARGS > "$OUT/pmc$i.log" 2>&1 || { echo "[gpu_pmc] pass $i failed"; exit 1; }
done
echo "[gpu_pmc] done"
