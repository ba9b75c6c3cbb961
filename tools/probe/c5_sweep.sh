#!/bin/bash
# C5 decomposition on the GPU box (tools/probe/c5_decomp.py):
#   bash tools/probe/c5_sweep.sh TAG
# 1. launch time and retired instructions per lane against the input range;
# 2. the machine kernel's knobs at bench.py's range (mask 1023);
# 3. executed VALU / SALU per launch at masks 0 and 1023 (one PMC pass each).
# Every GPU step has its own time limit; the first failure ends the script.
set -e -o pipefail
TAG=${1:?tag}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
P="python -u tools/probe/c5_decomp.py"
for m in 0 1 15 63 255 1023 4095; do
  timeout -k 10 120 $P $m | tee -a "$OUT/masks.jsonl"
done
for kv in MK_JIT_UNIFORM_SW=0 MK_JIT_TS_WAVES=8 MK_JIT_TS_ROUNDS=8 MK_JIT_TS_DYN=1 MK_JIT_LOOP_UNROLL=16 \
          MK_JIT_LOOP_UNROLL=64; do
  export "$kv"
  timeout -k 10 120 $P 1023 | tee -a "$OUT/knobs.jsonl"
  unset "${kv%%=*}"
done
for m in 0 1023; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_INSTS_LDS SQ_INSTS_BRANCH \
    SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -d "$OUT/pmc_$m" -o p -- python3 tools/probe/c5_decomp.py $m \
    > "$OUT/pmc_$m.log" 2>&1
done
echo "[c5_sweep] done"
