#!/bin/bash
# Counter passes for the bench workloads (rocprofv3 --pmc, kernel trace only,
# one pass per counter group, each under its own time limit):
#   FETCH_SIZE | WRITE_SIZE | SQ instruction / cycle counters + GRBM_GUI_ACTIVE | LDS counters
# then tools/pmc_profile.py folds them into profiles/pmc_<workload>.json,
# which bench.py reads for roofline.traffic and the executed-work roofline.
#   bash tools/gpu_pmc_all.sh TAG CONFIG [CONFIG ...]     (CONFIG: c2 c3 c4 c4d256 c4d1024 c5)
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
# LDS pass (stack slots kept in LDS by the heavy kernel; the tile-sorted kernel's buckets)
LDS="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES GRBM_GUI_ACTIVE"
for cfg in "$@"; do
  for pass in FETCH_SIZE WRITE_SIZE SQ LDS; do
    case $pass in SQ) ctr=$SQ ;; LDS) ctr=$LDS ;; *) ctr=$pass ;; esac
    echo "[pmc] $(date +%T) $cfg $pass"; mkdir -p "$OUT/$cfg"
    timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $ctr --output-format csv -d "$OUT/$cfg/$pass" -o p -- \
      python3 bench.py --config $cfg --steps 6 --warmup 1 --no-cpu-baseline > "$OUT/$cfg/$pass.log" 2>&1 \
      || { echo "[pmc] failed $cfg $pass"; tail -5 "$OUT/$cfg/$pass.log"; exit 1; }
  done
done
echo "[pmc] done"
