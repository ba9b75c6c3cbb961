#!/bin/bash
# Where a bench config's dominant kernel spends its wave cycles: one
# rocprofv3 --pmc pass (kernel trace only) of SQ wave / wait / active-instruction
# counters, each under its own time limit.
#   bash tools/gpu_pmc_stall.sh TAG CONFIG [ENV=VALUE ...]
set -o pipefail
TAG=$1; CFG=$2; shift 2
OUT=gpurun_out/$TAG/$CFG
mkdir -p "$OUT"
export TMPDIR=/tmp
for kv in "$@"; do export "$kv"; done
STALL="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SALU SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH GRBM_GUI_ACTIVE"
echo "[pmc-stall] $(date +%T) $CFG"
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $STALL --output-format csv -d "$OUT/STALL" -o p -- \
  python3 bench.py --config $CFG --steps 6 --warmup 1 --no-cpu-baseline > "$OUT/STALL.log" 2>&1 \
  || { echo "[pmc-stall] failed"; tail -5 "$OUT/STALL.log"; exit 1; }
python3 - "$OUT/STALL" <<'PY'
import collections, csv, glob, sys
rows = collections.defaultdict(lambda: collections.defaultdict(float))
for p in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        if r["Kernel_Name"].startswith("mk_jit_exec"):
            rows[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
ids = sorted(rows)[2:]
for c in sorted(rows[ids[0]]):
    print(f"{c:24s} {sum(rows[i][c] for i in ids) / len(ids):16.0f}")
PY
echo "[pmc-stall] done"
