#!/bin/bash
# Where a bench config's dominant kernel spends its wave cycles: one
# rocprofv3 --pmc pass (kernel trace only) of SQ wave / wait / active-instruction
# counters, each under its own time limit.
#   bash tools/gpu_pmc_stall.sh TAG CONFIG [ENV=VALUE ...]
# PMC_ARGS="script args" profiles `python3 script args` instead of the bench
# config (CONFIG then only names the output directory).
set -o pipefail
TAG=$1; CFG=$2; shift 2
OUT=gpurun_out/$TAG/$CFG
mkdir -p "$OUT"
export TMPDIR=/tmp
for kv in "$@"; do export "$kv"; done
STALL="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SALU SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH GRBM_GUI_ACTIVE"
# second pass: instruction mix and the LDS-issue share of the issue stalls
STALL2="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE"
for pass in STALL STALL2; do
echo "[pmc-stall] $(date +%T) $CFG $pass"
timeout -s KILL 150 rocprofv3 --kernel-trace --pmc ${!pass} --output-format csv -d "$OUT/$pass" -o p -- \
  python3 ${PMC_ARGS:-bench.py --config $CFG --steps 6 --warmup 1 --no-cpu-baseline} > "$OUT/$pass.log" 2>&1 \
  || { echo "[pmc-stall] failed"; tail -5 "$OUT/$pass.log"; exit 1; }
python3 - "$OUT/$pass" <<'PY'
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
done
echo "[pmc-stall] done"
