#!/bin/bash
# SQ counters of C5 (c5_decomp.py, full range) under each of two library
# builds (ab_new.so / ab_old.so as libmisaka_amd.so), one rocprofv3 --pmc
# pass each; the new build is left in place.   bash tools/probe/lib_pmc.sh TAG
set -o pipefail
OUT=gpurun_out/$1; mkdir -p $OUT; export TMPDIR=/tmp
L=misaka-net_amd/lib
CTR="SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH GRBM_GUI_ACTIVE"
for v in new old; do
  cp $L/ab_$v.so $L/libmisaka_amd.so || exit 1
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $CTR --output-format csv -d $OUT/pmc_$v -o p -- \
    python3 tools/probe/c5_decomp.py 1023 4194304 4 > $OUT/pmc_$v.log 2>&1 || { echo "fail $v"; tail -5 $OUT/pmc_$v.log; exit 1; }
done
cp $L/ab_new.so $L/libmisaka_amd.so
python3 - $OUT <<'PY'
import csv, collections, glob, sys
for v in ("new", "old"):
    rows = collections.defaultdict(lambda: collections.defaultdict(float))
    for p in glob.glob(f"{sys.argv[1]}/pmc_{v}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(p)):
            if r["Kernel_Name"].startswith("mk_jit_exec"):
                rows[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    d = sorted(rows)[-1]
    print(v, {k: int(x) for k, x in sorted(rows[d].items())})
PY
