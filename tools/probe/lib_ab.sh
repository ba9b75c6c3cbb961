#!/bin/bash
# A/B of two builds of the library (the kernel generator is compiled into
# it): misaka-net_amd/lib/ab_new.so and ab_old.so take turns as
# libmisaka_amd.so; C5 at full range and all-zero (c5_decomp.py) and bench
# lines for the given configs, two passes.  The new build is left in place.
#   bash tools/probe/lib_ab.sh TAG "cfg ..."
set -o pipefail
OUT=gpurun_out/$1; CFGS=$2; mkdir -p $OUT; export TMPDIR=/tmp
L=misaka-net_amd/lib
for pass in 1 2; do
 for v in new old; do
  cp $L/ab_$v.so $L/libmisaka_amd.so || exit 1
  for m in 1023 0; do
   echo "{\"label\": \"$v\", \"r\": $(timeout -k 10 120 python -u tools/probe/c5_decomp.py $m 4194304 20)}" >> $OUT/c5.jsonl || exit 1
  done
  for c in $CFGS; do
   timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --steps 20 > $OUT/b.log 2>&1 || { echo "fail $v $c"; tail -5 $OUT/b.log; exit 1; }
   grep -h '^{' $OUT/b.log | sed "s/^/{\"label\": \"$v\", \"r\": /; s/\$/}/" >> $OUT/ab.jsonl
  done
 done
done
cp $L/ab_new.so $L/libmisaka_amd.so
python3 - $OUT <<'PY'
import json, sys
for l in open(sys.argv[1] + "/c5.jsonl"):
    d = json.loads(l); r = d["r"]
    print(f'{d["label"]:5s} c5 mask {r["mask"]:5d} {r["us_per_launch"]:8.2f} us  {r["kernel"]}')
try:
    for l in open(sys.argv[1] + "/ab.jsonl"):
        d = json.loads(l); r = d["r"]
        print(f'{d["label"]:5s} {r["config"]["workload"]:22s} {r["kernel_ms_per_step"] * 1e3:9.2f} us')
except FileNotFoundError:
    pass
PY
