#!/bin/bash
# A/B of bench lines under labelled knob sets: "label:VAR=v VAR=v" per set,
# each set run over the given configs, two passes.
#   bash tools/probe/env_bench.sh TAG "cfg cfg" "lab:ENV..." ...
set -o pipefail
OUT=gpurun_out/$1; CFGS=$2; shift 2; mkdir -p $OUT; export TMPDIR=/tmp
for pass in 1 2; do
 for set in "$@"; do
  lab=${set%%:*}; envs=${set#*:}
  for c in $CFGS; do
   env $envs timeout -k 10 200 python bench.py --config $c --no-cpu-baseline --steps 20 > $OUT/b.log 2>&1 || { echo "fail $lab $c"; tail -5 $OUT/b.log; exit 1; }
   grep -h '^{' $OUT/b.log | sed "s/^/{\"label\": \"$lab\", \"r\": /; s/\$/}/" >> $OUT/ab.jsonl
  done
 done
done
python3 - $OUT/ab.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l); r = d["r"]; rf = r["roofline"]
    print(f'{d["label"]:10s} {r["config"]["workload"]:22s} {r["kernel_ms_per_step"] * 1e3:9.2f} us  {rf["bound"]} {rf["frac"]:.3f}')
PY
