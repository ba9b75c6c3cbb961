#!/bin/bash
# Round 6 A/B: C5 under labelled knob sets ("label:VAR=v VAR=v"), full range
# and all-zero inputs, two passes.   bash tools/probe/c5_exp.sh TAG "lab:ENV..." ...
set -o pipefail
OUT=gpurun_out/$1; shift; mkdir -p $OUT; export TMPDIR=/tmp
for pass in 1 2; do
 for m in ${C5_MASKS:-1023 0}; do
  for set in "$@"; do
   lab=${set%%:*}; envs=${set#*:}
   env $envs timeout -k 10 120 python -u tools/probe/c5_decomp.py $m 4194304 20 \
     | sed "s/^/{\"label\": \"$lab\", \"r\": /; s/\$/}/" >> $OUT/exp.jsonl || { echo fail $lab; exit 1; }
  done
 done
done
python3 - $OUT/exp.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l); r = d["r"]
    print(f'{d["label"]:10s} mask {r["mask"]:5d} {r["us_per_launch"]:8.2f} us  {r["kernel"]}')
PY
