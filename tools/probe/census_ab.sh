#!/bin/bash
# Alternating A/B of one bench config's launch time over labelled knob sets,
# two passes, each run under its own time limit.
#   bash tools/probe/census_ab.sh TAG CONFIG "label: VAR=v ..." ...
set -o pipefail
TAG=$1; CFG=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for pass in 1 2; do
  for set in "$@"; do
    label=${set%%:*}
    envs=${set#*:}
    env $envs timeout -k 10 200 python3 bench.py --config $CFG --steps 5 --warmup 1 --no-cpu-baseline \
      > "$OUT/${CFG}_${label}_$pass.log" 2>&1 || { echo "[census_ab] failed: $label"; exit 1; }
    grep -h '^{' "$OUT/${CFG}_${label}_$pass.log" | python3 -c "
import json, sys
d = json.loads(sys.stdin.read())
print(f\"$CFG $label pass $pass  {d['roofline_hbm']['launch_us']:10.1f} us\")"
  done
done
