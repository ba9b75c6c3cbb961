#!/bin/bash
# Alternating A/B of C5 launch times (tools/probe/c5_decomp.py, 4M lanes,
# inputs in [0, 1023]) over labelled knob sets, two passes, each run under
# its own time limit.   bash tools/probe/c5_ab.sh TAG "label: VAR=v ..." ...
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
for pass in 1 2; do
  for set in "$@"; do
    label=${set%%:*}
    envs=${set#*:}
    echo "[c5_ab] $(date +%T) pass $pass $label"
    env $envs timeout -k 10 120 python tools/probe/c5_decomp.py 1023 $((1 << 22)) 20 \
      | sed "s/^/{\"label\": \"$label\", \"pass\": $pass, \"r\": /; s/\$/}/" >> "$OUT/c5_ab.jsonl" \
      || { echo "[c5_ab] failed: $label"; exit 1; }
  done
done
python3 - "$OUT/c5_ab.jsonl" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    print(f"{d['label']:14s} pass {d['pass']}  {d['r']['us_per_launch']:8.2f} us  {d['r'].get('kernel', '')}")
PY
