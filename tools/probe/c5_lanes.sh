#!/bin/bash
# C5 launch time per lane against the lane count (tiles per block of the
# tile-sorted kernel's resident grid): tools/probe/c5_decomp.py at mask 1023.
#   bash tools/probe/c5_lanes.sh TAG [ENV=VALUE ...]
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for kv in "$@"; do export "$kv"; done
for n in 4194304 5242880 6291456 8388608 3145728; do
  echo "[c5_lanes] $(date +%T) $n $*"
  timeout -k 10 120 python tools/probe/c5_decomp.py 1023 $n 20 >> "$OUT/c5_lanes.jsonl" || exit 1
done
python3 -c "
import json
for l in open('$OUT/c5_lanes.jsonl'):
    d = json.loads(l); print(d['lanes'], d['us_per_launch'], round(d['ns_per_lane'] * 1e3, 3), 'ps/lane', d['knobs'])
"
