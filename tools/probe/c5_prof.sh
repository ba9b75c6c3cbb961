#!/bin/bash
# C5 phase profile (MK_JIT_PROF) and launch times at a few input ranges:
#   bash tools/probe/c5_prof.sh TAG [knob=value ...]
set -e -o pipefail
TAG=${1:?tag}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for kv in "$@"; do export "$kv"; done
for m in 0 63 1023; do
  timeout -k 10 120 python -u tools/probe/c5_decomp.py $m | tee -a "$OUT/plain.jsonl"
  MK_JIT_PROF=1 timeout -k 10 120 python -u tools/probe/c5_decomp.py $m | tee -a "$OUT/prof.jsonl"
done
echo "[c5_prof] done"
