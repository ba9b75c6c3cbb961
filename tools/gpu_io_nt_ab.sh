#!/bin/bash
# A/B: normal vs non-temporal out/status stores in the light stream kernel
# (MK_JIT_IO_NT), alternating runs of the C2 and C3 bench lines.
set -e
OUT=gpurun_out/io_nt_ab
mkdir -p "$OUT"
for rep in 1 2; do
  for nt in 0 1; do
    for c in c2 c3; do
      MK_JIT_IO_NT=$nt timeout -k 10 120 python3 bench.py --config $c --steps 50 > "$OUT/${c}_nt${nt}_r${rep}.json"
      python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2],sys.argv[3],round(d['roofline']['launch_us'],2),round(d['roofline']['frac'],3))" "$OUT/${c}_nt${nt}_r${rep}.json" $c nt$nt | tee -a "$OUT/summary.txt"
    done
  done
done
