#!/bin/bash
# Round 6: C5's tile-to-block quantization.  Launch time against lanes (1, 2,
# 2.67, 3 tiles per resident block at 6 blocks per CU) and against the grid
# (MK_JIT_PER_CU: blocks per CU; 16 = one tile per block, hardware refill).
#   bash tools/probe/c5_grid.sh TAG
set -o pipefail
OUT=gpurun_out/$1; mkdir -p $OUT; export TMPDIR=/tmp
for m in 1023 0; do
 for n in 1572864 3145728 4194304 4718592; do
  for pc in "" 4 16; do
   echo "{\"per_cu\": \"$pc\", \"r\": $(MK_JIT_PER_CU=$pc timeout -k 10 120 python -u tools/probe/c5_decomp.py $m $n 20)}" >> $OUT/grid.jsonl || exit 1
  done
 done
done
python3 - $OUT/grid.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l); r = d["r"]
    print(f'per_cu {d["per_cu"] or "-":3s} mask {r["mask"]:5d} lanes {r["lanes"]:8d} {r["us_per_launch"]:8.2f} us  {r["lanes"] / r["us_per_launch"] / 1e3:7.2f} Glanes/s')
PY
