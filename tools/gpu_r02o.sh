#!/bin/bash
# r02o: the N>1 path of bench.py (shards, counter all-reduce, ordered gather
# of outputs + statuses, end-to-end value) rehearsed with 2 and 4 ranks on the
# one GPU of the box (gloo; the driver's 8-GPU runs use RCCL).
set -o pipefail
OUT=gpurun_out/r02o; mkdir -p $OUT; export TMPDIR=/tmp
step() { local t=$1; shift; echo "[r02o] $(date +%T) $*"; timeout -k 10 "$t" "$@"; }
for n in 2 4; do
  step 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 29517 \
    bench.py --gpus $n --steps 5 --warmup 1 --same-device --dist-backend gloo > $OUT/bench_n$n.log 2>&1 \
    || { tail -30 $OUT/bench_n$n.log; exit 1; }
  grep -h '^{' $OUT/bench_n$n.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); print('n=$n', d['n_gpus'], round(d['value']/1e12,3),'T', d.get('end_to_end'))"
done
