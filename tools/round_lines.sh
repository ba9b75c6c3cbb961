#!/bin/bash
# Every bench line of a round on one box (the results table of DESIGN.md /
# README.md): the configs at their bench sizes, the sessions row, and a
# two-rank gather rehearsal on the one GPU (gloo; not a scaling figure).
# Lines go to gpurun_out/TAG/lines.jsonl (bench_set.sh), each step under
# its own time limit.      bash tools/round_lines.sh TAG
set -o pipefail
TAG=$1
bash tools/probe/bench_set.sh $TAG "--config c2" "--config c3" "--config c4" "--config c4d256 --steps 10" \
  "--config c4d1024 --steps 5" "--config c5 --steps 10" "--config c2 --sessions 1048576 --steps 5 --warmup 1" \
  "--config t2_dyn_depth --steps 10" "--config t1_two_stacks --steps 10" "--config t_jro_heavy --steps 10" \
  "--config t_ring16 --steps 10" || exit 1
export TMPDIR=/tmp
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --same-device --dist-backend gloo --steps 5 --no-cpu-baseline \
  > gpurun_out/$TAG/two_rank.log 2>&1 || { tail -20 gpurun_out/$TAG/two_rank.log; exit 1; }
grep -h '^{' gpurun_out/$TAG/two_rank.log >> gpurun_out/$TAG/lines.jsonl
echo "[round_lines] done"
