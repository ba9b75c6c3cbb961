#!/bin/bash
# r02b: GPU suite (sessions seq, master concurrency), 2-rank same-device gloo
# gather check, PMC passes for every bench workload, default bench with the
# CPU baselines and the HTTP leg.
set -o pipefail
OUT=gpurun_out/r02b; mkdir -p $OUT; export TMPDIR=/tmp
step() { local t=$1; shift; echo "[r02b] $(date +%T) $*"; timeout -k 10 "$t" "$@"; }
step 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; [ $rc -le 1 ] || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
step 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --gpus 2 --same-device --dist-backend gloo --config c3 --lanes 1048576 --steps 3 --warmup 1 \
  --no-cpu-baseline --verify-gather > $OUT/bench_2rank_gloo.log 2>&1 || { tail -30 $OUT/bench_2rank_gloo.log; exit 1; }
grep -h '^{' $OUT/bench_2rank_gloo.log | cut -c1-300
step 1200 bash tools/gpu_pmc_all.sh r02b/pmc c2 c3 c4 c4d256 c4d1024 c5 > $OUT/pmc.log 2>&1 || { tail -20 $OUT/pmc.log; exit 1; }
step 300 python bench.py --steps 20 --warmup 3 --cpu-seconds 10 --http 64 > $OUT/bench_c2.log 2>&1 || { tail -20 $OUT/bench_c2.log; exit 1; }
grep -h '^{' $OUT/bench_c2.log | cut -c1-300
echo "[r02b] done"
