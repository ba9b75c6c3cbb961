#!/bin/bash
# Round 5, hybrid sweep (one sweep pass, then rounds): GPU suite, C5 sessions
# burst timing, the 190-variant random network, PMC passes of the machine
# configs, C5 stall pass and kernel stats.  Each GPU step under its own limit.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r07m
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > "$OUT/pytest_gpu.log" 2>&1 || { tail -30 "$OUT/pytest_gpu.log"; exit 1; }
tail -1 "$OUT/pytest_gpu.log"
for sw in 0 1; do
  echo -n "sessions c5 sweep=$sw "
  MK_JIT_SWEEP=$sw timeout -k 10 120 python3 tools/probe/session_prof.py burst 1048576 5 8 countdown | cut -c1-120 || exit 1
done
for seed in 139 328; do
  echo -n "random $seed "; timeout -k 10 120 python3 tools/probe/random_net_timing.py $seed 1048576 3 2>/dev/null || exit 1
done
bash tools/gpu_pmc_all.sh r07m c5 t2_dyn_depth t1_two_stacks t_jro_heavy > "$OUT/pmc.log" 2>&1 || { tail -5 "$OUT/pmc.log"; exit 1; }
bash tools/gpu_pmc_stall.sh r07m c5 > "$OUT/stall.txt" 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c5_stats" -o p -- \
  python3 bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/c5_stats.log" 2>&1 || exit 1
echo "[r07m] done"
