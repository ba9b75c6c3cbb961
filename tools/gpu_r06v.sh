#!/bin/bash
# Round 5, sweep dispatch: PMC passes of the machine-shape configs, the C5
# stall pass and kernel stats, and census-class bench lines with the sweep
# off and on.  Every GPU step under its own time limit, chained.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06v
mkdir -p "$OUT"
bash tools/gpu_pmc_all.sh r06v c5 t2_dyn_depth t1_two_stacks t_jro_heavy || exit 1
bash tools/gpu_pmc_stall.sh r06v c5 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/c5_stats" -o p -- \
  python3 bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/c5_stats.log" 2>&1 || exit 1
for cfg in t2_dyn_depth t1_two_stacks t_jro_heavy c5; do
  for sw in 0 1; do
    echo "[r06v] $(date +%T) $cfg sweep=$sw"
    MK_JIT_SWEEP=$sw timeout -k 10 200 python3 bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline \
      > "$OUT/bench_${cfg}_sw$sw.log" 2>&1 || { echo "[r06v] failed $cfg $sw"; tail -5 "$OUT/bench_${cfg}_sw$sw.log"; exit 1; }
    grep -h '^{' "$OUT/bench_${cfg}_sw$sw.log" | python3 tools/benchline.py "$cfg sweep=$sw" || true
  done
done
echo "[r06v] done"
