# r03r: final tree -- C5 counter passes folded on the box (profiles/pmc_c5_*.json
# for the bench lines below), rocprofv3 kernel stats of C5, the full GPU suite,
# smoke, every config's bench line (tools/gpu_r03o.sh)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03r; mkdir -p $OUT
bash tools/gpu_pmc_all.sh r03r_pmc c5 || exit 1
python3 tools/pmc_profile.py r03r_pmc c5 > $OUT/pmc_fold.log 2>&1 || { cat $OUT/pmc_fold.log; exit 1; }
cp profiles/pmc_c5_countdown_4M.json $OUT/
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c5stats -o p -- \
  python3 bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/c5stats.log 2>&1 || { tail -20 $OUT/c5stats.log; exit 1; }
bash tools/gpu_r03o.sh
