# r03h: rocprofv3 kernel stats + PMC passes (FETCH / WRITE / SQ / LDS, then
# stall counters) of the final tree's bench configs, each pass its own run
set -o pipefail
export TMPDIR=/tmp
bash tools/gpu_profiles.sh r03h c2 c4 c4d256 c4d1024 c5 || exit 1
bash tools/gpu_pmc_all.sh r03h_pmc c2 c4 c4d256 c4d1024 c5 || exit 1
bash tools/gpu_pmc_stall.sh r03h_stall c4d256 || exit 1
bash tools/gpu_pmc_stall.sh r03h_stall c5 || exit 1
bash tools/gpu_pmc_stall.sh r03h_stall c4 || exit 1
echo done
