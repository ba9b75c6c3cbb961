set -o pipefail
mkdir -p gpurun_out/r01o
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r01o/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r01o/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r01o/pytest_gpu.log
bash tools/gpu_pmc_bytes.sh r01o_b_c4 "--config c4 --steps 5 --warmup 1 --no-cpu-baseline" &&
bash tools/gpu_pmc_bytes.sh r01o_b_c4d256 "--config c4d256 --steps 5 --warmup 1 --no-cpu-baseline" &&
bash tools/gpu_pmc_bytes.sh r01o_b_c4d1024 "--config c4d1024 --steps 5 --warmup 1 --no-cpu-baseline" &&
bash tools/gpu_profiles.sh r01o c4 c4d256 c4d1024
