set -o pipefail
mkdir -p gpurun_out/r01w
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --durations=25 --timeout 300 --timeout-method thread > gpurun_out/r01w/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r01w/pytest_gpu.log; exit 1; }
grep -A30 "slowest" gpurun_out/r01w/pytest_gpu.log | head -32
bash tools/gpu_round.sh r01w --no-tests -- "python bench.py --steps 20 --warmup 3 --cpu-seconds 10" "python bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline" "python bench.py --config c5 --steps 5 --warmup 1 --no-cpu-baseline" "python bench.py --config c4 --steps 10 --warmup 2 --no-cpu-baseline" "python bench.py --config c4d256 --steps 5 --warmup 1 --no-cpu-baseline" "python bench.py --config c4d1024 --steps 5 --warmup 1 --no-cpu-baseline"
