set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r02s
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r02s/prof -o s -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --sessions 1048576 > gpurun_out/r02s/b.log 2>&1 || { tail -20 gpurun_out/r02s/b.log; exit 1; }
cat gpurun_out/r02s/prof/s_kernel_stats.csv | cut -c1-160
