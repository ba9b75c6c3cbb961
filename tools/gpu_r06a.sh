set -o pipefail
OUT=gpurun_out/r06a; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -k "c3_full_64m or readme_kat" > $OUT/pytest.log 2>&1 &&
timeout -k 10 300 python bench.py --gpus 2 --same-device --dist-backend gloo --steps 10 --warmup 2 > $OUT/bench_2rank.log 2> $OUT/bench_2rank.err &&
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-seconds 10 > $OUT/bench_c2.log 2> $OUT/bench_c2.err
rc=$?; echo rc=$rc; tail -3 $OUT/pytest.log; cat $OUT/bench_2rank.log | cut -c1-600; exit $rc
