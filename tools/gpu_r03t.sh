# r03t: the C client of the ABI (no PyTorch: this ROCm's hiprtc and runtime)
# on C2 / C4 d64 / C5, its GPU tests, and C5's wave-cycle split after the
# saturating countdown (tools/gpu_pmc_stall.sh)
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03t; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_abi.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_abi.log 2>&1 || { tail -30 $OUT/pytest_abi.log; exit 1; }
tail -1 $OUT/pytest_abi.log
gcc -std=c99 -O2 -D__HIP_PLATFORM_AMD__ -I include -I /opt/rocm/include integration/c/mk_bench.c -L misaka-net_amd/lib -lmisaka_amd -L /opt/rocm/lib -lamdhip64 -Wl,-rpath,$PWD/misaka-net_amd/lib -Wl,-rpath,/opt/rocm/lib -o /tmp/mk_bench || exit 1
for a in "c2 20 3" "c4:64 20 3" "c5 10 2"; do timeout -k 10 120 /tmp/mk_bench $a | tee -a $OUT/cbench.jsonl || exit 1; done
bash tools/gpu_pmc_stall.sh r03t_stall c5 | tee $OUT/stall_c5.txt
