set -o pipefail
mkdir -p gpurun_out/r02an
for d in 320 400 500 640; do
  for cfg in "MK_JIT_LDS_SLOTS=0" "MK_JIT_LDS_SLOTS=163840"; do
    timeout -k 10 120 env $cfg python tools/probe/pipeline_timing.py $d 262144 2>&1 | tail -1 | sed "s/^/$cfg /" || exit 1
  done
done
