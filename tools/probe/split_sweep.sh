# Heavy-kernel slots split between LDS and HBM (MK_JIT_LDS_SPLIT) against HBM only
set -o pipefail
for d in ${DEPTHS:-400 480 560 640 1024}; do
  for cfg in "MK_JIT_LDS_SPLIT=0" "MK_JIT_LDS_SPLIT=1"; do
    timeout -k 10 180 env $cfg python tools/probe/pipeline_timing.py $d 262144 2>&1 | tail -1 | sed "s/^/$cfg /" || exit 1
  done
done
