# HBM-slot heavy kernels: stack entries kept in registers (MK_SCHED_SOFT_REGS) at several depths
set -o pipefail
for d in 400 640 1024; do
  for r in 24 48 64; do
    timeout -k 10 180 env MK_SCHED_SOFT_REGS=$r MK_JIT_TUNE_REGS=0 python tools/probe/pipeline_timing.py $d 262144 2>&1 | tail -1 | sed "s/^/regs=$r /" || exit 1
  done
done
