#!/bin/bash
# r02p: the other two census classes (JRO-heavy loop, 16-node ring) as bench
# workloads, with PMC passes and kernel stats.
set -o pipefail
OUT=gpurun_out/r02p; mkdir -p $OUT; export TMPDIR=/tmp
bash tools/gpu_pmc_all.sh r02p t_jro_heavy t_ring16 && bash tools/gpu_profiles.sh r02p t_jro_heavy t_ring16
