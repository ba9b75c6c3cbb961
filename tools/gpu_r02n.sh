#!/bin/bash
# r02n: PMC passes + kernel stats for the machine-shape workloads after the
# side exits and the sort kernel's counters.
set -o pipefail
bash tools/gpu_pmc_all.sh r02n c5 t2_dyn_depth t1_two_stacks && bash tools/gpu_profiles.sh r02n c5 t2_dyn_depth t1_two_stacks
