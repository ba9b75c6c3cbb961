#!/bin/bash
# r02k: PMC passes and kernel stats for the machine-shape workloads after the
# tile-sorted kernel (the committed profiles/pmc_*.json feed bench.py's
# executed-work roofline).
set -o pipefail
bash tools/gpu_pmc_all.sh r02k c5 t2_dyn_depth t1_two_stacks && bash tools/gpu_profiles.sh r02k c5 t2_dyn_depth t1_two_stacks
