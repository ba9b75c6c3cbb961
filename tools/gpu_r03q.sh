# r03q: the C5 / C4 d256 knob A/B (r03p), then the crash-at-exit probe with
# MK_JIT_KEEP_MODULES=1 (modules never unloaded; r03k/r03m: the same probe
# without it ended rc=139)
set -o pipefail
export TMPDIR=/tmp
bash tools/gpu_r03p.sh || exit 1
OUT=gpurun_out/r03q; mkdir -p $OUT
MK_JIT_KEEP_MODULES=1 PYTHONFAULTHANDLER=1 timeout -k 10 400 python -u tools/probe/dyn_stack_probe.py torch > $OUT/probe_keep.log 2>&1
echo "keep rc=$?" | tee $OUT/rcs.txt
tail -3 $OUT/probe_keep.log | cut -c1-200
