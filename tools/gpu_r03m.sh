# r03m: the crash-at-exit probe without pytest: no PyTorch (this ROCm's
# runtime + hiprtc in process), PyTorch first (helper compile), PyTorch first
# with its bundled hiprtc; concurrent processes started together
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03m; mkdir -p $OUT
run() { local tag=$1; shift; env "$@" PYTHONFAULTHANDLER=1 timeout -k 10 400 python -u tools/probe/dyn_stack_probe.py $ARG > $OUT/probe_$tag.log 2>&1; echo "$tag rc=$?" >> $OUT/rcs.txt; }
ARG=none run notorch MK_NONE=1 &
ARG=torch run torch_helper MK_NONE=1 &
ARG=torch run torch_linked MK_HIPRTC=linked &
wait
cat $OUT/rcs.txt
for t in notorch torch_helper torch_linked; do echo "== $t"; tail -3 $OUT/probe_$t.log | cut -c1-160; done
