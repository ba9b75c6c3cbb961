"""Diagnostic: launch time of the C4 pipeline at any depth on generated
inputs, for A/B runs of MK_JIT_LDS_SLOTS / MK_SCHED_SOFT_REGS / MK_JIT_TUNE_REGS.
  python tools/probe/pipeline_timing.py DEPTH LANES"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import misaka_net_amd as mk  # noqa: E402
from misaka_net_amd import _native as N  # noqa: E402

depth, n = int(sys.argv[1]), int(sys.argv[2])
net = mk.Network(mk.networks.pipeline_network(depth))
net.prepare(device=0)
plan = net.plan()
f = dict(w.split("=", 1) for w in plan.split() if "=" in w)
out = torch.empty(n, dtype=torch.int32, device="cuda")
st = torch.empty(n, dtype=torch.uint8, device="cuda")
sh = torch.cuda.current_stream().cuda_stream
run = lambda: net.compute_device(n, out_ptr=out.data_ptr(), status_ptr=st.data_ptr(), gen_kind=N.MK_GEN_FULL,
                                 seed=1, stream=sh)
for _ in range(2):
    run()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(5):
    run()
e1.record()
torch.cuda.synchronize()
us = e0.elapsed_time(e1) / 5 * 1e3
print(f"depth {depth} lanes {n} shape {f.get('shape')} regs {f.get('regs')} slots {f.get('slots')}: "
      f"{us:.1f} us per launch, {n / us:.1f} lanes/us", flush=True)
