"""Diagnostic: launch time of the signed-pop network (tests/test_gpu_parity.py)
on HBM-resident inputs, for A/B runs of MK_JIT_PREFETCH / MK_JIT_HEAVY_OPS.
  python tools/probe/pops_timing.py DEPTH LANES"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402

import misaka_net_amd as mk  # noqa: E402
from misaka_net_amd import _native as N  # noqa: E402
from test_gpu_parity import signed_pop_network  # noqa: E402

depth, n = int(sys.argv[1]), int(sys.argv[2])
net = mk.Network(signed_pop_network(depth))
net.prepare(device=0)
print(net.plan(), flush=True)
out = torch.empty(n, dtype=torch.int32, device="cuda")
st = torch.empty(n, dtype=torch.uint8, device="cuda")
sh = torch.cuda.current_stream().cuda_stream
run = lambda: net.compute_device(n, out_ptr=out.data_ptr(), status_ptr=st.data_ptr(), gen_kind=N.MK_GEN_FULL,
                                 seed=1, stream=sh)
for _ in range(3):
    run()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(10):
    run()
e1.record()
torch.cuda.synchronize()
print(f"depth {depth} lanes {n}: {e0.elapsed_time(e1) / 10 * 1e3:.1f} us per launch", flush=True)
