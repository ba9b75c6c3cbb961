"""Launch time of one tests/tisgen.py random network on the native tier
(inputs from the device generator, resident in HBM), for A/B runs of
MK_JIT_* knobs.   python tools/probe/random_net_timing.py SEED [LANES] [LAUNCHES]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402

import misaka_net_amd as mk  # noqa: E402
from misaka_net_amd import _native as N  # noqa: E402
from tisgen import random_network  # noqa: E402

seed = int(sys.argv[1])
n = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 20
K = int(sys.argv[3]) if len(sys.argv) > 3 else 10
net = mk.Network(random_network(seed))
net.prepare(device=0)
out = torch.empty(n, dtype=torch.int32, device="cuda")
st = torch.empty(n, dtype=torch.uint8, device="cuda")
sp = torch.empty(n, dtype=torch.int32, device="cuda")
x = torch.empty(n, dtype=torch.int32, device="cuda")
sh = torch.cuda.current_stream().cuda_stream
mk.generate_inputs_device(n, x.data_ptr(), seed=seed, gen_kind=N.MK_GEN_MASKED, gen_mask=1023, stream=sh)
run = net.device_launcher(n, out_ptr=out.data_ptr(), status_ptr=st.data_ptr(), steps_ptr=sp.data_ptr(),
                          in_ptr=x.data_ptr(), in_kind=N.MK_IN_I32)
for _ in range(2):
    run(sh)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(K):
    run(sh)
e1.record()
torch.cuda.synchronize()
plan = net.plan()
print(json.dumps({"seed": seed, "lanes": n, "us_per_launch": round(e0.elapsed_time(e1) / K * 1e3, 2),
                  "instr_per_lane": int(sp.to(torch.int64).sum()) / n,
                  "kernel": plan.split("kernel=")[1].split()[0] if "kernel=" in plan else None,
                  "shape": plan.split("shape=")[1].split()[0] if "shape=" in plan else None}))
