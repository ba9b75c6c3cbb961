"""Diagnostic: C5 (countdown network) launch time and retired node-instructions
per lane against the input range, to split the kernel's time into a per-lane
fixed part (tile sort, dispatcher rounds, results) and the loops' part.
  python tools/probe/c5_decomp.py MASK [LANES] [LAUNCHES]
MASK: inputs uniform in [0, MASK] (bench.py's C5 uses 1023).  Run it under
`rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU ...` for the executed work, or
with MK_JIT_* knobs set for A/B runs."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import misaka_net_amd as mk  # noqa: E402
from misaka_net_amd import _native as N  # noqa: E402

mask = int(sys.argv[1])
n = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 22
K = int(sys.argv[3]) if len(sys.argv) > 3 else 10
net = mk.Network(mk.networks.countdown_network())
net.prepare(device=0)
plan = net.plan()
f = dict(w.split("=", 1) for w in plan.split() if "=" in w)
out = torch.empty(n, dtype=torch.int32, device="cuda")
st = torch.empty(n, dtype=torch.uint8, device="cuda")
sp = torch.empty(n, dtype=torch.int32, device="cuda")
sh = torch.cuda.current_stream().cuda_stream
x = torch.empty(n, dtype=torch.int32, device="cuda")  # inputs resident in HBM, as in bench.py
mk.generate_inputs_device(n, x.data_ptr(), seed=0x4D49534B41, gen_kind=N.MK_GEN_MASKED, gen_mask=mask, stream=sh)
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
us = e0.elapsed_time(e1) / K * 1e3
instr = int(sp.to(torch.int64).sum())
knobs = {k: v for k, v in os.environ.items() if k.startswith("MK_JIT_")}
prof = None
if os.environ.get("MK_JIT_PROF") == "1":
    # the kernel's per-wave phase cycles (kMachineSortKernel under MK_PROF), summed over waves
    stats = torch.zeros(N.MK_STATS_LEN, dtype=torch.int64, device="cuda")
    net.compute_device(n, out_ptr=out.data_ptr(), status_ptr=st.data_ptr(), stats_ptr=stats.data_ptr(),
                       in_ptr=x.data_ptr(), in_kind=N.MK_IN_I32, stream=sh)
    torch.cuda.synchronize()
    v = [int(x) for x in stats.cpu()]
    names = ["total", "sort", "chunks", "run_loop", "run_other", "results", "rounds", "loop_rounds"]
    prof = dict(zip(names, v))
    tot = max(1, v[0])
    prof["frac"] = {k: round(prof[k] / tot, 4) for k in names[1:6]}
    prof["dispatch_other"] = round((v[2] - v[3] - v[4]) / tot, 4)  # chunk time outside mk_run

print(json.dumps({"mask": mask, "lanes": n, "us_per_launch": round(us, 2), "instr_per_lane": instr / n,
                  "ns_per_lane": us * 1e3 / n, "tinstr_per_s": instr / us / 1e6, "kernel": f.get("kernel"),
                  "knobs": knobs, "prof": prof}), flush=True)
