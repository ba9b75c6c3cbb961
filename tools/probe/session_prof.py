"""Stateful sessions under rocprofv3: n instances of a
network, K launches of one kind only, so that the kernel statistics and the
PMC passes describe that kind of launch alone.

    python tools/probe/session_prof.py percall|burst [n] [K] [calls] [network]

percall: K launches of mk_session_compute_device (one call per instance per
launch); burst: K launches of mk_session_compute_seq_device with `calls`
sequential calls per instance.  Prints the session plan and the host-clock
time per launch; the per-launch byte model is in tools/sess_roofline.py."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import misaka_net_amd as mk  # noqa: E402

mode = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 20
K = int(sys.argv[3]) if len(sys.argv) > 3 else 10
calls = int(sys.argv[4]) if len(sys.argv) > 4 else 8
torch.cuda.init()
net_name = sys.argv[5] if len(sys.argv) > 5 else "example"
net = mk.Network(getattr(mk.networks, net_name + "_network")())
sess = net.sessions(n)
sh = torch.cuda.current_stream().cuda_stream
x32 = torch.empty(calls * n, dtype=torch.int32, device="cuda")
mk.generate_inputs_device(calls * n, x32.data_ptr(), seed=0x4D49534B41, stream=sh)
if net_name == "countdown":  # C5's inputs: uniform in [0, 1023]
    x32 &= 1023
x = x32.to(torch.int64).view(calls, n)
out = torch.empty((calls, n), dtype=torch.int32, device="cuda")
st = torch.empty((calls, n), dtype=torch.uint8, device="cuda")
sp = torch.empty((calls, n), dtype=torch.int32, device="cuda")


def launch():
    if mode == "percall":
        sess.compute_device(x[0].data_ptr(), out[0].data_ptr(), st[0].data_ptr(), sp[0].data_ptr(), stream=sh)
    else:
        sess.compute_seq_device(x.data_ptr(), calls, out.data_ptr(), st.data_ptr(), sp.data_ptr(), stream=sh)


launch()  # module load, first touch
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(K):
    launch()
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / K
ncalls = 1 if mode == "percall" else calls
print(json.dumps({"mode": mode, "instances": n, "launches": K, "calls_per_launch": ncalls,
                  "us_per_launch": dt * 1e6, "us_per_call": dt * 1e6 / ncalls,
                  "steps_per_call": int(sp[:ncalls].to(torch.int64).sum()) / ncalls, "plan": sess.plan()}),
      flush=True)
sess.close()
