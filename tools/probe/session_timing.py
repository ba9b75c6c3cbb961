"""Host-side cost of stateful session calls (mk_session_compute_device):
wall time per call with the caller's stream, with the session's own stream
(stream=None), and the kernel alone (HIP events around the launches)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import misaka_net_amd as mk  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
net = mk.Network(mk.networks.example_network())
sess = net.sessions(n)
x = torch.randint(-1000, 1000, (n,), dtype=torch.int64, device="cuda")
out = torch.empty(n, dtype=torch.int32, device="cuda")
st = torch.empty(n, dtype=torch.uint8, device="cuda")
sp = torch.empty(n, dtype=torch.int32, device="cuda")
cs = torch.cuda.current_stream()
for label, stream in (("caller stream", cs.cuda_stream), ("own stream", None)):
    sess.compute_device(x.data_ptr(), out.data_ptr(), st.data_ptr(), sp.data_ptr(), stream=stream)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(8):
        sess.compute_device(x.data_ptr(), out.data_ptr(), st.data_ptr(), sp.data_ptr(), stream=stream)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 8
    print(f"{label:14s} n={n}: {dt * 1e3:8.3f} ms per call (wall)", flush=True)
print("status 0x%x steps %d out %d" % (int(st[0]), int(sp[0]), int(out[0])))
