"""Diagnostic: how much of C4's deep-pipeline time is the pop loop's serial
accumulation.  Times the bench network (sum = 3*sum + v per pop) against the
same network with sum = sum + v (a one-add chain) at one depth.
  python tools/probe/chain_cost.py DEPTH LANES"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import misaka_net_amd as mk  # noqa: E402
from misaka_net_amd import _native as N  # noqa: E402
from misaka_net_amd.network import NodeSpec  # noqa: E402

depth, n = int(sys.argv[1]), int(sys.argv[2])


def network(kind):
    nodes = mk.networks.pipeline_network(depth)
    if kind == "add":  # drop the doubling and the R3 add: sum' = sum + v
        nodes = [NodeSpec(s.name, s.kind, s.program.replace("ADD ACC\nADD R3\n", "")) if s.kind == "program" else s
                 for s in nodes]
    return nodes


for kind in ("mul3", "add"):
    net = mk.Network(network(kind))
    net.prepare(device=0)
    plan = net.plan()
    f = dict(w.split("=", 1) for w in plan.split() if "=" in w)
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    st = torch.empty(n, dtype=torch.uint8, device="cuda")
    sh = torch.cuda.current_stream().cuda_stream
    run = lambda: net.compute_device(n, out_ptr=out.data_ptr(), status_ptr=st.data_ptr(), gen_kind=N.MK_GEN_FULL,  # noqa: E731
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
    print(f"{kind}: depth {depth} lanes {n} shape {f.get('shape')} regs {f.get('regs')} slots {f.get('slots')} "
          f"kernel {f.get('kernel')}: {us:.1f} us per launch", flush=True)
    net.close()
