"""Diagnostic: the signed-pop network (tests/test_gpu_parity.py) on the
machine shape, with and without pipelined pops (MK_JIT_PREFETCH), vs the
oracle.  Run each setting in its own process under a timeout."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402

import misaka_net_amd as mk  # noqa: E402
from oracle import pyoracle as po  # noqa: E402
from test_gpu_parity import signed_pop_network  # noqa: E402

depth = int(sys.argv[1]) if len(sys.argv) > 1 else 300
n = int(sys.argv[2]) if len(sys.argv) > 2 else 777
nodes = signed_pop_network(depth)
net = mk.Network(nodes)
print("plan", net.plan(), flush=True)
xs = po.gen_inputs(0x4D49534B41 + 3, n)
t = time.time()
net.prepare(device=0)
print("prepared", time.time() - t, flush=True)
r = net.compute_batch(xs)
print("computed", time.time() - t, flush=True)
ref = po.OracleNet(nodes).compute_batch(xs)
bad = np.nonzero((r.out != ref[0]) | (r.status != ref[1]) | (r.steps != ref[2]))[0]
print("bad lanes", bad.size, flush=True)
