"""Crash-at-exit probe (r03c-r03m): tests/test_gpu_parity.py's
test_dynamic_stack_networks_bit_exact for the native tier (mode auto), as a
plain script so that PyTorch is loaded only when asked (argv[1] == "torch"):
without it the process runs this ROCm's HIP runtime and hiprtc."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
if len(sys.argv) > 1 and sys.argv[1] == "torch":
    import torch  # noqa: F401  (PyTorch's bundled HIP runtime and hiprtc load first)

    torch.cuda.init()
import numpy as np  # noqa: E402

import misaka_net_amd as mk  # noqa: E402
from oracle import pyoracle as po  # noqa: E402
from tisgen import stack_loop_network  # noqa: E402

bad = 0
for seed in range(60):
    rows, gen = stack_loop_network(seed)
    xs = po.gen_inputs(seed + 5, 2048, **gen)
    kw = dict(budget=[None, 57, 300, 2000][seed % 4], stack_cap=[None, 3, 17, 64, 200][seed % 5])
    kw = {k: v for k, v in kw.items() if v is not None}
    got = mk.Network(rows).compute_batch(xs, **kw)
    ref = po.OracleNet(rows).compute_batch(xs, threads=16, **kw)
    ok = np.array_equal(got.out, ref[0]) and np.array_equal(got.status, ref[1]) and np.array_equal(got.steps, ref[2])
    bad += not ok
print(f"probe done: {60 - bad}/60 bit-exact, rtc={mk.Network(stack_loop_network(6)[0]).plan().split('rtc=')[1].split()[0]}",
      flush=True)
