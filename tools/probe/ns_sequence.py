"""Round-4 probe: test_loop_phases_bit_exact's auto then machine-early-exit
variants as a plain script, compile only (`plan`) or compile and launch
(`run`), so that a crash can be placed in the compiler or the launches.

    python tools/probe/ns_sequence.py plan|run|orc [variants...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import torch  # noqa: E402

torch.cuda.init()
import numpy as np  # noqa: E402

import misaka_net_amd as mk  # noqa: E402
from oracle import pyoracle as po  # noqa: E402
from tisgen import loop_cases  # noqa: E402

ENVS = {
    "auto": {},
    "early": {"MK_JIT_SHAPE": "machine", "MK_JIT_POLICY": "8,12,16"},
    "pool64": {"MK_JIT_SHAPE": "machine", "MK_JIT_POOL": "64"},
    "k2": {"MK_JIT_SHAPE": "machine", "MK_JIT_POOL": "2"},
}
what = sys.argv[1]
for variant in sys.argv[2:] or ["auto", "early"]:
    for k in ("MK_JIT_SHAPE", "MK_JIT_POLICY", "MK_JIT_POOL"):
        os.environ.pop(k, None)
    os.environ.update(ENVS[variant])
    for label, nodes, xs, kw in loop_cases(n=4096):
        net = mk.Network(nodes)
        print(f"{variant} {label} compile", flush=True)
        p = net.plan()
        print(f"{variant} {label} {p.split('rtc=')[-1].split()[0] if 'rtc=' in p else p[:60]}", flush=True)
        if what in ("run", "orc"):
            r = net.compute_batch(np.asarray(xs, np.int64), **kw)
            print(f"{variant} {label} ran {int(r.steps.sum())}", flush=True)
        if what == "orc":  # the test's checker: the C oracle on 16 threads
            ref = po.OracleNet(nodes).compute_batch(np.asarray(xs, np.int64), threads=16, **kw)
            print(f"{variant} {label} oracle {'same' if np.array_equal(ref[2], r.steps) else 'DIFFERS'}", flush=True)
print("probe done", flush=True)
