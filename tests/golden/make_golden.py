"""Regenerate tests/golden/*.json: seeded inputs and the oracle's outputs for
the five BASELINE configs plus the README known answer.

The reference (Go 1.14, un-vendored deps) cannot be built or run in this
environment, so these vectors are produced by the CPU oracle
(oracle/tis_oracle.c), whose pinning is documented in its header and in
DESIGN.md section 6.  They freeze that oracle against regressions and give
the GPU tiers a fixed target.  Run:  python tests/golden/make_golden.py
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

import misaka_net_amd as mk  # noqa: E402
from oracle import pyoracle as po  # noqa: E402

SEED = 0x4D49534B41
EDGE = [0, 1, -1, 2, -2, 5, 7, 2147483646, 2147483647, -2147483648, -2147483647, 4294967301, -4294967296,
        9223372036854775807, -9223372036854775808]

CASES = {
    "c1_example_readme": (mk.networks.example_network, EDGE, {}),
    "c2_example": (mk.networks.example_network, ("gen", 0, 0, 256), {}),
    "c3_sample": (mk.networks.sample_network, ("gen", 0, 0, 256), {}),
    "c3_sample_stop_on_output": (mk.networks.sample_network, ("gen", 0, 0, 64), {"stop_on_output": True}),
    "c4_pipeline_d64": (lambda: mk.networks.pipeline_network(64), ("gen", 0, 0, 32), {}),
    "c4_pipeline_d1024": (lambda: mk.networks.pipeline_network(1024), ("gen", 0, 0, 8), {}),
    "c4_pipeline_overflow": (lambda: mk.networks.pipeline_network(64), ("gen", 0, 0, 8), {"stack_cap": 63}),
    "c5_countdown": (mk.networks.countdown_network, ("gen", 1, 1023, 256), {}),
    "c5_countdown_budget": (mk.networks.countdown_network, ("gen", 1, 1023, 64), {"budget": 700}),
}


def rows(nodes):
    return [[n.name, n.kind, n.program] for n in nodes]


def main():
    for name, (factory, inputs, opts) in CASES.items():
        nodes = factory()
        if isinstance(inputs, tuple):
            _, kind, mask, n = inputs
            xs = po.gen_inputs(SEED, n, kind=kind, mask=mask).tolist()
        else:
            xs = list(inputs)
        out, st, sp = po.OracleNet(nodes).compute_batch(xs, **opts)
        rec = {
            "source": "oracle/tis_oracle.c (CPU restatement; see DESIGN.md section 6)",
            "network": rows(nodes),
            "options": opts,
            "inputs": xs,
            "out": out.tolist(),
            "status": st.tolist(),
            "steps": sp.tolist(),
        }
        with open(os.path.join(HERE, name + ".json"), "w") as f:
            json.dump(rec, f, separators=(",", ":"))
        print(name, len(xs))


if __name__ == "__main__":
    main()
