"""The reference-structured CPU emulation (oracle/refstruct.py, bench.py's
cpu_baseline leg): one thread per node and a gRPC call per network hop, as
the reference runs (program.go:80-92, 475-566).  It must compute what the
oracle computes on determinate networks."""
import numpy as np
import pytest

import misaka_net_amd as mk
from oracle import pyoracle as po
from oracle import refstruct


@pytest.mark.parametrize("name,nodes,xs", [
    ("example", mk.networks.example_network(), [5, 2147483646, 2147483647, -2147483648, 0]),
    ("sample", mk.networks.sample_network(), [3, -4, 2147483647, 77]),
    ("countdown", mk.networks.countdown_network(), [0, 1, 2, 3, 100, 1023]),
    ("pipeline_d4", mk.networks.pipeline_network(4), [1, -7, 123456]),
])
def test_emulation_matches_oracle(name, nodes, xs):
    net = refstruct.RefStructNet(nodes, dial_per_hop=(name == "example"))
    try:
        got = [net.compute(x) for x in xs]
    finally:
        net.close()
    ref = po.OracleNet(nodes).compute_batch(np.asarray(xs, np.int64))
    assert (ref[1] & po.ST_HAS_OUTPUT).all()
    assert got == ref[0].tolist(), name


def test_time_compute_bounded():
    xs = po.gen_inputs(1, 64)
    r = refstruct.time_compute(mk.networks.example_network(), xs, seconds=1.0)
    assert r["results"] > 5 and r["results_per_s"] > 0
    exp = [((int(x) + 2 + 2**31) % 2**32) - 2**31 for x in xs]
    assert r["outputs"] == [exp[(i + 1) % len(xs)] for i in range(len(r["outputs"]))]
    # ~12 retired instructions per /compute (6 per node, README.md:39-44 network)
    assert 10 <= r["node_instr_per_s"] / r["results_per_s"] <= 14
