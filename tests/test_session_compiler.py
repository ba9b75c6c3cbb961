"""Stateful sessions compiled by the schedule compiler (row f2 on the native
tier; tis_sched.h compile_session_schedule), executed by the host model of
its device form (sched_check.cpp mkc_sess_*) and checked, call by call,
against the oracle's session restatement (tis_oracle.c session_step).

A call that would reach its budget slice inside a superblock is handed off
(U_HANDOFF): the host model exports the instance's state in the
interpreter's terms (sess_convert.h) and the oracle, importing it, must
finish that call and every later one exactly as the oracle's own run does.
CPU only."""
import numpy as np
import pytest

import misaka_net_amd as mk
from oracle import pyoracle as po
from schedcheck import HANDOFF, HostSessions, NotCompiled
from tisgen import random_network, stack_loop_network

CALLS = 6


def _nstack(nodes):
    return sum(1 for n in nodes if (n.kind if hasattr(n, "name") else n[1]) == "stack")


def run_pair(nodes, n, *, budget=None, stack_cap=None, seed=1, calls=CALLS, resumes=3, kind=0, mask=0):
    """Returns (calls checked, hand-offs seen)."""
    host = HostSessions(nodes, n, stack_cap=stack_cap)
    ref = po.OracleSessions(po.OracleNet(nodes), n, stack_cap=stack_cap)
    probes = {}  # lane -> (oracle instance finishing it, keep-alive)
    checked = handoffs = 0
    b = budget or (1 << 20)
    for k in range(calls):
        row = po.gen_inputs(seed * 7919 + k, n, kind=kind, mask=mask)
        ho, hs, hp = host.call(row, budget=b)
        ro, rs, rp = ref.compute(row, budget=b)
        for i in range(n):
            if i in probes:
                po_, _keep = probes[i]
                got = tuple(int(a[0]) for a in po_.compute([row[i]], budget=b))
            elif hs[i] == HANDOFF:
                flat, ent = host.export(i, _nstack(nodes))
                po_ = po.OracleSessions(po.OracleNet(nodes), 1, stack_cap=stack_cap)
                po_.import_state(0, flat)
                probes[i] = (po_, (flat, ent))
                got = tuple(int(a[0]) for a in po_.resume(budget=b))
                handoffs += 1
            else:
                got = (int(ho[i]), int(hs[i]), int(hp[i]))
            assert got == (int(ro[i]), int(rs[i]), int(rp[i])), (k, i, int(row[i]), got, (ro[i], rs[i], rp[i]))
            checked += 1
        # open calls (handed-off lanes only) get more slices, then are cancelled
        for _ in range(resumes):
            ro, rs, rp = ref.resume(budget=b)
            for i, (po_, _keep) in probes.items():
                got = tuple(int(a[0]) for a in po_.resume(budget=b))
                assert got == (int(ro[i]), int(rs[i]), int(rp[i])), ("resume", k, i, got)
            for i in range(n):
                if i not in probes:
                    assert rs[i] in (0, po.ST_STACK_OVERFLOW), ("a native lane left a call open", k, i)
        ref.cancel()
        for po_, _keep in probes.values():
            po_.cancel()
    return checked, handoffs


def test_example_network_sessions():
    nodes = mk.networks.example_network()
    host = HostSessions(nodes, 4)
    out, st, sp = host.call([5, 2147483647, -3, 4294967301])
    assert out.tolist() == [7, -2147483647, -1, 7] and (st == 0x10).all() and (sp == 11).all()
    out, st, sp = host.call([1, 2, 3, 4])
    assert out.tolist() == [3, 4, 5, 6] and (sp == 12).all()
    run_pair(nodes, 64)


@pytest.mark.parametrize("name", ["sample", "countdown", "pipeline8"])
def test_config_networks(name):
    nodes = {"sample": mk.networks.sample_network, "countdown": mk.networks.countdown_network,
             "pipeline8": lambda: mk.networks.pipeline_network(8)}[name]()
    kind, mask = (1, 1023) if name == "countdown" else (0, 0)
    run_pair(nodes, 48, kind=kind, mask=mask)
    # small budget slices: the long calls hand off and the oracle finishes them
    _, h = run_pair(nodes, 48, budget=60, kind=kind, mask=mask)
    if name == "countdown":
        assert h > 0


def test_state_that_persists():
    # running sum, second output returned by the next call, quiescent calls
    run_pair([("n", "program", "IN NIL\nADD 10\nOUT ACC")], 8)
    run_pair([("n", "program", "IN ACC\nOUT ACC\nOUT ACC")], 8)
    run_pair([("n", "program", "IN ACC\nJEZ Z\nOUT ACC\nZ: NOP")], 16, kind=1, mask=3)
    run_pair([("n", "program", "IN ACC\nPUSH ACC, s\nPOP s, ACC\nPUSH ACC, s\nOUT ACC"), ("s", "stack", "")], 8,
             stack_cap=3)


def test_long_call_hands_off_mid_loop():
    nodes = [("n", "program", "IN ACC\nL: SUB 1\nJGZ L\nOUT ACC")]
    host = HostSessions(nodes, 2)
    out, st, sp = host.call([3, 5000], budget=1000)
    assert st[0] == 0x10 and st[1] == HANDOFF
    checked, h = run_pair(nodes, 32, budget=500, kind=1, mask=1023)
    assert h > 0


@pytest.mark.parametrize("seed", range(150))
def test_random_networks(seed):
    nodes = random_network(seed)
    cap = [1, 3, 8, 16, 17, 40, 1024][seed % 7]
    try:
        run_pair(nodes, 24, budget=[37, 200, 1000, 5000][seed % 4], stack_cap=cap, seed=seed)
    except NotCompiled:
        pytest.skip("not compilable")


@pytest.mark.parametrize("seed", range(60))
def test_stack_loop_networks(seed):
    nodes, gen = stack_loop_network(seed)
    try:
        run_pair(nodes, 24, budget=[100, 2000, 6000][seed % 3], stack_cap=[16, 40, 1024][seed % 3], seed=seed,
                 kind=gen.get("kind", 0), mask=gen.get("mask", 0))
    except NotCompiled:
        pytest.skip("not compilable")
