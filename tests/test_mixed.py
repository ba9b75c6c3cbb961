"""Mixed deployments (misaka_net_amd.mixed): part
of a network on the GPU (one stateful session), the rest played by stand-in
reference nodes (oracle/refstruct.py: the reference's node loop, a fresh
gRPC channel per hop).  Program.Send / Stack.Push / Stack.Pop cross the
wire in both directions (messenger.proto:9-28); the answers of a sequence
of /compute calls equal the oracle's session restatement of the whole
network (tis_oracle.c session_call)."""
import numpy as np
import pytest

import misaka_net_amd as mk
from misaka_net_amd import _native as N
from oracle import pyoracle as po
from oracle import refstruct

M1, M2 = mk.networks.EXAMPLE_MISAKA1, mk.networks.EXAMPLE_MISAKA2


def test_remote_kinds_lower_to_remote_ops():
    # CPU: remote peers lower to XSEND / XPUSH / XPOP; wrong service types keep
    # the reference's retry semantics; the schedule compiler leaves such
    # networks to the interpreters
    net = mk.Network([("g", "program", "IN ACC\nMOV ACC, p:R2\nPUSH ACC, s\nPOP s, ACC\nPUSH 1, p\nOUT ACC"),
                      ("p", "remote_program", ""), ("s", "remote_stack", "")])
    d = net.disasm()
    assert "XSEND" in d and "arg=2" in d and "XPUSH" in d and "XPOP" in d and "RETRY" not in d
    assert "STUCK" in d  # PUSH of an immediate to a program node: Unimplemented, retried without effect
    assert net.plan().startswith("tier=interp reason=network addresses remote peers")


def _oracle_calls(nodes, xs):
    o = po.OracleSessions(po.OracleNet(nodes), 1)
    return [(int(a[0]), int(b[0])) for a, b, _ in (o.compute([x]) for x in xs)]


@pytest.mark.gpu
def test_gpu_node_and_stack_with_remote_program(gpu):
    # example network (docker-compose.yml): misaka1 and the stack misaka3 on
    # the GPU, misaka2 a reference node.  GPU -> peer: Program.Send (misaka1's
    # MOV ACC, misaka2:R0); peer -> GPU: Stack.Push / Stack.Pop on misaka3 and
    # Program.Send into misaka1:R0.  README.md:39-44: x + 2.
    from misaka_net_amd.mixed import MixedHost

    emu = refstruct.RefStructNet([("misaka2", "program", M2)])
    host = MixedHost([("misaka1", "program", M1), ("misaka3", "stack", ""), ("last_order", "master", ""),
                      ("misaka2", "remote_program", "")], {"misaka2": emu.addr["misaka2"]})
    emu.addr.update(misaka1=host.addresses["misaka1"], misaka3=host.addresses["misaka3"])
    try:
        xs = po.gen_inputs(0x4D49534B41, 12).tolist() + [5, 2147483647, -2147483648]
        got = []
        for x in xs:
            ok, v, st = host.compute(x, timeout=60)
            got.append((v, st))
            assert ok, (x, st)
        ref = _oracle_calls(mk.networks.example_network(), xs)
        assert [g[0] for g in got] == [r[0] for r in ref]
        assert all(st == N.MK_ST_HAS_OUTPUT for _, st in got) and all(r[1] == po.ST_HAS_OUTPUT for r in ref)
    finally:
        host.close()
        emu.close()


@pytest.mark.gpu
def test_gpu_node_with_remote_stack(gpu):
    # a GPU node pushing to and popping from a reference stack node
    # (Stack.Push / Stack.Pop from the GPU side, program.go:509-536): 2x - 6
    from misaka_net_amd.mixed import MixedHost

    prog = "IN ACC\nPUSH ACC, rs\nPUSH 7, rs\nSAV\nPOP rs, ACC\nPOP rs, NIL\nSWP\nSUB 3\nADD ACC\nOUT ACC"
    full = [("g", "program", prog), ("rs", "stack", "")]
    emu = refstruct.RefStructNet([("rs", "stack", "")])
    host = MixedHost([("g", "program", prog), ("rs", "remote_stack", "")], {"rs": emu.addr["rs"]})
    try:
        xs = [11, -4, 2147483647, 0, 99, -2147483648]
        got = [host.compute(x, timeout=60) for x in xs]
        ref = _oracle_calls(full, xs)
        assert [(int(v), int(st)) for ok, v, st in got] == ref
    finally:
        host.close()
        emu.close()


@pytest.mark.gpu
def test_remote_node_does_in_and_out(gpu):
    # a reference program node r does IN / OUT against the
    # GPU-backed master (Master.GetInput / SendOutput, master.go:233-249); g
    # and the stack s are GPU-resident.  Checked against the oracle's session
    # restatement of the whole network: 2x - 1 on int32 hops.
    from misaka_net_amd.mixed import MixedHost

    r_prog = "IN ACC\nMOV ACC, g:R0\nMOV R1, ACC\nOUT ACC"
    g_prog = "MOV R0, ACC\nADD ACC\nPUSH ACC, s\nPOP s, ACC\nSUB 1\nMOV ACC, r:R1"
    emu = refstruct.RefStructNet([("r", "program", r_prog)], start=False)
    host = MixedHost([("g", "program", g_prog), ("s", "stack", ""), ("boss", "master", ""),
                      ("r", "remote_program", "")], {"r": emu.addr["r"]})
    emu.addr.update(g=host.addresses["g"])
    emu.master_addr = host.addresses["boss"]
    emu.start()
    try:
        xs = [5, -4, 2147483647, 0, -2147483648] + po.gen_inputs(0x4D49534B41, 6).tolist()
        got = [host.compute(x, timeout=60) for x in xs]
        ref = _oracle_calls([("g", "program", g_prog), ("r", "program", r_prog), ("s", "stack", "")], xs)
        assert [(int(v), int(st)) for ok, v, st in got] == ref
        assert all(ok for ok, _, _ in got)
    finally:
        host.close()
        emu.close()


@pytest.mark.gpu
def test_timed_out_call_is_abandoned_and_calls_are_serialised(gpu):
    # a call that times out while parked on a peer must not be
    # resumed or overwritten by the next call, and concurrent compute() calls
    # must not interleave their steps.  x = 0 sends to the peer r, which never
    # reads that port, and outputs nothing: it parks until the timeout.
    import threading

    from misaka_net_amd.mixed import MixedHost

    g_prog = "S: IN ACC\nJEZ Z\nOUT ACC\nJMP S\nZ: MOV ACC, r:R0\nJMP S"
    emu = refstruct.RefStructNet([("r", "program", "MOV R1, ACC")])
    host = MixedHost([("g", "program", g_prog), ("r", "remote_program", "")], {"r": emu.addr["r"]})
    try:
        ok, v, st = host.compute(0, timeout=1.0)
        assert not ok and (st & N.MK_ST_REASON_MASK) == N.MK_ST_REMOTE_WAIT
        assert host.compute(7, timeout=30)[:2] == (True, 7)
        res = {}

        def client(i):
            res[i] = host.compute(100 + i, timeout=60)[:2]

        ts = [threading.Thread(target=client, args=(i,)) for i in range(8)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(120)
        assert res == {i: (True, 100 + i) for i in range(8)}
    finally:
        host.close()
        emu.close()


@pytest.mark.gpu
def test_budget_resume_in_a_mixed_deployment(gpu):
    # a long local countdown between two remote hops: the call outlives
    # several budget slices and still answers
    from misaka_net_amd.mixed import MixedHost

    g_prog = "IN ACC\nL: SUB 1\nJGZ L\nPUSH ACC, rs\nPOP rs, ACC\nADD 9\nOUT ACC"
    emu = refstruct.RefStructNet([("rs", "stack", "")])
    host = MixedHost([("g", "program", g_prog), ("rs", "remote_stack", "")], {"rs": emu.addr["rs"]}, budget=1000)
    try:
        assert host.compute(5000, timeout=60)[:2] == (True, 9)
        assert host.compute(3, timeout=60)[:2] == (True, 9)
    finally:
        host.close()
        emu.close()
