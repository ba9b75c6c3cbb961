"""Known-answer tests of the oracle's restatement of the node runtime.

Pinning: README.md:39-44 (example network returns input + 2) is the only
in-tree known answer of the reference; every other case is hand-derived from
internal/nodes/program.go:219-566, stack.go:95-155, master.go:197-249 and Go
integer semantics (SURVEY.md section 8 row c).
"""
import numpy as np
import pytest

import misaka_net_amd as mk
from oracle import pyoracle as po

Q, B, OV, OS, H = po.ST_QUIESCENT, po.ST_BUDGET, po.ST_STACK_OVERFLOW, po.ST_OUTPUT_STOP, po.ST_HAS_OUTPUT

EX1 = "IN ACC\nADD 1\nMOV ACC, misaka2:R0\nMOV R0, ACC\nOUT ACC\n"
EX2 = "MOV R0, ACC\nADD 1\nPUSH ACC, misaka3\nPOP misaka3, ACC\nMOV ACC, misaka1:R0\n"
EXAMPLE = [("misaka1", "program", EX1), ("misaka2", "program", EX2), ("misaka3", "stack", ""),
           ("last_order", "master", "")]


def run(nodes, xs=(0,), **kw):
    out, st, sp = po.OracleNet(nodes).compute_batch(list(xs), **kw)
    return [(int(o), int(s), int(p)) for o, s, p in zip(out, st, sp)]


def one(program, x=0, **kw):
    return run([("n", "program", program), ("stk", "stack", ""), ("m", "master", "")], [x], **kw)[0]


def test_readme_example_network_returns_input_plus_two():
    # README.md:39-44; int32 wrap at the hops (program.go:498,516,561; master.go:237)
    got = run(EXAMPLE, [5, 0, -7, 2147483646, 2147483647, -2147483648, 4294967301, -4294967296])
    assert [g[0] for g in got] == [7, 2, -5, -2147483648, -2147483647, -2147483646, 7, 2]
    assert all(g[1] == Q | H and g[2] == 12 for g in got)


def test_acc_is_int64_with_wrap_and_out_truncates():
    assert one("MOV 9223372036854775807, ACC\nADD 1\nOUT ACC")[0] == 0  # MinInt64 -> int32 0
    assert one("MOV 9223372036854775807, ACC\nADD 1\nSUB 1\nOUT ACC")[0] == -1
    assert one("ADD 1073741824\nADD 1073741824\nOUT ACC")[0] == -2147483648
    assert one("IN ACC\nADD ACC\nOUT ACC", 2**31 - 1)[0] == -2  # ADD ACC doubles ACC
    assert one("OUT 4294967301")[0] == 5


def test_neg_minint64_stays_minint64():
    p = "MOV -9223372036854775808, ACC\nNEG\nJLZ OK\nOUT 0\nJMP E\nOK: OUT 1\nE: NOP"
    assert one(p)[0] == 1


def test_swp_sav():
    assert one("IN ACC\nSAV\nADD 5\nSWP\nOUT ACC\nSWP\nOUT ACC", 3)[0] == 3


def test_jro_clamps_without_wrap():
    assert one("JRO 100\nOUT 1\nOUT 2")[:2] == (2, Q | H)
    # JRO -5 from line 1 clamps to 0; IN then blocks (single input)
    assert one("IN ACC\nJRO -5\nOUT 9") == (0, Q, 2)
    # ptr + MaxInt64 wraps negative -> clamp to 0 (int64 wrapping add)
    assert one("IN NIL\nJRO 9223372036854775807\nOUT 1") == (0, Q, 2)
    assert one("IN ACC\nJRO ACC\nOUT 1\nOUT 2\nOUT 3", 2)[0] == 2
    assert one("IN ACC\nJRO ACC\nOUT 1\nOUT 2\nOUT 3", -2**31)[:2] == (0, Q)


def test_jro_zero_spins_until_budget():
    assert one("JRO 0", budget=10) == (0, B, 10)


def test_budget_checked_at_round_end():
    nodes = [("a", "program", "JRO 0"), ("b", "program", "JRO 0")]
    assert run(nodes, budget=11) == [(0, B, 12)]


def test_atoi_range_error_is_stuck():
    assert one("MOV 9223372036854775808, ACC\nOUT 1") == (0, Q, 0)
    assert one("OUT -9223372036854775809\nOUT 1") == (0, Q, 0)


def test_two_outs_complete_third_blocks():
    assert one("OUT 1\nOUT 2\nOUT 3\nOUT 4") == (1, Q | H, 2)


def test_second_in_blocks():
    assert one("IN ACC\nIN ACC\nOUT 5", 9) == (0, Q, 1)


def test_in_nil_discards():
    assert one("IN NIL\nOUT ACC", 9) == (0, Q | H, 2)


def test_stack_lifo_and_int32_push():
    assert one("PUSH 1, stk\nPUSH 2, stk\nPOP stk, ACC\nOUT ACC")[0] == 2
    assert one("PUSH 4294967297, stk\nPOP stk, ACC\nOUT ACC")[0] == 1
    assert one("MOV -2147483649, ACC\nPUSH ACC, stk\nPOP stk, ACC\nSUB 1\nOUT ACC")[0] == 2147483646


def test_pop_empty_blocks():
    assert one("POP stk, ACC\nOUT 1") == (0, Q, 0)


def test_stack_overflow_status():
    assert one("PUSH 1, stk\nPUSH 2, stk\nPUSH 3, stk\nOUT 1", stack_cap=2) == (0, OV, 2)


def test_stop_on_output():
    assert one("OUT 1\nOUT 2\nNOP", stop_on_output=True) == (1, OS | H, 1)


def test_port_capacity_one_and_pending_send():
    # a's second MOV finds b:R0 full and waits inside Send (pending) until b
    # drains it; "MOV R3, NIL" parks each node on an empty port at the end.
    a = "MOV 1, b:R0\nMOV 2, b:R0\nMOV 3, b:R0\nMOV R3, NIL"
    b = "NOP\nNOP\nMOV R0, ACC\nMOV R0, ACC\nADD R0\nOUT ACC\nMOV R3, NIL"
    assert run([("a", "program", a), ("b", "program", b)]) == [(5, Q | H, 9)]


def test_unknown_host_hangs_after_consuming_source():
    # ghost is not a node: grpc.Dial WithBlock never returns (program.go:72,492)
    a = "MOV R0, ghost:R1\n"
    b = "MOV 1, a:R0\nMOV 2, a:R0\nMOV 3, a:R0\nOUT 7\nMOV R3, NIL"
    # a consumes 1 then hangs; b deposits 2, blocks on 3 -> no output
    assert run([("a", "program", a), ("b", "program", b)]) == [(0, Q, 2)]


def test_wrong_service_retries_and_consumes():
    # Program.Send to a stack: Unimplemented, retried forever, each retry
    # re-reads R0 first (program.go:268-272, :80-92) -> b is never blocked
    a = "MOV R0, s:R1\n"
    b = "MOV 1, a:R0\nMOV 2, a:R0\nMOV 3, a:R0\nOUT 7\nMOV R3, NIL"
    assert run([("a", "program", a), ("b", "program", b), ("s", "stack", "")]) == [(7, Q | H, 4)]


def test_wrong_service_without_port_source_is_pure_stuck():
    assert one("PUSH 1, n\nOUT 1") == (0, Q, 0)  # n is a program node
    assert one("POP m, ACC\nOUT 1") == (0, Q, 0)  # m is the master
    assert one("MOV 1, stk:R0\nOUT 1") == (0, Q, 0)


def test_self_send():
    assert one("IN ACC\nMOV ACC, n:R2\nMOV R2, ACC\nADD 1\nOUT ACC", 41)[0] == 42


def test_schedule_is_sorted_by_name():
    # Two writers race for the first OUT; canonical schedule runs "a" first.
    nodes = [("b", "program", "OUT 2"), ("a", "program", "OUT 1")]
    assert run(nodes)[0][0] == 1


def test_batch_threads_agree():
    xs = po.gen_inputs(7, 2000)
    a = po.OracleNet(EXAMPLE).compute_batch(xs, threads=1)
    b = po.OracleNet(EXAMPLE).compute_batch(xs, threads=4)
    for u, v in zip(a, b):
        assert np.array_equal(u, v)


def test_generator_edges_every_16th_lane():
    xs = po.gen_inputs(0x4D49534B41, 64)
    edges = {-(2**31), -(2**31) + 1, -(2**31) + 2, -1, 0, 1, 2**31 - 2, 2**31 - 1}
    assert all(int(xs[i]) in edges for i in range(15, 64, 16))
    m = po.gen_inputs(0x4D49534B41, 1000, kind=1, mask=1023)
    assert m.min() >= 0 and m.max() <= 1023


def test_lane_trace_kat_example_network():
    # README.md:39-44 network, x = 5: misaka1 IN/ADD 1/MOV, misaka2 MOV/ADD 1/
    # PUSH/POP/MOV, misaka1 MOV R0/OUT, then both trailing NOPs: 12 retired
    # instructions in the canonical schedule; ACC after the last OUT is 7
    t, st = po.trace_lane(po.OracleNet(mk.networks.example_network()), 5)
    assert st == po.ST_HAS_OUTPUT | po.ST_QUIESCENT
    assert [(int(e["node"]), int(e["ip"])) for e in t] == [
        (0, 0), (0, 1), (0, 2), (1, 0), (1, 1), (1, 2), (1, 3), (1, 4), (0, 3), (1, 5), (0, 4), (0, 5)]
    assert [int(e["acc"]) for e in t] == [5, 6, 6, 6, 7, 7, 7, 7, 7, 7, 7, 7]
    assert [int(e["round"]) for e in t] == [0, 1, 2, 2, 3, 4, 5, 6, 7, 7, 8, 9]
    # the trace is bounded by max_entries; the status is still the lane's
    t2, st2 = po.trace_lane(po.OracleNet(mk.networks.example_network()), 5, max_entries=4)
    assert len(t2) == 4 and st2 == st
