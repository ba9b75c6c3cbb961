"""Known answers of the oracle's stateful-session restatement (SURVEY.md
section 8 row f2): the reference keeps node state between /compute calls
(program.go:80-92) and the master's inChan / outChan are capacity-1
channels (master.go:58-59, 216-219).  Hand-derived from that code."""
import numpy as np

import misaka_net_amd as mk
from oracle import pyoracle as po

H, Q, B, OV, OPEN = po.ST_HAS_OUTPUT, po.ST_QUIESCENT, po.ST_BUDGET, po.ST_STACK_OVERFLOW, po.ST_CALL_OPEN

EX1 = "IN ACC\nADD 1\nMOV ACC, misaka2:R0\nMOV R0, ACC\nOUT ACC\n"
EX2 = "MOV R0, ACC\nADD 1\nPUSH ACC, misaka3\nPOP misaka3, ACC\nMOV ACC, misaka1:R0\n"
EXAMPLE = [("misaka1", "program", EX1), ("misaka2", "program", EX2), ("misaka3", "stack", ""),
           ("last_order", "master", "")]
COUNTDOWN = [("n", "program", "IN ACC\nL: SUB 1\nJGZ L\nOUT ACC")]


def calls(nodes, xs, **kw):
    s = po.OracleSessions(po.OracleNet(nodes), 1, stack_cap=kw.pop("stack_cap", None))
    return [tuple(int(a[0]) for a in s.compute([x], **kw)) for x in xs]


def test_example_network_every_call_returns_input_plus_two():
    # misaka1 loops back to IN ACC and blocks there until the next input
    got = calls(EXAMPLE, [5, 2147483647, -3, 4294967301])
    assert [g[0] for g in got] == [7, -2147483647, -1, 7]
    # the call ends at the round end after OUT: misaka1's trailing NOP (the
    # sixth, empty line) retires in the next call, so 11 steps, then 12 each
    assert [g[1] for g in got] == [H] * 4 and [g[2] for g in got] == [11, 12, 12, 12]


def test_state_persists_across_calls():
    # a running sum: ACC is never reset between calls
    got = calls([("n", "program", "IN NIL\nADD 10\nOUT ACC")], [0, 0, 0])
    assert [g[0] for g in got] == [10, 20, 30]


def test_second_output_is_returned_by_the_next_call():
    # two OUTs per input: call 2 returns the buffered second output of call 1,
    # call 3 the first output of input 2 (inChan held input 2 until IN took it)
    got = calls([("n", "program", "IN ACC\nOUT ACC\nOUT ACC")], [5, 7, 9])
    assert [g[0] for g in got] == [5, 5, 7]


def test_quiescent_call_leaves_the_instance_alive():
    # x = 0 takes the JEZ and never outputs: the call closes (the reference's
    # handler would block forever; the master answers 504) and the next input
    # runs on the same instance
    got = calls([("n", "program", "IN ACC\nJEZ Z\nOUT ACC\nZ: NOP")], [4, 0, 6])
    assert got[0][:2] == (4, H)
    assert got[1][:2] == (0, Q)
    assert got[2][:2] == (6, H)


def test_c3_zero_then_five():
    # the docs/sample.txt network (BASELINE config 3): zero has no output, and
    # the instance still doubles the next input
    got = calls(mk.networks.sample_network(), [0, 5, -7])
    assert [g[:2] for g in got] == [(0, Q), (10, H), (-14, H)]


def test_long_call_resumes_past_the_budget():
    # the reference's node loop never gives up
    # (program.go:80-92), so a /compute that needs more than one budget of
    # instructions still answers.  x = 3 * 2^20: IN, x times (SUB, JGZ), OUT.
    s = po.OracleSessions(po.OracleNet(COUNTDOWN), 1)
    x = 3 << 20
    out, st, sp = s.compute([x])
    assert st[0] == B and sp[0] >= 1 << 20
    # a new call while this one is open does nothing
    out, st, sp = s.compute([9])
    assert st[0] == OPEN and sp[0] == 0
    slices = 1
    while True:
        out, st, sp = s.resume()
        slices += 1
        if st[0] != B:
            break
    assert (int(out[0]), int(st[0])) == (0, H) and slices == 7
    assert int(sp[0]) == 2 * x + 2
    # nothing open any more: a resume reports nothing, the next call runs
    assert s.resume()[1][0] == 0
    assert [int(a[0]) for a in s.compute([3])[:2]] == [0, H]


def test_cancel_abandons_the_open_call():
    s = po.OracleSessions(po.OracleNet(COUNTDOWN), 1)
    assert s.compute([1000], budget=50)[1][0] == B
    s.cancel()
    # the abandoned call's input was deposited and taken by IN; its countdown
    # goes on, and its OUT is what the next call receives (outChan is the
    # master's, master.go:219)
    out, st, _ = s.compute([5], budget=5000)
    assert (int(out[0]), int(st[0])) == (0, H)
    # that call's own input 5 was deposited meanwhile and counts down next
    out, st, _ = s.compute([7], budget=5000)
    assert (int(out[0]), int(st[0])) == (0, H)


def test_budget_per_slice_and_reset():
    s = po.OracleSessions(po.OracleNet(COUNTDOWN), 2)
    out, st, sp = s.compute([3, 100], budget=50)
    assert st.tolist() == [H, B] and out[0] == 0 and sp[0] == 8
    out, st, sp = s.compute([2, 2], budget=50)
    assert st.tolist() == [H, OPEN] and sp[1] == 0
    out, st, sp = s.resume(budget=50)
    assert st.tolist() == [0, B] and sp[1] == 100
    out, st, sp = s.resume(budget=50)
    assert st.tolist() == [0, B] and sp[1] == 150
    out, st, sp = s.resume(budget=500)
    assert st.tolist() == [0, H] and out[1] == 0 and sp[1] == 202
    s.reset()
    out, st, _ = s.compute([1, 1], budget=50)
    assert st.tolist() == [H, H]


def test_stack_contents_persist_and_overflow():
    nodes = [("n", "program", "IN ACC\nPUSH ACC, s\nPOP s, ACC\nPUSH ACC, s\nOUT ACC"), ("s", "stack", "")]
    got = calls(nodes, [1, 2, 3], stack_cap=2)
    assert [g[0] for g in got[:2]] == [1, 2]
    assert got[2][1] == OV  # the third call's PUSH finds two entries left behind
    # stack_cap is ours (the reference's stacks are unbounded): an overflow
    # ends the session until reset
    s = po.OracleSessions(po.OracleNet(nodes), 1, stack_cap=2)
    for x in (1, 2, 3):
        s.compute([x])
    assert s.compute([4])[1][0] == OV
    s.reset()
    assert s.compute([4])[1][0] == H


def test_sessions_are_independent_and_threads_agree():
    nodes = [("n", "program", "IN ACC\nADD ACC\nOUT ACC\nSAV")]
    xs = po.gen_inputs(11, 3000).reshape(3, 1000)
    a = po.OracleSessions(po.OracleNet(nodes), 1000)
    b = po.OracleSessions(po.OracleNet(nodes), 1000)
    for row in xs:
        ra, rb = a.compute(row, threads=1), b.compute(row, threads=4)
        for u, v in zip(ra, rb):
            assert np.array_equal(u, v)
        assert np.array_equal(ra[0], (row.astype(np.int64) * 2).astype(np.int32))
