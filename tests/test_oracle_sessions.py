"""Known answers of the oracle's stateful-session restatement (SURVEY.md
section 8 row f2): the reference keeps node state between /compute calls
(program.go:80-92) and the master's inChan / outChan are capacity-1
channels (master.go:58-59, 216-219).  Hand-derived from that code."""
import numpy as np

from oracle import pyoracle as po

H, Q, B, OV = po.ST_HAS_OUTPUT, po.ST_QUIESCENT, po.ST_BUDGET, po.ST_STACK_OVERFLOW

EX1 = "IN ACC\nADD 1\nMOV ACC, misaka2:R0\nMOV R0, ACC\nOUT ACC\n"
EX2 = "MOV R0, ACC\nADD 1\nPUSH ACC, misaka3\nPOP misaka3, ACC\nMOV ACC, misaka1:R0\n"
EXAMPLE = [("misaka1", "program", EX1), ("misaka2", "program", EX2), ("misaka3", "stack", ""),
           ("last_order", "master", "")]


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


def test_call_without_output_ends_the_session():
    got = calls([("n", "program", "IN ACC\nJEZ Z\nOUT ACC\nZ: NOP")], [4, 0, 6])
    assert got[0][:2] == (4, H)
    assert got[1][:2] == (0, Q)
    assert got[2] == (0, Q, 0)  # dead until reset


def test_budget_per_call_and_reset():
    nodes = [("n", "program", "IN ACC\nL: SUB 1\nJGZ L\nOUT ACC")]
    s = po.OracleSessions(po.OracleNet(nodes), 2)
    out, st, sp = s.compute([3, 100], budget=50)
    assert st.tolist() == [H, B] and out[0] == 0 and sp[0] == 8
    out, st, sp = s.compute([2, 2], budget=50)
    assert st.tolist() == [H, B] and sp[1] == 0
    s.reset()
    out, st, _ = s.compute([1, 1], budget=50)
    assert st.tolist() == [H, H]


def test_stack_contents_persist_and_overflow():
    nodes = [("n", "program", "IN ACC\nPUSH ACC, s\nPOP s, ACC\nPUSH ACC, s\nOUT ACC"), ("s", "stack", "")]
    got = calls(nodes, [1, 2, 3], stack_cap=2)
    assert [g[0] for g in got[:2]] == [1, 2]
    assert got[2][1] == OV  # the third call's PUSH finds two entries left behind


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
