"""HTTP master surface (misaka_net_amd.master)
against master.go:90-249: routes, methods, status codes and error texts.
The compute paths run on the GPU (marked)."""
import http.client
import json
import threading
import time

import pytest

import misaka_net_amd as mk
from misaka_net_amd import _native as N
from misaka_net_amd.master import Coalescer, MasterNode, go_atoi, make_server, parse_query

NODE_INFO = {"misaka1": {"type": "program"}, "misaka2": {"type": "program"}, "misaka3": {"type": "stack"}}
PROGRAMS = {"misaka1": mk.networks.EXAMPLE_MISAKA1, "misaka2": mk.networks.EXAMPLE_MISAKA2}
FORM = "application/x-www-form-urlencoded"


def master():
    return MasterNode(NODE_INFO, PROGRAMS, name="last_order")


@pytest.mark.parametrize("path", ["/run", "/pause", "/reset", "/load", "/compute"])
def test_non_post_is_405(path):
    r = master().handle("GET", path)
    assert (r.code, r.body) == (405, "method GET not allowed\n")


def test_compute_requires_running():
    r = master().handle("POST", "/compute", body=b"value=5", ctype=FORM)
    assert (r.code, r.body) == (400, "network is not running\n")


@pytest.mark.parametrize("value", ["", "abc", "1.5", " 5", "0x10", "9223372036854775808", "1_0"])
def test_compute_cannot_parse_value(value):
    m = master()
    assert m.handle("POST", "/run").body == "Success"
    r = m.handle("POST", "/compute", body=f"value={value}".encode(), ctype=FORM)
    assert (r.code, r.body) == (400, "cannot parse value\n")


def test_cannot_parse_form():
    m = master()
    m.handle("POST", "/run")
    r = m.handle("POST", "/compute", body=b"value=%zz", ctype=FORM)
    assert (r.code, r.body) == (400, "cannot parse form\n")
    r = m.handle("POST", "/load", body=b"program=%4", ctype=FORM)
    assert (r.code, r.body) == (400, "cannot parse form\n")


def test_load_unknown_node():
    r = master().handle("POST", "/load", body=b"program=NOP&targetURI=nope", ctype=FORM)
    assert (r.code, r.body) == (400, "error loading program on node nope: node nope not valid on this network\n")


def test_load_parse_error_keeps_program_and_resets():
    m = master()
    m.handle("POST", "/run")
    r = m.handle("POST", "/load", body=b"program=MOV+1%2CACC&targetURI=misaka1", ctype=FORM)
    assert r.code == 400
    assert r.body == "error loading program on node misaka1: line 0, 'MOV 1,ACC' not a valid instruction\n"
    assert m.programs["misaka1"] == PROGRAMS["misaka1"]
    assert not m.is_running  # /load resets the network first


def test_load_success_and_run_pause_reset():
    m = master()
    r = m.handle("POST", "/load", body=b"program=IN+ACC%0AOUT+ACC&targetURI=misaka1", ctype=FORM)
    assert (r.code, r.body) == (200, "Success")
    assert m.programs["misaka1"] == "IN ACC\nOUT ACC"
    for path in ("/run", "/pause", "/reset"):
        assert m.handle("POST", path).body == "Success"
    assert not m.is_running


class _FakeSession:
    def __init__(self):
        self.closed = False

    def close(self):
        self.closed = True


class _FakeWire:
    def __init__(self):
        self.resets = 0

    def reset(self):
        self.resets += 1

    def cancel(self):
        pass


@pytest.mark.parametrize("program,code", [(b"program=MOV+1%2CACC", 400), (b"program=NOP", 200)])
def test_load_resets_state_even_when_rejected(program, code):
    # master.go:165-175 resets every node and the master's channels before the
    # Load RPC, so a rejected program still leaves a reset network
    m = master()
    m.handle("POST", "/run")
    sess = m._sess = _FakeSession()
    m.wire = _FakeWire()
    r = m.handle("POST", "/load", body=program + b"&targetURI=misaka1", ctype=FORM)
    assert r.code == code
    assert sess.closed and m._sess is None and m.wire.resets == 1 and not m.is_running
    # a stack target is rejected after the reset too
    m._sess = sess2 = _FakeSession()
    assert m.handle("POST", "/load", body=b"program=NOP&targetURI=misaka3", ctype=FORM).code == 400
    assert sess2.closed and m.wire.resets == 2


def test_default_is_stateful():
    assert master().stateful  # the reference's semantics (program.go:80-92)


def test_coalescer_routes_results_in_arrival_order():
    seen = []
    gate = threading.Event()

    def run(vals):
        gate.wait(5)
        seen.append(list(vals))
        return [(True, v * 10) for v in vals]

    c = Coalescer(run)
    out = {}

    def client(i):
        out[i] = c.submit(i)

    ts = [threading.Thread(target=client, args=(i,)) for i in range(64)]
    for t in ts:
        t.start()
        time.sleep(0.002)  # arrival order = i
    gate.set()
    for t in ts:
        t.join(10)
    assert out == {i: (True, 10 * i) for i in range(64)}
    assert sum(map(len, seen)) == 64 and c.requests == 64
    assert c.batches < 64  # requests that arrived during a launch shared the next one
    flat = [v for b in seen for v in b]
    assert flat == sorted(flat)  # each batch keeps arrival order, batches in order


def test_coalescer_delivers_errors_to_the_batch():
    c = Coalescer(lambda vals: 1 / 0)
    with pytest.raises(ZeroDivisionError):
        c.submit(1)
    c2 = Coalescer(lambda vals: [(True, v) for v in vals], max_batch=3)
    assert [c2.submit(i) for i in range(5)] == [(True, i) for i in range(5)]


def test_boot_program_error_keeps_default_nop():
    m = MasterNode(NODE_INFO, {"misaka1": "bad instr", "misaka2": "NOP"})
    assert m.programs["misaka1"] == ""  # cmd/app.go:21-24 logs and keeps [["NOP"]]


def test_invalid_node_type():
    m = MasterNode({"a": {"type": "router"}}, {})
    r = m.handle("POST", "/run")
    assert (r.code, r.body) == (400, "error running network: invalid node type\n")


def test_go_helpers():
    assert go_atoi("+7") == 7 and go_atoi("-0") == 0 and go_atoi("9223372036854775807") == 2**63 - 1
    assert parse_query("a=1;b=2&a=%41+B") == {"a": ["1", "A B"], "b": ["2"]}


# ---- GPU: compute through a real HTTP server ---------------------------------

@pytest.fixture
def server(gpu):
    m = master()
    srv = make_server(m, port=0)
    t = threading.Thread(target=srv.serve_forever, daemon=True)
    t.start()
    yield srv.server_address[1]
    srv.shutdown()


def post(port, path, body="", ctype=FORM):
    c = http.client.HTTPConnection("127.0.0.1", port, timeout=60)
    c.request("POST", path, body=body, headers={"Content-Type": ctype})
    r = c.getresponse()
    return r.status, r.getheader("Content-Type"), r.read().decode()


@pytest.mark.gpu
def test_http_compute_example(server):
    assert post(server, "/run") == (200, "text/plain; charset=utf-8", "Success")
    # Go's json.Encoder: compact, newline-terminated (master.go:219)
    assert post(server, "/compute", "value=5") == (200, "application/json", '{"value":7}\n')
    assert post(server, "/compute", "value=4294967301")[2] == '{"value":7}\n'  # int32(v), master.go:237
    assert post(server, "/compute", "value=2147483647")[2] == '{"value":-2147483647}\n'


@pytest.mark.gpu
def test_http_compute_batch_and_load(server):
    post(server, "/run")
    st, ct, body = post(server, "/compute_batch", "value=1&value=-3&value=2147483646")
    assert st == 200 and json.loads(body)["values"] == [3, -1, -2147483648]
    st, _, body = post(server, "/compute_batch", json.dumps({"values": list(range(1000))}), "application/json")
    assert json.loads(body)["values"] == [v + 2 for v in range(1000)]
    # a program that never outputs: the reference hangs; we answer 504
    assert post(server, "/load", "program=IN+ACC&targetURI=misaka1")[0] == 200
    post(server, "/run")
    assert post(server, "/compute", "value=1")[:1] == (504,)


@pytest.mark.gpu
def test_stateful_master_keeps_node_state(gpu):
    # row f2: a running sum survives between /compute calls, /pause keeps it,
    # /reset clears it (program.go:80-92, 207-216; master.go:126-143)
    m = MasterNode({"acc": {"type": "program"}}, {"acc": "IN NIL\nADD 10\nOUT ACC"}, stateful=True)
    m.handle("POST", "/run")
    vals = [m.handle("POST", "/compute", body=b"value=0", ctype=FORM).body for _ in range(3)]
    assert vals == ['{"value":10}\n', '{"value":20}\n', '{"value":30}\n']
    m.handle("POST", "/pause")
    assert m.handle("POST", "/compute", body=b"value=0", ctype=FORM).code == 400
    m.handle("POST", "/run")
    assert m.handle("POST", "/compute", body=b"value=0", ctype=FORM).body == '{"value":40}\n'
    m.handle("POST", "/reset")
    m.handle("POST", "/run")
    assert m.handle("POST", "/compute", body=b"value=0", ctype=FORM).body == '{"value":10}\n'
    r = m.handle("POST", "/compute_batch", body=b"value=0&value=0", ctype=FORM)
    assert json.loads(r.body)["values"] == [20, 30]
    # the example network is stateless in effect: x + 2 on every call
    e = MasterNode(NODE_INFO, PROGRAMS, stateful=True)
    e.handle("POST", "/run")
    assert [e.handle("POST", "/compute", body=f"value={x}".encode(), ctype=FORM).body for x in (5, 6)] == \
        ['{"value":7}\n', '{"value":8}\n']


def _concurrent(port, path_vals, n_threads):
    """n_threads clients released together; returns {i: (status, body)}."""
    res = {}
    bar = threading.Barrier(n_threads)

    def client(i):
        bar.wait(10)
        st, _, body = post(port, "/compute", f"value={path_vals(i)}")
        res[i] = (st, body)

    ts = [threading.Thread(target=client, args=(i,)) for i in range(n_threads)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(60)
    return res


@pytest.mark.gpu
@pytest.mark.parametrize("stateful", [True, False])
def test_http_64_concurrent_clients(gpu, stateful):
    m = MasterNode(NODE_INFO, PROGRAMS, stateful=stateful)
    srv = make_server(m, port=0)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    port = srv.server_address[1]
    try:
        post(port, "/run")
        res = _concurrent(port, lambda i: 1000 * i - 7, 64)
        assert {i: r for i, r in res.items()} == {i: (200, f'{{"value":{1000 * i - 5}}}\n') for i in range(64)}
        assert m.coalescer.requests == 64 and m.coalescer.batches <= 64
    finally:
        srv.shutdown()


@pytest.mark.gpu
def test_http_concurrent_stateful_running_sum(gpu):
    # 64 concurrent /compute on one persistent instance: the calls are
    # serialised (the reference's capacity-1 inChan/outChan), so the answers
    # are exactly 10, 20, ..., 640 in some order
    m = MasterNode({"acc": {"type": "program"}}, {"acc": "IN NIL\nADD 10\nOUT ACC"})
    srv = make_server(m, port=0)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    port = srv.server_address[1]
    try:
        post(port, "/run")
        res = _concurrent(port, lambda i: 0, 64)
        vals = sorted(json.loads(b)["value"] for st, b in res.values())
        assert vals == [10 * (k + 1) for k in range(64)]
        assert m.coalescer.batches < 64  # bursts shared launches
    finally:
        srv.shutdown()


def test_http_server_takes_bursts_of_clients():
    # 64 clients connecting at once (the listen backlog must hold them; the
    # executor is replaced by a fake so this runs without a GPU)
    m = master()
    m.coalescer._run = lambda vals: [(True, v + 2) for v in vals]
    srv = make_server(m, port=0)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    port = srv.server_address[1]
    try:
        post(port, "/run")
        res = _concurrent(port, lambda i: i, 64)
        assert res == {i: (200, f'{{"value":{i + 2}}}\n') for i in range(64)}
        assert m.coalescer.requests == 64
    finally:
        srv.shutdown()


# ---- stateful calls that outlive the budget, and calls without output -------
# (VERDICT r02 item 1).  The reference's node loop never gives up
# (program.go:80-92) and its /compute handler waits for the output
# (master.go:216-219): a call that spends its budget slice stays open and is
# resumed; a call that can never output closes and the instance lives on.

COUNTDOWN = {"n": "IN ACC\nL: SUB 1\nJGZ L\nOUT ACC"}
# a answers x != 0 at once; x = 0 goes to b, which spins forever and never
# reads it: that call neither outputs nor goes quiescent
SPINNER = {"a": "S: IN ACC\nJEZ Z\nOUT ACC\nJMP S\nZ: MOV ACC, b:R0\nJMP S", "b": "L: JMP L"}


class _OracleSession:
    """SessionSet's call interface over the oracle's session restatement
    (tis_oracle.c session_step), so the master's call loop runs on CPU."""

    def __init__(self, programs, budget=None):
        from oracle import pyoracle as po

        self.o = po.OracleSessions(po.OracleNet([(k, "program", v) for k, v in programs.items()]), 1)
        self.budget, self.launches, self.closed = budget, 0, False

    def _res(self, rows):
        from misaka_net_amd.network import BatchResult
        import numpy as np

        return BatchResult(np.array([r[0] for r in rows], np.int32), np.array([r[1] for r in rows], np.uint8), None)

    def compute_seq(self, vals, steps=False, busy_ok=False):
        self.launches += 1
        rows = []
        for v in vals.tolist():
            o, st, _ = self.o.compute([v], budget=self.budget)
            rows.append((int(o[0]), int(st[0])))
        return self._res(rows)

    def resume(self, steps=False):
        self.launches += 1
        o, st, _ = self.o.resume(budget=self.budget)
        return self._res([(int(o[0]), int(st[0]))])

    def cancel(self):
        self.o.cancel()

    def reset(self):
        self.resets = getattr(self, "resets", 0) + 1
        self.o.reset()

    def close(self):
        self.closed = True


def _stateful(programs, sess_budget=None, **kw):
    m = MasterNode({k: {"type": "program"} for k in programs}, programs, **kw)
    m._sess = _OracleSession(programs, sess_budget)
    m.handle("POST", "/run")
    return m


def _compute(m, x):
    r = m.handle("POST", "/compute", body=f"value={x}".encode(), ctype=FORM)
    return r.code, r.body


def test_long_call_is_resumed_not_dropped():
    m = _stateful(COUNTDOWN)
    assert _compute(m, 3 << 20) == (200, '{"value":0}\n')  # 6.3M instructions, 7 budget slices
    assert m._sess.launches == 7
    assert _compute(m, 4) == (200, '{"value":0}\n')


def test_long_call_in_a_burst_keeps_the_order():
    # the burst's calls behind the long one did not run (MK_ST_CALL_OPEN) and
    # go in the next launch, in order
    m = _stateful({"n": "IN ACC\nL: SUB 1\nJGZ L\nADD 7\nOUT ACC"}, sess_budget=100)
    assert m._run_batch([3, 500, 2, 1]) == [(True, 7)] * 4
    r = m.handle("POST", "/compute_batch", body=b"value=400&value=0", ctype=FORM)
    assert json.loads(r.body) == {"values": [7, 6], "status": [0x10, 0x10]}  # 0 - 1 + 7


def test_quiescent_call_then_next_input():
    # BASELINE config 3's network: zero has no output (504 at once, the
    # instance lives on), then 5 doubles
    progs = {s.name: s.program for s in mk.networks.sample_network() if s.kind == "program"}
    m = _stateful(progs, name="master")
    assert _compute(m, 0) == (504, "network produced no output\n")
    assert _compute(m, 5) == (200, '{"value":10}\n')


def test_call_timeout_abandons_the_call():
    m = _stateful(SPINNER, sess_budget=1000, call_timeout=0.2)
    t0 = time.monotonic()
    assert _compute(m, 0) == (504, "network produced no output\n")
    assert time.monotonic() - t0 >= 0.2
    assert _compute(m, 5) == (200, '{"value":5}\n')  # the abandoned call left its 0 with b
    assert m._sess.launches > 3


def _spin_in_thread(m, x):
    box = {}
    t = threading.Thread(target=lambda: box.update(r=_compute(m, x)), daemon=True)
    t.start()
    time.sleep(0.15)  # the call is being resumed slice after slice
    assert t.is_alive()
    return t, box


def test_reset_during_a_spinning_call_returns_at_once():
    # a call being resumed holds the executor one slice at a
    # time, so /reset does not wait for it; the call stops at its next slice
    # (504) and the instance restarts from its initial state (kept compiled:
    # mk_session_reset, not a new session)
    m = _stateful(SPINNER, sess_budget=1000, call_timeout=None)
    sess = m._sess
    t, box = _spin_in_thread(m, 0)
    t0 = time.monotonic()
    assert m.handle("POST", "/reset").code == 200
    assert time.monotonic() - t0 < 0.5
    t.join(timeout=5)
    assert not t.is_alive() and box["r"] == (504, "network produced no output\n")
    assert m._sess is sess and sess.resets == 1 and not sess.closed
    m.handle("POST", "/run")
    assert _compute(m, 5) == (200, '{"value":5}\n')
    # b's port is empty again after /reset: a zero goes in, a later 5 answers
    assert m._run_batch([7]) == [(True, 7)]


class _GateSession:
    """A call that stays open (MK_ST_BUDGET each slice) until `gate` is set,
    then answers 42: the master's resume loop without an executor."""

    def __init__(self):
        self.gate, self.launches, self.cancels = threading.Event(), 0, 0

    def _res(self, o, st):
        from misaka_net_amd.network import BatchResult
        import numpy as np

        return BatchResult(np.array([o], np.int32), np.array([st], np.uint8), None)

    def compute_seq(self, vals, steps=False, busy_ok=False):
        self.launches += 1
        return self._res(0, N.MK_ST_BUDGET)

    def resume(self, steps=False):
        self.launches += 1
        return self._res(42, N.MK_ST_HAS_OUTPUT | N.MK_ST_QUIESCENT) if self.gate.is_set() else \
            self._res(0, N.MK_ST_BUDGET)

    def cancel(self):
        self.cancels += 1

    def reset(self):
        pass

    def close(self):
        pass


def test_pause_keeps_a_call_open_until_run():
    # the reference's /compute handler stays blocked on outChan while the
    # nodes are paused and answers once /run resumes them (master.go:216-219,
    # program.go:80-92): no slice runs while paused, the call is not cancelled
    m = _stateful(SPINNER, call_timeout=None)
    g = m._sess = _GateSession()
    t, box = _spin_in_thread(m, 0)
    t0 = time.monotonic()
    assert m.handle("POST", "/pause").code == 200
    assert time.monotonic() - t0 < 0.5
    time.sleep(0.1)
    n = g.launches
    time.sleep(0.3)
    assert g.launches == n and t.is_alive() and g.cancels == 0  # waiting, open
    assert _compute(m, 5) == (400, "network is not running\n")  # new calls: master.go:200-202
    g.gate.set()
    m.handle("POST", "/run")
    t.join(timeout=5)
    assert box["r"] == (200, '{"value":42}\n')


def test_pause_then_reset_ends_the_open_call():
    m = _stateful(SPINNER, call_timeout=None)
    m._sess = _GateSession()
    t, box = _spin_in_thread(m, 0)
    m.handle("POST", "/pause")
    time.sleep(0.1)
    assert t.is_alive()
    assert m.handle("POST", "/reset").code == 200
    t.join(timeout=5)
    assert not t.is_alive() and box["r"] == (504, "network produced no output\n")


def test_call_timeout_runs_while_paused():
    m = _stateful(SPINNER, call_timeout=0.3)
    g = m._sess = _GateSession()
    t, box = _spin_in_thread(m, 0)
    m.handle("POST", "/pause")
    t.join(timeout=5)
    assert box["r"] == (504, "network produced no output\n") and g.cancels == 1


class _FakeNet:
    """Network stand-in for the /load race: a session built on a
    closed network, or used after its network closed, is the use-after-free
    the native handles would suffer."""
    errors: list = []

    def __init__(self, specs):
        self.tag = {s.name: s.program for s in specs}.get("p", "")
        self.closed = False

    def sessions(self, n, **kw):
        if self.closed:
            _FakeNet.errors.append("session built on a closed network")
        return _FakeSess(self)

    def close(self):
        self.closed = True


class _FakeSess:
    def __init__(self, net):
        self.net, self.live = net, True

    def compute_seq(self, vals, steps=False, busy_ok=False):
        from misaka_net_amd.network import BatchResult
        import numpy as np

        if self.net.closed or not self.live:
            _FakeNet.errors.append("session used after its network closed")
        time.sleep(0.0005)  # a launch
        v = int(self.net.tag.split()[1])  # "OUT <k>"
        return BatchResult(np.full(len(vals), v, np.int32),
                           np.full(len(vals), N.MK_ST_HAS_OUTPUT | N.MK_ST_QUIESCENT, np.uint8), None)

    def reset(self):
        pass

    def close(self):
        self.live = False


def test_load_during_stateful_bursts_never_uses_the_old_network(monkeypatch):
    # /compute bursts from 8 threads while /load replaces the program 40
    # times: no session is built on, or runs after, a network that /load
    # closed; once /load (+ /run) returned, every call answers the new program
    from misaka_net_amd import master as M

    monkeypatch.setattr(M, "Network", _FakeNet)
    _FakeNet.errors = []
    m = MasterNode({"p": {"type": "program"}}, {"p": "OUT 0"})
    m.handle("POST", "/run")
    stop = threading.Event()
    seen = []

    def client():
        while not stop.is_set():
            r = m.handle("POST", "/compute", body=b"value=1", ctype=FORM)
            if r.code == 200:
                seen.append(json.loads(r.body)["value"])

    ts = [threading.Thread(target=client, daemon=True) for _ in range(8)]
    for t in ts:
        t.start()
    for k in range(1, 41):
        assert m.handle("POST", "/load", body=f"program=OUT+{k}&targetURI=p".encode(), ctype=FORM).code == 200
        m.handle("POST", "/run")
        r = m.handle("POST", "/compute", body=b"value=1", ctype=FORM)
        assert r.code == 200 and json.loads(r.body)["value"] == k, (k, r.body)
    stop.set()
    for t in ts:
        t.join(10)
    assert not _FakeNet.errors, _FakeNet.errors[:3]
    assert len(seen) > 40


def test_one_deadline_for_the_whole_burst():
    # three calls that never answer: the burst ends at call_timeout, not
    # three times it
    m = _stateful(SPINNER, sess_budget=1000, call_timeout=0.3)
    t0 = time.monotonic()
    got = m._run_batch([0, 0, 0])
    dt = time.monotonic() - t0
    assert got == [(False, 0)] * 3
    assert 0.3 <= dt < 0.6, dt


@pytest.mark.gpu
def test_http_long_call_on_the_gpu(gpu):
    # the same through a real server and the GPU session kernel (default
    # budget 2^20 per slice)
    m = MasterNode({"n": {"type": "program"}}, COUNTDOWN)
    srv = make_server(m, port=0)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    port = srv.server_address[1]
    try:
        post(port, "/run")
        assert post(port, "/compute", f"value={3 << 20}")[::2] == (200, '{"value":0}\n')
        assert post(port, "/compute", "value=9")[::2] == (200, '{"value":0}\n')
    finally:
        srv.shutdown()


@pytest.mark.gpu
def test_http_c3_zero_then_five(gpu):
    nodes = mk.networks.sample_network()
    m = MasterNode({s.name: {"type": s.kind} for s in nodes if s.kind != "master"},
                   {s.name: s.program for s in nodes if s.kind == "program"}, name="master")
    srv = make_server(m, port=0)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    port = srv.server_address[1]
    try:
        post(port, "/run")
        assert post(port, "/compute", "value=0")[::2] == (504, "network produced no output\n")
        assert post(port, "/compute", "value=5")[::2] == (200, '{"value":10}\n')
        assert post(port, "/compute", "value=-3")[::2] == (200, '{"value":-6}\n')
    finally:
        srv.shutdown()


@pytest.mark.gpu
def test_gpu_load_during_concurrent_compute(gpu):
    # ADVICE r04 on the executor: /compute from 4 threads while /load swaps
    # the program 6 times; after each /load + /run the new program answers
    m = MasterNode({"p": {"type": "program"}}, {"p": "IN ACC\nADD 0\nOUT ACC"})
    m.handle("POST", "/run")
    stop = threading.Event()
    codes = []

    def client():
        while not stop.is_set():
            codes.append(m.handle("POST", "/compute", body=b"value=1", ctype=FORM).code)

    ts = [threading.Thread(target=client, daemon=True) for _ in range(4)]
    for t in ts:
        t.start()
    for k in range(1, 7):
        assert m.handle("POST", "/load", body=f"program=IN+ACC%0AADD+{k}%0AOUT+ACC&targetURI=p".encode(),
                        ctype=FORM).code == 200
        m.handle("POST", "/run")
        assert _compute(m, 1) == (200, f'{{"value":{1 + k}}}\n')
    stop.set()
    for t in ts:
        t.join(30)
    assert set(codes) <= {200, 400, 504} and codes.count(200) > 0


@pytest.mark.gpu
def test_gpu_call_timeout_then_next_call(gpu):
    m = MasterNode({k: {"type": "program"} for k in SPINNER}, SPINNER, budget=5000, call_timeout=0.3)
    m.handle("POST", "/run")
    assert _compute(m, 0) == (504, "network produced no output\n")
    assert _compute(m, 5) == (200, '{"value":5}\n')
