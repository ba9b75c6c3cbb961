"""HTTP master surface (misaka_net_amd.master)
against master.go:90-249: routes, methods, status codes and error texts.
The compute paths run on the GPU (marked)."""
import http.client
import json
import threading

import pytest

import misaka_net_amd as mk
from misaka_net_amd.master import MasterNode, go_atoi, make_server, parse_query

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
