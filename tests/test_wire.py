"""gRPC wire compatibility: the hand-written
codecs of misaka_net_amd.wire against golden bytes and against the protobuf
runtime (descriptors built from messenger.proto:30-41 in Python, no protoc),
and the master's gRPC side (GetInput / SendOutput, master.go:233-249) over a
loopback channel with a stand-in for the reference's program nodes."""
import threading

import grpc
import pytest
from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

from misaka_net_amd import wire

EDGES = [0, 1, -1, 2, -2, 63, -64, 64, 127, 128, -129, 300, 2**31 - 1, -2**31, 2**31, 2**32 + 5, -2**33 - 7,
         123456789, -987654321]


def _proto_classes():
    F = descriptor_pb2.FieldDescriptorProto
    fdp = descriptor_pb2.FileDescriptorProto(name="messenger_check.proto", package="grpc", syntax="proto3")
    vm = fdp.message_type.add(name="ValueMessage")
    vm.field.add(name="value", number=1, type=F.TYPE_SINT32, label=F.LABEL_OPTIONAL)
    sm = fdp.message_type.add(name="SendMessage")
    sm.field.add(name="value", number=1, type=F.TYPE_SINT32, label=F.LABEL_OPTIONAL)
    sm.field.add(name="register", number=2, type=F.TYPE_INT32, label=F.LABEL_OPTIONAL)
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fdp)
    get = message_factory.GetMessageClass
    return get(pool.FindMessageTypeByName("grpc.ValueMessage")), get(pool.FindMessageTypeByName("grpc.SendMessage"))


def i32(v):
    return ((v + 2**31) % 2**32) - 2**31


def test_golden_bytes():
    assert wire.encode_value(7) == b"\x08\x0e"
    assert wire.encode_value(-1) == b"\x08\x01"
    assert wire.encode_value(0) == b""
    assert wire.encode_value(2**31 - 1) == b"\x08\xfe\xff\xff\xff\x0f"
    assert wire.encode_value(-2**31) == b"\x08\xff\xff\xff\xff\x0f"
    assert wire.encode_value(2**32 + 5) == b"\x08\x0a"  # int32(v) before the wire (program.go:561)
    assert wire.encode_send(-3, 2) == b"\x08\x05\x10\x02"
    assert wire.decode_value(b"") == 0 and wire.decode_value(b"\x08\x0e") == 7


def test_codecs_match_protobuf_runtime():
    VM, SM = _proto_classes()
    for v in EDGES:
        ref = VM(value=i32(v)).SerializeToString()
        assert wire.encode_value(v) == ref, v
        assert wire.decode_value(ref) == i32(v)
        for r in (0, 1, 3, -1, 2**31 - 1):
            ref = SM(value=i32(v), register=r).SerializeToString()
            assert wire.encode_send(v, r) == ref, (v, r)
            assert wire.decode_send(ref) == (i32(v), r)
    # unknown fields are skipped
    assert wire.decode_value(b"\x18\x05" + wire.encode_value(9) + b"\x22\x01x") == 9


@pytest.fixture
def master():
    svc = wire.MasterService()
    server, port = wire.serve_master(svc, "127.0.0.1:0")
    yield svc, port
    server.stop(None)


def _example_network_node(port, stop):
    """Stand-in for the reference's misaka1/misaka2 pair: IN, +1, +1, OUT."""
    c = wire.MasterClient(f"127.0.0.1:{port}")
    while not stop.is_set():
        try:
            v = c.get_input(timeout=0.5)
        except grpc.RpcError:
            continue
        c.send_output(v + 2)
    c.close()


def test_master_get_input_send_output_roundtrip(master):
    svc, port = master
    stop = threading.Event()
    t = threading.Thread(target=_example_network_node, args=(port, stop), daemon=True)
    t.start()
    try:
        assert svc.compute(5, timeout=10) == 7
        assert svc.compute(4294967301, timeout=10) == 7  # int32(v) at GetInput (master.go:237)
        assert svc.compute(2147483647, timeout=10) == -2147483647
    finally:
        stop.set()
        t.join(5)


def test_get_input_cancelled_by_pause(master):
    svc, port = master
    c = wire.MasterClient(f"127.0.0.1:{port}")
    err = {}

    def call():
        try:
            c.get_input(timeout=10)
        except grpc.RpcError as e:
            err["e"] = e

    t = threading.Thread(target=call)
    t.start()
    import time
    time.sleep(0.5)
    svc.cancel()
    t.join(10)
    assert err["e"].code() == grpc.StatusCode.UNKNOWN and "input retrieval cancelled" in err["e"].details()
    c.close()


def test_outchan_capacity_one(master):
    svc, port = master
    c = wire.MasterClient(f"127.0.0.1:{port}")
    c.send_output(1, timeout=5)  # fills outChan
    with pytest.raises(grpc.RpcError):
        c.send_output(2, timeout=0.5)  # blocks while full (master.go:246)
    svc._put(svc._in, 3, 1)
    assert svc._get(svc._out, 1) == 1
    c.close()


def test_http_master_over_the_wire(master):
    # /compute through MasterNode with the wire backend: the value goes out by
    # grpc.Master.GetInput to an external node and comes back by SendOutput
    from misaka_net_amd.master import MasterNode

    svc, port = master
    stop = threading.Event()
    t = threading.Thread(target=_example_network_node, args=(port, stop), daemon=True)
    t.start()
    try:
        m = MasterNode({"misaka1": {"type": "program"}}, {}, wire=svc, wire_timeout=10)
        form = "application/x-www-form-urlencoded"
        assert m.handle("POST", "/compute", body=b"value=5", ctype=form).code == 400  # not running
        m.handle("POST", "/run")
        r = m.handle("POST", "/compute", body=b"value=40", ctype=form)
        assert (r.code, r.body) == (200, '{"value":42}\n')
    finally:
        stop.set()
        t.join(5)
