"""Reference-structured CPU emulation of a Misaka Net deployment.

TEST / BASELINE INFRASTRUCTURE ONLY (bench.py's cpu_baseline leg and tests):
never imported by the product package.  It is labelled an *emulation*: the
reference itself (Go 1.14 + grpc-go over TLS, one container per node) cannot
be built or run here (SURVEY.md 8.2 d(ii)).

Structure, as the reference has it:
  * one thread per program node looping ``update()`` (program.go:80-92),
    one instruction per call, a failed instruction retried (ptr does not
    advance, :219-432), immediates re-parsed by an Atoi restatement on every
    execution (:230, :286, ...), jumps through the label map (:315-347), JRO
    clamped with IntClamp (:348-363);
  * every network operation is a gRPC call on a FRESH channel (grpc.Dial per
    op, program.go:492, 510, 525, 540, 555) to the peer's server:
    Program.Send into a capacity-1 register channel (:160-175), Stack.Push /
    Stack.Pop (stack.go:95-155, pop blocks while empty), Master.GetInput /
    SendOutput (master.go:233-249, capacity-1 inChan / outChan);
  * values cross every hop as int32 (the sint32 wire form).
Differences: Python threads under the GIL instead of goroutines, insecure
loopback channels instead of TLS, 127.0.0.1:<port> per node instead of
docker service names on :8001.
"""
from __future__ import annotations

import queue
import threading
from concurrent import futures
from typing import Optional, Sequence

import grpc

from . import pyoracle

_I64 = 1 << 63


def _wrap64(v: int) -> int:
    return ((v + _I64) % (1 << 64)) - _I64


def _int32(v: int) -> int:
    return ((int(v) + 2**31) % 2**32) - 2**31


def _atoi(s: str) -> int:
    """strconv.Atoi on a 64-bit platform (raises ValueError like Go returns err)."""
    return pyoracle.go_atoi(s)


# ---- wire codecs (messenger.proto: ValueMessage{sint32}, SendMessage{sint32, int32}) ----
def _varint(u: int) -> bytes:
    out = bytearray()
    while True:
        b, u = u & 0x7F, u >> 7
        out.append(b | 0x80 if u else b)
        if not u:
            return bytes(out)


def _read_varint(buf: bytes, i: int):
    u = shift = 0
    while True:
        b = buf[i]
        i += 1
        u |= (b & 0x7F) << shift
        if not b & 0x80:
            return u, i
        shift += 7


def _fields(buf: bytes):
    i = 0
    while i < len(buf):
        key, i = _read_varint(buf, i)
        v, i = _read_varint(buf, i)
        yield key >> 3, v


def enc_value(v: int) -> bytes:
    v = _int32(v)
    z = ((v << 1) ^ (v >> 31)) & 0xFFFFFFFF
    return b"\x08" + _varint(z) if z else b""


def dec_value(buf: bytes) -> int:
    out = 0
    for num, x in _fields(buf):
        if num == 1:
            out = (x >> 1) ^ -(x & 1)
    return out


def enc_send(t) -> bytes:
    value, reg = t
    out = enc_value(value)
    if reg:
        out += b"\x10" + _varint(reg & 0xFFFFFFFFFFFFFFFF)
    return out


def dec_send(buf: bytes):
    value = reg = 0
    for num, x in _fields(buf):
        if num == 1:
            value = (x >> 1) ^ -(x & 1)
        elif num == 2:
            reg = _int32(x)
    return value, reg


def enc_empty(_=None) -> bytes:
    return b""


def dec_empty(_b):
    return ()


class Stopped(Exception):
    pass


class _Chan:
    """A Go channel of capacity 1 whose blocked operations give up on stop."""

    def __init__(self, stop: threading.Event):
        self.q: queue.Queue = queue.Queue(maxsize=1)
        self.stop = stop

    def put(self, v):
        while True:
            try:
                return self.q.put(v, timeout=0.05)
            except queue.Full:
                if self.stop.is_set():
                    raise Stopped()

    def get(self):
        while True:
            try:
                return self.q.get(timeout=0.05)
            except queue.Empty:
                if self.stop.is_set():
                    raise Stopped()


def _server(service: str, handlers: dict, workers: int = 8):
    srv = grpc.server(futures.ThreadPoolExecutor(max_workers=workers))
    srv.add_generic_rpc_handlers((grpc.method_handlers_generic_handler(f"grpc.{service}", handlers),))
    port = srv.add_insecure_port("127.0.0.1:0")
    srv.start()
    return srv, f"127.0.0.1:{port}"


class _Dialer:
    """grpc.Dial per operation (program.go:492 ...), or one cached channel per
    peer with ``dial_per_hop=False``."""

    def __init__(self, per_hop: bool):
        self.per_hop = per_hop
        self.cache: dict = {}

    def call(self, addr: str, method: str, req, ser, de):
        opts = [("grpc.enable_http_proxy", 0)]
        if self.per_hop:
            ch = grpc.insecure_channel(addr, options=opts)
            try:
                return ch.unary_unary(method, request_serializer=ser, response_deserializer=de)(req, timeout=5.0)
            finally:
                ch.close()
        ch = self.cache.get(addr)
        if ch is None:
            ch = self.cache[addr] = grpc.insecure_channel(addr, options=opts)
        return ch.unary_unary(method, request_serializer=ser, response_deserializer=de)(req, timeout=5.0)


class ProgramNodeEmu:
    def __init__(self, name: str, program: str, net: "RefStructNet"):
        self.name, self.net = name, net
        self.asm = pyoracle.tokenize(program)  # LoadProgram (program.go:178-193)
        self.labels = pyoracle.label_map(program)
        self.acc = self.bak = self.ptr = 0
        self.r = [_Chan(net.stop) for _ in range(4)]
        self.retired = 0
        self.dial = _Dialer(net.dial_per_hop)
        self.srv, self.addr = _server("Program", {
            "Send": grpc.unary_unary_rpc_method_handler(self._send, request_deserializer=dec_send,
                                                        response_serializer=enc_empty)})

    # Program.Send (program.go:160-175)
    def _send(self, req, context):
        value, reg = req
        if not 0 <= reg <= 3:
            context.abort(grpc.StatusCode.UNKNOWN, "not a valid register")
        try:
            self.r[reg].put(value)
        except Stopped:
            context.abort(grpc.StatusCode.CANCELLED, "stopped")
        return ()

    def _src(self, s: str) -> int:  # getFromSrc (program.go:434-472)
        if s == "ACC":
            return self.acc
        if s == "NIL":
            return 0
        if s in ("R0", "R1", "R2", "R3"):
            return self.r[int(s[1])].get()
        raise ValueError(f"'{s}' not a valid src")

    def _addr(self, name: str) -> str:
        a = self.net.addr.get(name)
        if a is None:  # unknown host: grpc.Dial WithBlock hangs (program.go:72, 492)
            self.net.stop.wait()
            raise Stopped()
        return a

    def _send_value(self, v: int, target: str):  # program.go:475-506
        name, _, reg = target.partition(":")
        self.dial.call(self._addr(name), "/grpc.Program/Send", (_int32(v), int(reg[1])), enc_send, dec_empty)

    def _push(self, v: int, target: str):  # program.go:509-521
        self.dial.call(self._addr(target), "/grpc.Stack/Push", _int32(v), enc_value, dec_empty)

    def _pop(self, source: str) -> int:  # program.go:524-536
        return self.dial.call(self._addr(source), "/grpc.Stack/Pop", None, enc_empty, dec_value)

    def _in(self) -> int:  # program.go:539-551
        return self.dial.call(self.net.master_addr, "/grpc.Master/GetInput", None, enc_empty, dec_value)

    def _out(self, v: int):  # program.go:554-566
        self.dial.call(self.net.master_addr, "/grpc.Master/SendOutput", _int32(v), enc_value, dec_empty)

    def update(self):  # program.go:219-432
        t = self.asm[self.ptr]
        op = t[0]
        if op == "NOP":
            pass
        elif op == "MOV_VAL_LOCAL":
            v = _atoi(t[1])
            if t[2] == "ACC":
                self.acc = v
        elif op == "MOV_VAL_NETWORK":
            self._send_value(_atoi(t[1]), t[2])
        elif op == "MOV_SRC_LOCAL":
            v = self._src(t[1])
            if t[2] == "ACC":
                self.acc = v
        elif op == "MOV_SRC_NETWORK":
            self._send_value(self._src(t[1]), t[2])
        elif op == "SWP":
            self.acc, self.bak = self.bak, self.acc
        elif op == "SAV":
            self.bak = self.acc
        elif op == "ADD_VAL":
            self.acc = _wrap64(self.acc + _atoi(t[1]))
        elif op == "SUB_VAL":
            self.acc = _wrap64(self.acc - _atoi(t[1]))
        elif op == "ADD_SRC":
            self.acc = _wrap64(self.acc + self._src(t[1]))
        elif op == "SUB_SRC":
            self.acc = _wrap64(self.acc - self._src(t[1]))
        elif op == "NEG":
            self.acc = _wrap64(-self.acc)
        elif op in ("JMP", "JEZ", "JNZ", "JGZ", "JLZ"):
            take = {"JMP": True, "JEZ": self.acc == 0, "JNZ": self.acc != 0, "JGZ": self.acc > 0,
                    "JLZ": self.acc < 0}[op]
            if take:
                self.ptr = self.labels[t[1]]
                self.retired += 1
                return
        elif op in ("JRO_VAL", "JRO_SRC"):
            v = _atoi(t[1]) if op == "JRO_VAL" else self._src(t[1])
            self.ptr = min(max(_wrap64(self.ptr + v), 0), len(self.asm) - 1)  # IntClamp (math.go:20-22)
            self.retired += 1
            return
        elif op == "PUSH_VAL":
            self._push(_atoi(t[1]), t[2])
        elif op == "PUSH_SRC":
            self._push(self._src(t[1]), t[2])
        elif op == "POP":
            v = self._pop(t[1])
            if t[2] == "ACC":
                self.acc = v
        elif op == "IN":
            v = self._in()
            if t[1] == "ACC":
                self.acc = v
        elif op == "OUT_VAL":
            self._out(_atoi(t[1]))
        elif op == "OUT_SRC":
            self._out(self._src(t[1]))
        else:
            raise ValueError(f"'{t}' not a valid instruction")
        self.ptr = (self.ptr + 1) % len(self.asm)
        self.retired += 1

    def loop(self):  # Start (program.go:80-92): update forever, errors retried
        while not self.net.stop.is_set():
            try:
                self.update()
            except Stopped:
                return
            except (grpc.RpcError, ValueError):
                if self.net.stop.is_set():
                    return
                self.net.stop.wait(0.01)  # the reference retries at once; the emulation backs off


class StackNodeEmu:
    """Stack.Push / Stack.Pop (stack.go:95-155): unbounded LIFO, pop blocks while empty."""

    def __init__(self, net: "RefStructNet"):
        self.net = net
        self.items: list = []
        self.cv = threading.Condition()
        self.srv, self.addr = _server("Stack", {
            "Push": grpc.unary_unary_rpc_method_handler(self._push, request_deserializer=dec_value,
                                                        response_serializer=enc_empty),
            "Pop": grpc.unary_unary_rpc_method_handler(self._pop, request_deserializer=dec_empty,
                                                       response_serializer=enc_value)})

    def _push(self, v, _ctx):
        with self.cv:
            self.items.append(int(v))
            self.cv.notify_all()
        return ()

    def _pop(self, _req, context):
        with self.cv:
            while not self.items:
                if self.net.stop.is_set():
                    context.abort(grpc.StatusCode.CANCELLED, "stopped")
                self.cv.wait(0.05)
            return self.items.pop()


class MasterEmu:
    """inChan / outChan (master.go:58-59) and GetInput / SendOutput (:233-249)."""

    def __init__(self, net: "RefStructNet"):
        self.inq, self.outq = _Chan(net.stop), _Chan(net.stop)
        self.srv, self.addr = _server("Master", {
            "GetInput": grpc.unary_unary_rpc_method_handler(self._get, request_deserializer=dec_empty,
                                                            response_serializer=enc_value),
            "SendOutput": grpc.unary_unary_rpc_method_handler(self._send, request_deserializer=dec_value,
                                                              response_serializer=enc_empty)}, workers=16)

    def _get(self, _req, context):
        try:
            return _int32(self.inq.get())  # master.go:237
        except Stopped:
            context.abort(grpc.StatusCode.CANCELLED, "input retrieval cancelled")

    def _send(self, v, context):
        try:
            self.outq.put(int(v))
        except Stopped:
            context.abort(grpc.StatusCode.CANCELLED, "stopped")
        return ()

    def compute(self, v: int) -> int:  # /compute (master.go:216-219)
        self.inq.put(int(v))
        return self.outq.get()


class RefStructNet:
    """A running emulated deployment; ``compute(x)`` is one /compute."""

    def __init__(self, nodes: Sequence, *, dial_per_hop: bool = True, start: bool = True):
        rows = [(n.name, n.kind, n.program) if hasattr(n, "name") else tuple(n) for n in nodes]
        self.stop = threading.Event()
        self.dial_per_hop = dial_per_hop
        self.master = MasterEmu(self)
        self.master_addr = self.master.addr
        self.addr: dict = {}
        self.programs: list = []
        self.stacks: list = []
        for name, kind, prog in rows:
            if kind == "program":
                p = ProgramNodeEmu(name, prog or "", self)
                self.programs.append(p)
                self.addr[name] = p.addr
            elif kind == "stack":
                s = StackNodeEmu(self)
                self.stacks.append(s)
                self.addr[name] = s.addr
            elif kind == "master":
                self.addr[name] = self.master.addr
        self.threads = [threading.Thread(target=p.loop, daemon=True) for p in self.programs]
        if start:
            self.start()

    def start(self):
        """Start the node loops (``start=False`` lets a test point ``addr`` /
        ``master_addr`` at other processes' services first)."""
        for t in self.threads:
            t.start()

    @property
    def retired(self) -> int:
        return sum(p.retired for p in self.programs)

    def compute(self, v: int) -> int:
        return self.master.compute(v)

    def close(self):
        self.stop.set()
        for t in self.threads:
            if t.is_alive():
                t.join(2.0)
        for x in [self.master] + self.programs + self.stacks:
            x.srv.stop(0)


def time_compute(nodes, xs, seconds: float = 5.0, dial_per_hop: bool = True) -> dict:
    """Sequential /compute calls through the emulated deployment for about
    ``seconds`` (a call still blocked at the deadline is abandoned):
    results/s and retired node-instructions/s over the completed calls."""
    import time

    net = RefStructNet(nodes, dial_per_hop=dial_per_hop)
    done = {"n": 0, "outs": [], "retired": 0, "t": 0.0}
    t0 = [0.0]
    r0 = [0]

    def work():
        try:
            net.compute(int(xs[0]))  # warm: servers up, first dials made
            r0[0] = net.retired
            t0[0] = time.perf_counter()
            i = 1
            while not net.stop.is_set():
                o = net.compute(int(xs[i % len(xs)]))
                done["outs"].append(o)
                done["n"] += 1
                done["t"] = time.perf_counter() - t0[0]
                done["retired"] = net.retired - r0[0]
                i += 1
        except Stopped:
            pass

    th = threading.Thread(target=work, daemon=True)
    th.start()
    deadline = time.perf_counter() + seconds
    while time.perf_counter() < deadline and th.is_alive():
        th.join(0.05)
        if t0[0] and time.perf_counter() - t0[0] >= seconds:
            break
    net.close()
    th.join(5.0)
    dt = done["t"]
    n = done["n"]
    return {"results": n, "seconds": dt, "results_per_s": n / dt if dt else 0.0,
            "node_instr_per_s": done["retired"] / dt if dt else 0.0, "outputs": done["outs"],
            "threads": len(net.programs)}
