"""gRPC wire compatibility with the reference's nodes.

The reference's processes talk gRPC (internal/grpc/messenger.proto:9-41,
package ``grpc``): program nodes call ``Master.GetInput`` for IN and
``Master.SendOutput`` for OUT (program.go:539-566), and each other's
``Program.Send`` / the stacks' ``Stack.Push`` / ``Stack.Pop``.  Values travel as
``sint32`` (zigzag varint) -- the int32 width at every hop.

This module speaks that wire format without generated code:
  * hand-written codecs for ValueMessage {sint32 value = 1}, SendMessage
    {sint32 value = 1; int32 register = 2} and google.protobuf.Empty;
  * ``MasterService``: the master's side of a mixed deployment -- inChan and
    outChan of capacity 1 (master.go:58-59), ``GetInput`` blocking on inChan
    and truncating to int32 (master.go:233-242), ``SendOutput`` blocking while
    outChan is full (master.go:245-249), cancellation on pause/reset
    (master.go:251-266);
  * ``serve_master`` registers it on a grpc server under the reference's
    method names (``/grpc.Master/GetInput``, ``/grpc.Master/SendOutput``), so
    reference program nodes pointed at this process (MASTER_URI) feed it;
  * ``MasterClient`` / ``ProgramClient`` / ``StackClient``: callers of the
    reference services (tests use them as stand-ins for reference nodes).

TLS: the reference dials with TLS credentials from CERT_FILE/KEY_FILE
(cmd/app.go:15-16, program.go:70-73); ``serve_master`` takes optional
PEM key/cert bytes and listens insecurely without them.
"""
from __future__ import annotations

import threading
from typing import Optional

import grpc

PACKAGE = "grpc"  # messenger.proto:3


# ---- varint / zigzag codecs ---------------------------------------------------
def _varint(u: int) -> bytes:
    out = bytearray()
    while True:
        b = u & 0x7F
        u >>= 7
        if u:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _read_varint(buf: bytes, i: int):
    shift = 0
    u = 0
    while True:
        if i >= len(buf):
            raise ValueError("truncated varint")
        b = buf[i]
        i += 1
        u |= (b & 0x7F) << shift
        if not b & 0x80:
            return u, i
        shift += 7
        if shift >= 70:
            raise ValueError("varint too long")


def _int32(v: int) -> int:
    return ((int(v) + 2**31) % 2**32) - 2**31


def _zigzag32(v: int) -> int:
    v = _int32(v)
    return ((v << 1) ^ (v >> 31)) & 0xFFFFFFFF


def _unzigzag(u: int) -> int:
    u &= 0xFFFFFFFF
    return (u >> 1) ^ -(u & 1)


def _fields(buf: bytes):
    """(field number, wire type, value) of a serialized message; length-
    delimited and fixed fields are returned as bytes."""
    i = 0
    while i < len(buf):
        key, i = _read_varint(buf, i)
        num, wt = key >> 3, key & 7
        if wt == 0:
            v, i = _read_varint(buf, i)
        elif wt == 1:
            v, i = buf[i:i + 8], i + 8
        elif wt == 2:
            n, i = _read_varint(buf, i)
            v, i = buf[i:i + n], i + n
        elif wt == 5:
            v, i = buf[i:i + 4], i + 4
        else:
            raise ValueError(f"unsupported wire type {wt}")
        yield num, wt, v


def encode_value(v: int) -> bytes:
    """ValueMessage{Value: int32(v)} (messenger.proto:39-41; the int32()
    conversions of program.go:516,561 and master.go:237)."""
    z = _zigzag32(v)
    return b"\x08" + _varint(z) if z else b""  # proto3 omits the default


def decode_value(buf: bytes) -> int:
    v = 0
    for num, wt, x in _fields(buf):
        if num == 1 and wt == 0:
            v = _unzigzag(x)
    return v


def encode_send(value: int, register: int) -> bytes:
    """SendMessage{Value: int32(v), Register: r} (messenger.proto:34-37, program.go:498)."""
    out = b""
    z = _zigzag32(value)
    if z:
        out += b"\x08" + _varint(z)
    r = _int32(register)
    if r:
        out += b"\x10" + _varint(r & 0xFFFFFFFFFFFFFFFF)  # int32: negative as 10-byte varint
    return out


def decode_send(buf: bytes):
    value = register = 0
    for num, wt, x in _fields(buf):
        if num == 1 and wt == 0:
            value = _unzigzag(x)
        elif num == 2 and wt == 0:
            register = _int32(x)
    return value, register


class Empty:
    """google.protobuf.Empty (grpc treats a deserializer returning None as a
    failure, so an empty message is this object)."""

    def __repr__(self):
        return "Empty()"


EMPTY = Empty()


def encode_empty(_=None) -> bytes:
    return b""


def decode_empty(_buf: bytes) -> Empty:
    return EMPTY


# ---- the master's gRPC side --------------------------------------------------------
class Cancelled(Exception):
    pass


class MasterService:
    """inChan / outChan of the reference master (master.go:58-59, capacity 1
    each) plus the node context whose cancellation (stopNode, master.go:251-260)
    makes a blocked GetInput return an error."""

    def __init__(self):
        self._cv = threading.Condition()
        self._in: list[int] = []
        self._out: list[int] = []
        self._epoch = 0  # bumped by cancel(): waiters of an older epoch give up

    # -- channel operations ----------------------------------------------------
    def _put(self, chan: list, v: int, timeout: Optional[float]) -> None:
        with self._cv:
            ep = self._epoch
            if not self._cv.wait_for(lambda: len(chan) < 1 or self._epoch != ep, timeout):
                raise TimeoutError("channel full")
            if self._epoch != ep:
                raise Cancelled()
            chan.append(v)
            self._cv.notify_all()

    def _get(self, chan: list, timeout: Optional[float]) -> int:
        with self._cv:
            ep = self._epoch
            if not self._cv.wait_for(lambda: chan or self._epoch != ep, timeout):
                raise TimeoutError("channel empty")
            if self._epoch != ep:
                raise Cancelled()
            v = chan.pop(0)
            self._cv.notify_all()
            return v

    # -- what /compute does (master.go:216-219) ------------------------------------
    def compute(self, v: int, timeout: Optional[float] = None) -> int:
        self._put(self._in, int(v), timeout)
        return self._get(self._out, timeout)

    def cancel(self) -> None:
        """stopNode (master.go:252-260): blocked calls return errors."""
        with self._cv:
            self._epoch += 1
            self._cv.notify_all()

    def reset(self) -> None:
        """resetNode (master.go:263-266): fresh channels."""
        with self._cv:
            self._epoch += 1
            self._in.clear()
            self._out.clear()
            self._cv.notify_all()

    # -- gRPC handlers ---------------------------------------------------------------
    def GetInput(self, _request, context):  # master.go:233-242
        try:
            v = self._get(self._in, None)
        except Cancelled:
            context.abort(grpc.StatusCode.UNKNOWN, "input retrieval cancelled")
        return _int32(v)  # ValueMessage{Value: int32(v)}

    def SendOutput(self, value, _context):  # master.go:245-249
        self._put(self._out, int(value), None)
        return EMPTY


def serve_master(service: MasterService, address: str = "127.0.0.1:8001", *, max_workers: int = 16,
                 private_key: Optional[bytes] = None, certificate_chain: Optional[bytes] = None):
    """Start a grpc server exposing ``service`` as grpc.Master on ``address``
    (grpcPort ":8001", master.go:20).  Returns (server, bound port)."""
    from concurrent import futures

    handlers = {
        "GetInput": grpc.unary_unary_rpc_method_handler(
            service.GetInput, request_deserializer=decode_empty, response_serializer=encode_value),
        "SendOutput": grpc.unary_unary_rpc_method_handler(
            service.SendOutput, request_deserializer=decode_value, response_serializer=encode_empty),
    }
    server = grpc.server(futures.ThreadPoolExecutor(max_workers=max_workers))
    server.add_generic_rpc_handlers((grpc.method_handlers_generic_handler(f"{PACKAGE}.Master", handlers),))
    if private_key and certificate_chain:
        creds = grpc.ssl_server_credentials([(private_key, certificate_chain)])
        port = server.add_secure_port(address, creds)
    else:
        port = server.add_insecure_port(address)
    server.start()
    return server, port


# ---- callers of the reference services ------------------------------------------------
class _Client:
    def __init__(self, target: str, channel: Optional[grpc.Channel] = None):
        # no HTTP proxy for node-to-node traffic (the reference dials peers directly)
        self.channel = channel or grpc.insecure_channel(target, options=[("grpc.enable_http_proxy", 0)])

    def _call(self, service: str, method: str, req, ser, de, timeout=None):
        fn = self.channel.unary_unary(f"/{PACKAGE}.{service}/{method}", request_serializer=ser,
                                      response_deserializer=de)
        return fn(req, timeout=timeout)

    def close(self):
        self.channel.close()


class MasterClient(_Client):
    """What a program node's IN / OUT do (program.go:539-566)."""

    def get_input(self, timeout=None) -> int:
        return self._call("Master", "GetInput", None, encode_empty, decode_value, timeout)

    def send_output(self, v: int, timeout=None) -> None:
        self._call("Master", "SendOutput", v, encode_value, decode_empty, timeout)


class ProgramClient(_Client):
    """Program.Send (program.go:160-175) as sendValue calls it (program.go:497-498)."""

    def send(self, value: int, register: int, timeout=None) -> None:
        self._call("Program", "Send", (value, register), lambda t: encode_send(*t), decode_empty, timeout)


class StackClient(_Client):
    """Stack.Push / Stack.Pop (stack.go:95-114) as program.go:509-536 calls them."""

    def push(self, v: int, timeout=None) -> None:
        self._call("Stack", "Push", v, encode_value, decode_empty, timeout)

    def pop(self, timeout=None) -> int:
        return self._call("Stack", "Pop", None, encode_empty, decode_value, timeout)
