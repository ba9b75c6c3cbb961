"""Mixed deployments: a network split between this executor and reference
nodes reached over the reference's gRPC wire.

The GPU holds one stateful instance (SessionSet of 1, row f2) of the nodes
declared local; nodes declared ``remote_program`` / ``remote_stack`` are
reference processes at the addresses given (the reference addresses peers as
``name:8001``, program.go:492, 510, 525).  ``MixedHost`` is the glue the
reference's processes talk to:

  * it serves, for every local program node, ``grpc.Program/Send`` into that
    node's port (program.go:160-175: blocks while the capacity-1 port is
    full) and, for every local stack, ``grpc.Stack/Push`` / ``grpc.Stack/Pop``
    (stack.go:95-114: a pop blocks while the stack is empty) -- each on its own
    address, ``addresses[name]``, which the peers are configured with;
  * a ``compute(x)`` call (the master's /compute, master.go:216-219) runs the
    GPU instance until it has the output; when the call parks
    (MK_ST_REMOTE_WAIT) the host makes every outstanding request's RPC --
    ``Program.Send`` to a remote port (program.go:475-506), ``Stack.Push`` /
    ``Stack.Pop`` on a remote stack (program.go:509-536), on a fresh channel
    per call as the reference dials per operation -- reports completions to
    the session, waits for a completion or an inbound RPC, and resumes.

  * for the network's master node (kind ``master``) it serves
    ``grpc.Master/GetInput`` and ``SendOutput`` (master.go:233-249) on the
    GPU instance's inChan / outChan, so remote program nodes can do IN / OUT.

Calls are serialised (the reference's capacity-1 inChan/outChan serve one
/compute at a time, master.go:216-219).  A call that spends its budget
slice stays open and is resumed; a call still open at its timeout is
abandoned (mk_session_cancel), so the next call starts cleanly.

Not covered: several GPU instances sharing one set of peers.
"""
from __future__ import annotations

import ctypes as C
import threading
import time
from concurrent import futures
from typing import Mapping, Optional, Sequence

import grpc

from . import _native as N
from . import wire
from .network import Network, NodeSpec

class MixedHost:
    def __init__(self, nodes: Sequence, peers: Mapping[str, str], *, budget=None, stack_cap=None, device: int = 0,
                 host: str = "127.0.0.1", rpc_timeout: float = 30.0):
        specs = [n if isinstance(n, NodeSpec) else NodeSpec(*n) for n in nodes]
        remote = [s.name for s in specs if s.kind.startswith("remote_")]
        missing = [r for r in remote if r not in peers]
        if missing:
            raise ValueError(f"no address for remote node(s) {missing}")
        self.net = Network(specs)
        self.sess = self.net.sessions(1, device=device, budget=budget, stack_cap=stack_cap)
        self.peers = dict(peers)
        self.rpc_timeout = rpc_timeout
        self.remote_names = remote  # MK_NODE_REMOTE_* in declaration order = the C index
        self._mu = threading.Lock()  # the session: steps and state edits
        self._call_mu = threading.Lock()  # one /compute call at a time, start to end
        self._cv = threading.Condition()
        self._gen = 0  # bumped by every inbound deposit and outbound completion
        self._inflight: set = set()
        self._closed = False
        self.addresses: dict = {}
        self._servers = []
        for s in specs:
            if s.kind == "program":
                self._serve(s.name, "Program", {"Send": grpc.unary_unary_rpc_method_handler(
                    self._send_handler(s.name), request_deserializer=wire.decode_send,
                    response_serializer=wire.encode_empty)}, host)
            elif s.kind == "stack":
                self._serve(s.name, "Stack", {
                    "Push": grpc.unary_unary_rpc_method_handler(self._push_handler(s.name),
                                                                request_deserializer=wire.decode_value,
                                                                response_serializer=wire.encode_empty),
                    "Pop": grpc.unary_unary_rpc_method_handler(self._pop_handler(s.name),
                                                               request_deserializer=wire.decode_empty,
                                                               response_serializer=wire.encode_value)}, host)
            elif s.kind == "master":
                self._serve(s.name, "Master", {
                    "GetInput": grpc.unary_unary_rpc_method_handler(self._get_input,
                                                                    request_deserializer=wire.decode_empty,
                                                                    response_serializer=wire.encode_value),
                    "SendOutput": grpc.unary_unary_rpc_method_handler(self._send_output,
                                                                      request_deserializer=wire.decode_value,
                                                                      response_serializer=wire.encode_empty)}, host)

    # ---- plumbing ---------------------------------------------------------------
    def _serve(self, name, service, handlers, host):
        srv = grpc.server(futures.ThreadPoolExecutor(max_workers=8))
        srv.add_generic_rpc_handlers((grpc.method_handlers_generic_handler(f"{wire.PACKAGE}.{service}", handlers),))
        port = srv.add_insecure_port(f"{host}:0")
        srv.start()
        self._servers.append(srv)
        self.addresses[name] = f"{host}:{port}"

    def _index(self, name):
        k, i = C.c_int(), C.c_int()
        N.check(N.lib().mk_net_node_index(self.net.handle, name.encode(), C.byref(k), C.byref(i)), name)
        return k.value, i.value

    def _event(self):
        with self._cv:
            self._gen += 1
            self._cv.notify_all()

    def _wait_event(self, gen, timeout):
        with self._cv:
            return self._cv.wait_for(lambda: self._gen != gen or self._closed, timeout)

    def _blocking(self, attempt, context):
        """Retry ``attempt()`` (returns a value or raises _Busy) after every
        state change until it succeeds, the RPC is cancelled or we close."""
        while True:
            with self._cv:
                gen = self._gen
            try:
                return attempt()
            except _Busy:
                pass
            if self._closed or (context is not None and not context.is_active()):
                if context is not None:
                    context.abort(grpc.StatusCode.CANCELLED, "node stopped")
                raise RuntimeError("closed")
            self._wait_event(gen, 0.5)

    # ---- inbound RPCs from the reference's nodes ----------------------------------
    def _send_handler(self, name):
        _, node = self._index(name)

        def send(req, context):  # Program.Send (program.go:160-175)
            value, reg = req
            if not 0 <= reg <= 3:
                context.abort(grpc.StatusCode.UNKNOWN, "not a valid register")

            def attempt():
                with self._mu:
                    rc = N.lib().mk_session_port_put(self.sess._h, 0, node, reg, value)
                if rc == N.MK_EBUSY:
                    raise _Busy()
                if rc != N.MK_OK:
                    context.abort(grpc.StatusCode.INTERNAL, f"{N.ERROR_NAMES.get(rc, rc)}: mk_session_port_put")
                self._event()
                return wire.EMPTY

            return self._blocking(attempt, context)

        return send

    def _push_handler(self, name):
        _, idx = self._index(name)

        def push(value, context):  # Stack.Push (stack.go:95-105)
            with self._mu:
                rc = N.lib().mk_session_stack_push(self.sess._h, 0, idx, value)
            if rc == N.MK_ELIMIT:
                context.abort(grpc.StatusCode.RESOURCE_EXHAUSTED, "stack_cap reached")
            if rc != N.MK_OK:
                context.abort(grpc.StatusCode.INTERNAL, f"{N.ERROR_NAMES.get(rc, rc)}: mk_session_stack_push")
            self._event()
            return wire.EMPTY

        return push

    def _pop_handler(self, name):
        _, idx = self._index(name)

        def pop(_req, context):  # Stack.Pop (stack.go:108-114): blocks while empty
            def attempt():
                v = C.c_int32()
                with self._mu:
                    rc = N.lib().mk_session_stack_pop(self.sess._h, 0, idx, C.byref(v))
                if rc == N.MK_EBUSY:
                    raise _Busy()
                if rc != N.MK_OK:
                    context.abort(grpc.StatusCode.INTERNAL, f"{N.ERROR_NAMES.get(rc, rc)}: mk_session_stack_pop")
                self._event()
                return v.value

            return self._blocking(attempt, context)

        return pop

    def _get_input(self, _req, context):  # Master.GetInput (master.go:233-242): blocks while inChan is empty
        def attempt():
            v = C.c_int32()
            with self._mu:
                rc = N.lib().mk_session_input_take(self.sess._h, 0, C.byref(v))
            if rc == N.MK_EBUSY:
                raise _Busy()
            if rc != N.MK_OK:
                context.abort(grpc.StatusCode.INTERNAL, f"{N.ERROR_NAMES.get(rc, rc)}: mk_session_input_take")
            self._event()
            return v.value

        return self._blocking(attempt, context)

    def _send_output(self, value, context):  # Master.SendOutput (master.go:245-249): blocks while outChan is full
        def attempt():
            with self._mu:
                rc = N.lib().mk_session_output_put(self.sess._h, 0, value)
            if rc == N.MK_EBUSY:
                raise _Busy()
            if rc != N.MK_OK:
                context.abort(grpc.StatusCode.INTERNAL, f"{N.ERROR_NAMES.get(rc, rc)}: mk_session_output_put")
            self._event()
            return wire.EMPTY

        return self._blocking(attempt, context)

    # ---- outbound RPCs of the GPU instance's nodes ----------------------------------
    def _rpc(self, req):
        target = self.peers[self.remote_names[req.remote]]
        ch = grpc.insecure_channel(target, options=[("grpc.enable_http_proxy", 0)])  # a dial per op (program.go:492)
        try:
            if req.op == N.MK_REMOTE_SEND:
                wire.ProgramClient(target, ch).send(req.value, req.reg, timeout=self.rpc_timeout)
                got = 0
            elif req.op == N.MK_REMOTE_PUSH:
                wire.StackClient(target, ch).push(req.value, timeout=self.rpc_timeout)
                got = 0
            else:
                got = wire.StackClient(target, ch).pop(timeout=self.rpc_timeout)
        finally:
            ch.close()
        with self._mu:
            N.check(N.lib().mk_session_remote_done(self.sess._h, 0, req.node, got), "mk_session_remote_done")
            self._inflight.discard(req.node)
        self._event()

    def _start_requests(self):
        reqs = (N.mk_remote_req * 16)()
        cnt = C.c_int()
        with self._mu:
            N.check(N.lib().mk_session_remote_poll(self.sess._h, 0, reqs, 16, C.byref(cnt)), "mk_session_remote_poll")
            new = [reqs[i] for i in range(cnt.value) if reqs[i].node not in self._inflight]
            for r in new:
                self._inflight.add(r.node)
        for r in new:
            copy = N.mk_remote_req(r.node, r.op, r.remote, r.reg, r.value)
            threading.Thread(target=self._rpc_safe, args=(copy,), daemon=True).start()
        return cnt.value

    def _rpc_safe(self, req):
        try:
            self._rpc(req)
        except Exception:  # the reference retries a failed RPC forever (program.go:80-92)
            with self._mu:
                self._inflight.discard(req.node)
            time.sleep(0.05)
            self._event()

    def _step(self, x: Optional[int]):
        """One launch; returns (status, out, gen) where gen is the event
        count right after it -- an inbound RPC or completion that lands
        later moves it (both take the session lock first)."""
        out, st, sp = C.c_int32(), C.c_uint8(), C.c_uint32()
        v = C.c_int64(0 if x is None else int(x))
        with self._mu:
            N.check(N.lib().mk_session_step(self.sess._h, None if x is None else C.byref(v), C.byref(out),
                                            C.byref(st), C.byref(sp)), "mk_session_step")
            with self._cv:  # inbound RPCs waiting on a full port / empty stack retry
                self._gen += 1
                gen = self._gen
                self._cv.notify_all()
        return st.value, out.value, gen

    # ---- /compute ----------------------------------------------------------------------
    def compute(self, x: int, timeout: Optional[float] = 60.0):
        """One /compute on the GPU instance: (has_output, value, status).
        A call parked on peers (MK_ST_REMOTE_WAIT) or out of its budget slice
        (MK_ST_BUDGET) is resumed until it has its output, closes, or
        ``timeout`` passes; then it is abandoned and the instance lives on."""
        with self._call_mu:
            deadline = None if timeout is None else time.monotonic() + timeout
            done = False
            try:
                st, out, gen = self._step(x)
                while True:
                    reason = st & N.MK_ST_REASON_MASK
                    if st & N.MK_ST_HAS_OUTPUT or reason not in (N.MK_ST_REMOTE_WAIT, N.MK_ST_BUDGET):
                        done = True
                        return bool(st & N.MK_ST_HAS_OUTPUT), out if st & N.MK_ST_HAS_OUTPUT else 0, st
                    left = None if deadline is None else deadline - time.monotonic()
                    if left is not None and left <= 0:
                        return False, 0, st
                    if reason == N.MK_ST_REMOTE_WAIT:
                        self._start_requests()
                        self._wait_event(gen, min(0.5, left) if left is not None else 0.5)
                    st, out, gen = self._step(None)
            finally:
                if not done and not self._closed:  # timed out (or failed) with the call open
                    with self._mu:
                        N.check(N.lib().mk_session_cancel(self.sess._h), "mk_session_cancel")
                    self._event()

    def close(self):
        self._closed = True
        self._event()
        for s in self._servers:
            s.stop(0)
        self.sess.close()


class _Busy(Exception):
    pass
