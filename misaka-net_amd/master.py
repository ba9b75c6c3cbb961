"""The master node's HTTP surface (internal/nodes/master.go:90-227) over the
batched GPU executor -- SURVEY.md section 8 row f1.

Routes, methods, status codes and error texts follow master.go:
  POST /run      -> "Success"                      (master.go:90-106)
  POST /pause    -> "Success"                      (master.go:108-124)
  POST /reset    -> "Success"                      (master.go:126-143)
  POST /load     program, targetURI -> "Success"   (master.go:145-195)
  POST /compute  value -> {"value": N}\\n           (master.go:197-224)
  any other method -> 405 "method GET not allowed"
Added: POST /compute_batch with repeated ``value`` fields (or a JSON body
``{"values": [...]}``) -> {"values": [...], "status": [...]}, evaluated as
one GPU batch.

Deliberate differences (DESIGN.md / INTEGRATION.md):
  * /load reaches the program node (the reference dials targetURI:8000 while
    program nodes serve :8001, master.go:178, so its /load never completes);
    a rejected program answers 400 "error loading program on node X: <Go
    error text>" and leaves the previous program in place (program.go:180-192).
  * by default (``stateful=True``) the reference's semantics: one network
    instance whose node state, stacks and channels persist across /compute
    calls (program.go:80-92, master.go:216-219), on the GPU (SessionSet, row
    f2); /reset and /load reset it, /pause keeps it (a call in flight when
    /pause comes stays open and waits, as the reference's handler stays
    blocked on outChan while the nodes are paused; /run lets it continue,
    its ``call_timeout`` still running; /reset and /load end it, 504).
    Concurrent /compute requests are coalesced: the ones that arrive while a
    launch is in flight run, in arrival order, as sequential calls of the next single launch
    (mk_session_compute_seq) -- the reference serves them one at a time
    through its capacity-1 inChan/outChan.
  * ``stateful=False`` is the batch extension (the lane model): every input
    runs on a fresh post-/reset copy of the network, and concurrent /compute
    requests are coalesced into one mk_compute_batch.  /compute_batch is the
    explicit many-values form of either mode.
  * ``wire=MasterService`` (misaka_net_amd.wire, row f4): /compute goes over
    the reference's gRPC wire instead -- inChan/outChan served as
    grpc.Master.GetInput/SendOutput to external (reference) program nodes,
    exactly master.go:216-219; /pause cancels blocked calls, /reset renews
    the channels.  ``wire_timeout`` bounds the wait (504), the reference has
    none.
  * a /compute whose network produces no output answers 504 "network
    produced no output" instead of hanging forever: at once when nothing
    can change without another input (the instance keeps its state and
    serves the next call), or, stateful, after ``call_timeout`` seconds of
    resuming a call that keeps running (it is abandoned; what it deposited
    stays).  The reference's abandoned handler would instead stay blocked on
    outChan and take the next output (master.go:219).
"""
from __future__ import annotations

import json
import threading
import time
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Mapping, Optional
from urllib.parse import unquote_to_bytes

import numpy as np

from . import _native as N
from .network import Network, NodeSpec, TisParseError, tokenize


class FormError(ValueError):
    pass


def _unescape(s: str) -> str:
    # url.QueryUnescape: '+' -> ' ', %XX must be two hex digits
    i = 0
    while True:
        i = s.find("%", i)
        if i < 0:
            break
        h = s[i + 1: i + 3]
        if len(h) != 2 or any(c not in "0123456789abcdefABCDEF" for c in h):
            raise FormError("invalid URL escape")
        i += 3
    return unquote_to_bytes(s.replace("+", " ")).decode("utf-8", "surrogateescape")


def parse_query(q: str) -> dict:
    """Go 1.14 url.ParseQuery: pairs split on '&' and ';', first error wins."""
    out: dict = {}
    for part in q.replace(";", "&").split("&"):
        if not part:
            continue
        k, _, v = part.partition("=")
        out.setdefault(_unescape(k), []).append(_unescape(v))
    return out


def go_atoi(s: str) -> int:
    """strconv.Atoi on a 64-bit platform."""
    if not s:
        raise ValueError("invalid syntax")
    body = s[1:] if s[0] in "+-" else s
    if not body or any(c not in "0123456789" for c in body):
        raise ValueError("invalid syntax")
    v = int(s)
    if not -(2**63) <= v < 2**63:
        raise ValueError("value out of range")
    return v


class Response:
    def __init__(self, code: int, body: str, ctype: str = "text/plain; charset=utf-8"):
        self.code, self.body, self.ctype = code, body, ctype


def http_error(msg: str, code: int) -> Response:
    return Response(code, msg + "\n")  # http.Error appends a newline


class _Slot:
    __slots__ = ("v", "done", "result", "error")

    def __init__(self, v):
        self.v, self.done, self.result, self.error = v, False, None, None


class Coalescer:
    """Group commit for concurrent single-value requests: a request that finds
    no batch in flight runs every request queued so far (``max_batch`` at a
    time) as one ``run(values) -> [(has_output, value)]`` call; requests that
    arrive meanwhile wait and form the next batch.  No timer: under load the
    batch is whatever accumulated during the previous launch, and a lone
    request runs at once."""

    def __init__(self, run, max_batch: int = 65536):
        self._run, self.max_batch = run, max_batch
        self._q: list = []
        self._cv = threading.Condition()
        self._busy = False
        self.batches = 0  # launches made (tests and the bench read it)
        self.requests = 0

    def submit(self, v):
        s = _Slot(v)
        with self._cv:
            self._q.append(s)
            while not s.done:
                if self._busy:
                    self._cv.wait()
                    continue
                self._busy = True
                batch, self._q = self._q[: self.max_batch], self._q[self.max_batch:]
                self._cv.release()
                try:
                    res, err = self._run([b.v for b in batch]), None
                except Exception as e:  # delivered to every request of the batch
                    res, err = None, e
                finally:
                    self._cv.acquire()
                for i, b in enumerate(batch):
                    b.result, b.error, b.done = (res[i] if res is not None else None), err, True
                self.batches += 1
                self.requests += len(batch)
                self._busy = False
                self._cv.notify_all()
        if s.error is not None:
            raise s.error
        return s.result


class MasterNode:
    """In-process master: the request handlers of master.go over a Network.

    ``node_info``: NODE_INFO (name -> {"type": "program"|"stack"});
    ``programs``: the PROGRAM text each program node booted with;
    ``name``: the master's own service name (MASTER_URI of the nodes).
    """

    def __init__(self, node_info: Mapping[str, Mapping], programs: Optional[Mapping[str, str]] = None,
                 name: str = "last_order", devices=None, budget=None, stack_cap=None, stateful: bool = True,
                 wire=None, wire_timeout: Optional[float] = 30.0, max_batch: int = 65536,
                 call_timeout: Optional[float] = 30.0):
        self.node_info = {k: dict(v) for k, v in node_info.items()}
        self.name = name
        self.programs = {k: "" for k, v in self.node_info.items() if v.get("type") == "program"}
        self.devices, self.budget, self.stack_cap = devices, budget, stack_cap
        self.is_running = False
        # Locks, always taken in this order: _lock guards the control state
        # (programs, the network and session handles, _epoch) and serialises
        # /run /pause /reset /load; _burst serialises stateful bursts (one
        # open call at a time); _exec is held for one executor launch.  A
        # stateful burst holds _exec per launch only, so /reset, /pause and
        # /load wait at most one budget slice, never a whole call:
        # they bump _epoch, and a burst that sees it changed stops resuming.
        self._lock = threading.Lock()
        self._burst = threading.Lock()
        self._exec = threading.Lock()
        self._epoch = 0  # bumped by /reset and /load (under _exec): calls in flight end
        self._running = threading.Event()  # is_running, for calls waiting out a /pause
        # cmd/app.go:21-24: a PROGRAM that fails to load is logged and the node
        # keeps its default program ([["NOP"]], program.go:64)
        for k, text in (programs or {}).items():
            if k in self.programs:
                try:
                    tokenize(text)
                    self.programs[k] = text
                except TisParseError:
                    pass
        self._net = None
        self.stateful = stateful
        self._sess = None
        self.wire, self.wire_timeout = wire, wire_timeout
        # stateful mode: how long a call that outlives its budget slice is
        # resumed before it is answered 504 and abandoned (the reference's
        # handler waits forever, master.go:219)
        self.call_timeout = call_timeout
        self.coalescer = Coalescer(self._run_batch, max_batch)

    # -- network handle ------------------------------------------------------
    def _specs(self):
        specs = []
        for k, v in self.node_info.items():
            t = v.get("type")
            if t not in ("program", "stack"):
                raise ValueError("invalid node type")  # master.go:437
            specs.append(NodeSpec(k, t, self.programs.get(k, "")))
        specs.append(NodeSpec(self.name, "master"))
        return specs

    def network(self) -> Network:
        if self._net is None:
            self._net = Network(self._specs())
        return self._net

    def session(self):
        """The one persistent network instance of stateful mode."""
        if self._sess is None:
            dev = next(iter(self.devices), 0) if self.devices else 0
            self._sess = self.network().sessions(1, device=dev, budget=self.budget, stack_cap=self.stack_cap)
        return self._sess

    def _drop_state(self, keep_session: bool = False):
        """Caller holds _lock and _exec.  /reset keeps the compiled session
        and clears its state (mk_session_reset); /load drops it."""
        if self._sess is not None:
            if keep_session:
                self._sess.reset()
            else:
                self._sess.close()
                self._sess = None

    def _run_batch(self, vals):
        """Values of coalesced requests -> [(has_output, value)] in order: on
        the one persistent instance as sequential calls (stateful), or as
        independent lanes (stateless); one executor launch either way."""
        if self.stateful:
            return [(h, o) for h, o, _ in self._run_stateful(vals)]
        with self._exec:
            r = self.network().compute_batch(np.asarray(vals, dtype=np.int64), budget=self.budget,
                                             stack_cap=self.stack_cap, devices=self.devices, steps=False)
        return [(bool(int(st) & N.MK_ST_HAS_OUTPUT), int(o)) for o, st in zip(r.out.tolist(), r.status.tolist())]

    def _run_stateful(self, vals):
        """Sequential /compute calls on the one instance -> [(has_output,
        value, status)].  A call that spends its budget slice stays open (the
        reference's nodes never give up, program.go:80-92): it is resumed
        until it has its output, closes, or the burst's ``call_timeout``
        passes (then 504, and the call is abandoned: the instance lives on).
        /reset, /pause and /load end the resuming at the next slice; the
        burst's calls that did not run answer no output (MK_ST_BUDGET).  The
        burst's later calls, which did not run behind an open call
        (MK_ST_CALL_OPEN), go in the next launch."""
        deadline = None if self.call_timeout is None else time.monotonic() + self.call_timeout
        res: list = []
        with self._burst:
            epoch = self._epoch
            while len(res) < len(vals):
                if not self._wait_running(epoch, deadline):
                    break
                with self._exec:
                    if self._epoch != epoch:
                        break
                    sess = self.session()
                    r = sess.compute_seq(np.asarray(vals[len(res):], dtype=np.int64), steps=False, busy_ok=True)
                for o, st in zip(r.out.tolist(), r.status.tolist()):
                    reason = st & N.MK_ST_REASON_MASK
                    if st & N.MK_ST_HAS_OUTPUT:
                        res.append((True, o, st))
                    elif reason == N.MK_ST_BUDGET:
                        res.append(self._finish_open_call(sess, epoch, deadline))
                        break
                    elif reason == N.MK_ST_CALL_OPEN:  # left open before this burst
                        with self._exec:
                            if self._sess is sess:
                                sess.cancel()
                        break
                    else:  # quiescent (the call closed, the instance lives on) or stack overflow
                        res.append((False, 0, st))
        res += [(False, 0, N.MK_ST_BUDGET)] * (len(vals) - len(res))
        return res

    def _wait_running(self, epoch, deadline) -> bool:
        """Wait out a /pause: the nodes do not run, and the reference's
        handler stays blocked on outChan until /run (master.go:216-219,
        program.go:80-92).  False when /reset or /load ended the burst, or
        its deadline passed."""
        while not self._running.is_set():
            if self._epoch != epoch:
                return False
            wait = 0.02
            if deadline is not None:
                wait = min(wait, deadline - time.monotonic())
                if wait <= 0:
                    return False
            self._running.wait(wait)
        return self._epoch == epoch

    def _finish_open_call(self, sess, epoch, deadline):
        while True:
            if not self._wait_running(epoch, deadline):
                with self._exec:
                    if self._sess is sess and self._epoch == epoch:  # the deadline passed while paused
                        sess.cancel()
                return False, 0, N.MK_ST_BUDGET
            with self._exec:
                if self._epoch != epoch or self._sess is not sess:  # /reset or /load
                    return False, 0, N.MK_ST_BUDGET
                r = sess.resume(steps=False)
                o, st = int(r.out[0]), int(r.status[0])
                if st & N.MK_ST_HAS_OUTPUT:
                    return True, o, st
                if (st & N.MK_ST_REASON_MASK) != N.MK_ST_BUDGET:
                    return False, 0, st
                if deadline is not None and time.monotonic() >= deadline:
                    sess.cancel()
                    return False, 0, st

    def _call(self, v: int):
        """One /compute: (has_output, value)."""
        if self.wire is not None:
            try:
                return True, self.wire.compute(v, timeout=self.wire_timeout)
            except Exception:  # timeout or cancelled by /pause, /reset
                return False, 0
        return self.coalescer.submit(v)

    # -- handlers -------------------------------------------------------------
    def handle(self, method: str, path: str, query: str = "", body: bytes = b"", ctype: str = "") -> Response:
        routes = {"/run": self._run, "/pause": self._pause, "/reset": self._reset, "/load": self._load,
                  "/compute": self._compute, "/compute_batch": self._compute_batch}
        fn = routes.get(path)
        if fn is None:
            return Response(404, "404 page not found\n")
        if method != "POST":
            return http_error("method GET not allowed", 405)
        return fn(query, body, ctype)

    def _form(self, query, body, ctype) -> dict:
        form = parse_query(query)
        if ctype.split(";")[0].strip().lower() == "application/x-www-form-urlencoded":
            for k, v in parse_query(body.decode("latin-1")).items():
                form.setdefault(k, [])
                form[k] = v + form[k]  # body values take precedence (r.Form order)
        return form

    def _check_types(self):
        for v in self.node_info.values():
            if v.get("type") not in ("program", "stack"):
                return "invalid node type"
        return None

    def _run(self, *_):
        with self._lock:
            self.is_running = True  # master.go:93 sets it before broadcasting
            self._running.set()
            e = self._check_types()
            if e:
                return http_error(f"error running network: {e}", 400)
            return Response(200, "Success")

    def _pause(self, *_):
        with self._lock:
            e = self._check_types()
            if e:
                return http_error(f"error pausing network: {e}", 400)
            self.is_running = False
            self._running.clear()  # a call in flight waits at its next slice, open, until /run
            if self.wire is not None:
                self.wire.cancel()  # stopNode: blocked GetInput calls return errors (master.go:117-119, 251-260)
            return Response(200, "Success")

    def _reset(self, *_):
        with self._lock:
            e = self._check_types()
            if e:
                return http_error(f"error resetting network: {e}", 400)
            self.is_running = False
            self._running.clear()
            with self._exec:  # at most one launch in flight to wait for
                self._epoch += 1  # a call in flight ends at its next slice
                # resetNode on every node and the master's channels (master.go:129-138)
                self._drop_state(keep_session=True)
            if self.wire is not None:
                self.wire.reset()
            return Response(200, "Success")

    def _load(self, query, body, ctype):
        try:
            form = self._form(query, body, ctype)
        except FormError:
            return http_error("cannot parse form", 400)
        program = (form.get("program") or [""])[0]
        target = (form.get("targetURI") or [""])[0]
        with self._lock:
            if target not in self.node_info:
                err = f"node {target} not valid on this network"
                return http_error(f"error loading program on node {target}: {err}", 400)
            e = self._check_types()
            if e:
                return http_error(f"error resetting network: {e}", 400)
            # ProgramNode.LoadProgram's parse (program.go:178-193) first: it
            # changes nothing
            err = None
            if self.node_info[target].get("type") != "program":
                err = "not a program node"
            else:
                try:
                    tokenize(program)
                except TisParseError as ex:
                    err = str(ex)
            # /load resets the whole network before the Load RPC, whatever the
            # RPC then does (master.go:165-175: broadcast reset, stopNode,
            # resetNode): node state, stacks and the master's channels.  All
            # of it in one executor section: a burst between two
            # sections would build a session on the old network, which the
            # second section then freed under it.  After this section the
            # next network() / session() is built from the new program.
            self.is_running = False
            self._running.clear()
            with self._exec:
                self._epoch += 1
                self._drop_state()
                if err is None:
                    self.programs[target] = program
                    if self._net is not None:
                        self._net.close()
                        self._net = None
            if self.wire is not None:
                self.wire.reset()
            if err is not None:
                return http_error(f"error loading program on node {target}: {err}", 400)
            return Response(200, "Success")

    def _values(self, form, key="value"):
        return form.get(key) or [""]

    def _compute(self, query, body, ctype):
        if not self.is_running:
            return http_error("network is not running", 400)
        try:
            form = self._form(query, body, ctype)
        except FormError:
            return http_error("cannot parse form", 400)
        try:
            v = go_atoi(self._values(form)[0])
        except ValueError:
            return http_error("cannot parse value", 400)
        ok, out = self._call(v)  # concurrent handlers, like net/http (master.go:197)
        if not ok:
            return http_error("network produced no output", 504)
        # json.NewEncoder(w).Encode(clientOutResponse{...}) (master.go:219): compact, newline-terminated
        return Response(200, json.dumps({"value": out}, separators=(",", ":")) + "\n", "application/json")

    def _compute_batch(self, query, body, ctype):
        if not self.is_running:
            return http_error("network is not running", 400)
        try:
            if ctype.split(";")[0].strip().lower() == "application/json":
                vals = [int(v) for v in json.loads(body.decode() or "{}").get("values", [])]
                for v in vals:
                    if not -(2**63) <= v < 2**63:
                        raise ValueError
            else:
                vals = [go_atoi(s) for s in self._form(query, body, ctype).get("value", [])]
        except FormError:
            return http_error("cannot parse form", 400)
        except (ValueError, TypeError, AttributeError):
            return http_error("cannot parse value", 400)
        if self.stateful:  # sequential /compute calls on the one instance
            got = self._run_stateful(vals)
            outs, sts = [g[1] for g in got], [g[2] for g in got]
        else:
            with self._exec:
                r = self.network().compute_batch(np.asarray(vals, dtype=np.int64), budget=self.budget,
                                                 stack_cap=self.stack_cap, devices=self.devices, steps=False)
            outs, sts = r.out.tolist(), r.status.tolist()
        has = [(x & N.MK_ST_HAS_OUTPUT) != 0 for x in sts]
        out = {"values": [x if h else None for x, h in zip(outs, has)], "status": sts}
        return Response(200, json.dumps(out) + "\n", "application/json")


def make_server(master: MasterNode, host: str = "127.0.0.1", port: int = 8000) -> ThreadingHTTPServer:
    """HTTP/1.1 server on :8000 (clientPort, master.go:18) around `master`."""

    class Handler(BaseHTTPRequestHandler):
        protocol_version = "HTTP/1.1"

        def _do(self):
            path, _, query = self.path.partition("?")
            n = int(self.headers.get("Content-Length") or 0)
            body = self.rfile.read(n) if n else b""
            r = master.handle(self.command, path, query, body, self.headers.get("Content-Type", ""))
            data = r.body.encode()
            self.send_response(r.code)
            self.send_header("Content-Type", r.ctype)
            if r.code >= 400:
                self.send_header("X-Content-Type-Options", "nosniff")
            self.send_header("Content-Length", str(len(data)))
            self.end_headers()
            self.wfile.write(data)

        do_GET = do_POST = do_PUT = do_DELETE = do_PATCH = _do

        def log_message(self, *a):
            pass

    class Server(ThreadingHTTPServer):
        # net/http accepts without a fixed backlog; socketserver's default of 5
        # resets bursts of concurrent clients
        request_queue_size = 1024
        daemon_threads = True

    return Server((host, port), Handler)
