"""Host-side mirror of the reference's node network for the batched /compute path.

``Network`` replaces the set of ``ProgramNode``/``StackNode`` processes of a
deployment (internal/nodes/program.go, internal/nodes/stack.go; topology from
NODE_INFO, cmd/app.go:31, and each node's PROGRAM, cmd/app.go:21) by one
loaded ``mk_net`` handle.  ``compute_batch`` evaluates many independent
``/compute`` inputs (master.go:197-224) at once on the GPU.
"""
from __future__ import annotations

import atexit
import ctypes as C
import weakref
from dataclasses import dataclass
from typing import Iterable, Mapping, Optional, Sequence

import numpy as np

from . import _native as N

STATUS_NAMES = {
    N.MK_ST_QUIESCENT: "quiescent",
    N.MK_ST_BUDGET: "budget",
    N.MK_ST_STACK_OVERFLOW: "stack_overflow",
    N.MK_ST_OUTPUT_STOP: "output_stop",
}


# Native handles still open at interpreter exit are freed by an atexit hook
# (sessions before the networks they run on), while the HIP runtime and the
# caller's GPU state are intact, instead of by garbage collection during
# teardown or never.
_LIVE: "weakref.WeakSet" = weakref.WeakSet()


@atexit.register
def _close_live():
    live = list(_LIVE)
    for o in [o for o in live if isinstance(o, SessionSet)] + [o for o in live if isinstance(o, Network)]:
        try:
            o.close()
        except Exception:  # pragma: no cover - best effort at exit
            pass


class TisParseError(ValueError):
    """A program was rejected; ``str(e)`` is the reference's Go error text."""


def tokenize(program: str) -> list[list[str]]:
    """tis.Tokenize (internal/tis/tokenizer.go:29-106) on one program: the
    ``[][]string`` the reference builds, or TisParseError with its message."""
    buf = C.create_string_buffer(max(4096, 64 * len(program) + 1024))
    rc = N.lib().mk_tokenize(program.encode(), buf, len(buf))
    text = buf.value.decode(errors="surrogateescape")
    if rc == N.MK_EPARSE:
        raise TisParseError(text)
    N.check(rc, "mk_tokenize")
    return [line.split("\x1f") for line in text.split("\n")]


@dataclass
class NodeSpec:
    name: str
    kind: str = "program"  # "program" | "stack" | "master" | "remote_program" | "remote_stack"
    program: str = ""


_KINDS = {"program": N.MK_NODE_PROGRAM, "stack": N.MK_NODE_STACK, "master": N.MK_NODE_MASTER,
          "remote_program": N.MK_NODE_REMOTE_PROGRAM, "remote_stack": N.MK_NODE_REMOTE_STACK}


@dataclass
class BatchResult:
    out: np.ndarray  # int32: first OUT value (the /compute result), 0 if none
    status: np.ndarray  # uint8: MK_ST_* reason | MK_ST_HAS_OUTPUT
    steps: Optional[np.ndarray]  # uint32 retired node-instructions, if requested

    @property
    def has_output(self) -> np.ndarray:
        return (self.status & N.MK_ST_HAS_OUTPUT) != 0

    @property
    def reason(self) -> np.ndarray:
        return self.status & N.MK_ST_REASON_MASK


_MODES = {None: 0, "interp": N.MK_FLAG_FORCE_INTERP, "tile": N.MK_FLAG_TILE, "refill": N.MK_FLAG_REFILL,
          "jit": N.MK_FLAG_JIT}


def make_opts(budget=None, stack_cap=None, stop_on_output=False, devices: Optional[Iterable[int]] = None,
              interp=False, mode=None):
    """mk_opts.  ``mode``: None (automatic), "jit" (demand the native
    per-network kernel, tier 3), "tile" or "refill" (the tier-2 superblock
    interpreter with that lane scheduling, see mk.h MK_FLAG_TILE), "interp"
    (the direct bytecode interpreter, tier 1; same as ``interp=True``)."""
    if mode not in _MODES:
        raise ValueError(f"unknown executor mode {mode!r}")
    o = N.mk_opts()
    o.budget = int(budget or 0)
    o.stack_cap = int(stack_cap or 0)
    o.flags = ((N.MK_FLAG_STOP_ON_OUTPUT if stop_on_output else 0) | (N.MK_FLAG_FORCE_INTERP if interp else 0)
               | _MODES[mode])
    mask = 0
    for d in devices or ():
        mask |= 1 << int(d)
    o.device_mask = mask
    return o


class Network:
    """A loaded network.

    ``nodes`` is a sequence of NodeSpec (or ``(name, kind, program)`` tuples).
    Program nodes are executed in sorted-name order (the canonical schedule).
    """

    def __init__(self, nodes: Sequence):
        specs = [n if isinstance(n, NodeSpec) else NodeSpec(*n) for n in nodes]
        arr = (N.mk_node_desc * len(specs))()
        self._keep = []
        for i, s in enumerate(specs):
            if s.kind not in _KINDS:
                raise ValueError(f"invalid node type {s.kind!r}")
            nm, pg = s.name.encode(), (s.program or "").encode()
            self._keep += [nm, pg]
            arr[i].name, arr[i].kind, arr[i].program = nm, _KINDS[s.kind], pg
        h = C.c_void_p()
        err = C.create_string_buffer(8192)
        rc = N.lib().mk_net_load(arr, len(specs), C.byref(h), err, len(err))
        if rc == N.MK_EPARSE:
            raise TisParseError(err.value.decode(errors="surrogateescape"))
        N.check(rc, err.value.decode(errors="surrogateescape"))
        self._h = h
        self.specs = specs
        _LIVE.add(self)

    @classmethod
    def from_node_info(cls, node_info: Mapping[str, Mapping], programs: Mapping[str, str], master: Optional[str] = None):
        """Build from the master's NODE_INFO JSON (docker-compose.yml:16-21) and
        each program node's PROGRAM env var (cmd/app.go:21)."""
        nodes = [NodeSpec(name, info["type"], programs.get(name, "")) for name, info in node_info.items()]
        if master:
            nodes.append(NodeSpec(master, "master"))
        return cls(nodes)

    def close(self):
        if getattr(self, "_h", None):
            N.lib().mk_net_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self) -> C.c_void_p:
        return self._h

    def info(self):
        c = (C.c_int * 3)()
        N.check(N.lib().mk_net_info(self._h, c))
        return {"program_nodes": c[0], "stack_nodes": c[1], "instructions": c[2]}

    def disasm(self) -> str:
        buf = C.create_string_buffer(1 << 20)
        N.check(N.lib().mk_net_disasm(self._h, buf, len(buf)))
        return buf.value.decode()

    def plan(self, *, stack_cap=None, stop_on_output=False, interp=False, mode=None) -> str:
        """Which executor tier runs this network (compiles the schedule, and
        the native kernel, once)."""
        buf = C.create_string_buffer(4096)
        o = make_opts(None, stack_cap, stop_on_output, None, interp, mode)
        rc = N.lib().mk_net_plan(self._h, C.byref(o), buf, len(buf))
        if rc == N.MK_ELIMIT:
            return buf.value.decode()
        N.check(rc)
        return buf.value.decode()

    def prepare(self, *, stack_cap=None, stop_on_output=False, mode=None, device=0):
        """Compile everything a launch with these options uses on ``device``."""
        o = make_opts(None, stack_cap, stop_on_output, None, False, mode)
        N.check(N.lib().mk_net_prepare(self._h, C.byref(o), device), self.plan(stack_cap=stack_cap,
                                                                             stop_on_output=stop_on_output, mode=mode))

    def jit_source(self, *, stack_cap=None, stop_on_output=False) -> str:
        """hiprtc source of the native (tier-3) kernel."""
        buf = C.create_string_buffer(1 << 24)
        o = make_opts(None, stack_cap, stop_on_output)
        rc = N.lib().mk_net_jit_source(self._h, C.byref(o), buf, len(buf))
        N.check(rc, buf.value.decode())
        return buf.value.decode()

    def sched_disasm(self, *, stack_cap=None, stop_on_output=False) -> str:
        buf = C.create_string_buffer(1 << 24)
        o = make_opts(None, stack_cap, stop_on_output)
        N.check(N.lib().mk_net_sched_disasm(self._h, C.byref(o), buf, len(buf)))
        return buf.value.decode()

    def compute_batch(self, values, *, budget=None, stack_cap=None, stop_on_output=False, devices=None, steps=True,
                      interp=False, mode=None):
        """Evaluate independent /compute inputs (strconv.Atoi int64 values,
        truncated to int32 at GetInput like master.go:237) on the GPU(s)."""
        v = np.ascontiguousarray(np.asarray(values, dtype=np.int64))
        n = v.size
        out = np.zeros(n, np.int32)
        st = np.zeros(n, np.uint8)
        sp = np.zeros(n, np.uint32) if steps else None
        o = make_opts(budget, stack_cap, stop_on_output, devices, interp, mode)
        rc = N.lib().mk_compute_batch(
            self._h,
            v.ctypes.data_as(C.c_void_p),
            n,
            out.ctypes.data_as(C.c_void_p),
            st.ctypes.data_as(C.c_void_p),
            sp.ctypes.data_as(C.c_void_p) if sp is not None else None,
            C.byref(o),
        )
        N.check(rc, "mk_compute_batch")
        return BatchResult(out, st, sp)

    def compute_device(self, n, *, out_ptr, status_ptr, steps_ptr=None, stats_ptr=None, device=0, stream=None,
                       in_ptr=None, in_kind=N.MK_IN_I32, seed=0, gen_kind=N.MK_GEN_FULL, gen_mask=0, offset=0,
                       budget=None, stack_cap=None, stop_on_output=False, interp=False, mode=None,
                       defer_stats=False):
        """Launch on device memory (raw pointers, e.g. torch ``data_ptr()``);
        asynchronous on ``stream`` (a HIP stream handle, e.g.
        ``torch.cuda.current_stream().cuda_stream``).  ``defer_stats``: keep
        this launch's counters on the device until :meth:`stats_fold`."""
        mi = N.mk_input()
        mi.kind = N.MK_IN_GEN if in_ptr is None else in_kind
        mi.data = in_ptr
        mi.seed = seed
        mi.gen_kind = gen_kind
        mi.gen_mask = gen_mask
        mi.offset = offset
        o = make_opts(budget, stack_cap, stop_on_output, None, interp, mode)
        if defer_stats:
            o.flags |= N.MK_FLAG_DEFER_STATS
        rc = N.lib().mk_compute_device(
            self._h, device, C.byref(mi), n, out_ptr, status_ptr, steps_ptr, stats_ptr, C.byref(o), stream
        )
        N.check(rc, "mk_compute_device")

    def device_launcher(self, n, *, out_ptr, status_ptr, steps_ptr=None, device=0, in_ptr=None,
                        in_kind=N.MK_IN_I32, seed=0, gen_kind=N.MK_GEN_FULL, gen_mask=0, offset=0, budget=None,
                        stack_cap=None, stop_on_output=False, mode=None, defer_stats=False):
        """``compute_device`` with every argument fixed: returns ``launch(stream)``
        whose host cost is one foreign call (the ctypes structs are built once)."""
        mi = N.mk_input()
        mi.kind = N.MK_IN_GEN if in_ptr is None else in_kind
        mi.data = in_ptr
        mi.seed = seed
        mi.gen_kind = gen_kind
        mi.gen_mask = gen_mask
        mi.offset = offset
        o = make_opts(budget, stack_cap, stop_on_output, None, False, mode)
        if defer_stats:
            o.flags |= N.MK_FLAG_DEFER_STATS
        fn, h, pmi, po = N.lib().mk_compute_device, self._h, C.byref(mi), C.byref(o)

        def launch(stream=None):
            rc = fn(h, device, pmi, n, out_ptr, status_ptr, steps_ptr, None, po, stream)
            if rc:
                N.check(rc, "mk_compute_device")

        launch.keep = (mi, o, self)
        return launch

    TRACE_DTYPE = np.dtype([("round", "<u4"), ("node", "<u2"), ("ip", "<u2"), ("acc", "<i8"), ("bak", "<i8")])

    def trace(self, value, *, max_entries=4096, budget=None, stack_cap=None, stop_on_output=False, device=0):
        """Lane trace of one /compute input (mk_trace_lane): the first
        ``max_entries`` retired instructions as a structured array
        (round, node, ip, acc, bak) and the lane's status byte."""
        out = np.zeros(max_entries, self.TRACE_DTYPE)
        cnt = C.c_uint32()
        st = C.c_uint8()
        o = make_opts(budget, stack_cap, stop_on_output)
        N.check(N.lib().mk_trace_lane(self._h, device, int(value), C.byref(o), out.ctypes.data_as(C.c_void_p),
                                      max_entries, C.byref(cnt), C.byref(st)), "mk_trace_lane")
        return out[: cnt.value], st.value

    def sessions(self, n, *, device=0, budget=None, stack_cap=None) -> "SessionSet":
        """``n`` stateful instances of this network (row f2, :class:`SessionSet`)."""
        return SessionSet(self, n, device=device, budget=budget, stack_cap=stack_cap)

    def stats_fold(self, stats_ptr, *, device=0, stream=None):
        """Add the counters of deferred launches on ``device`` into the
        device uint64[MK_STATS_LEN] at ``stats_ptr`` (asynchronous)."""
        N.check(N.lib().mk_stats_fold(self._h, device, stats_ptr, stream), "mk_stats_fold")


class SessionSet:
    """``n`` stateful instances of a network on one GPU (SURVEY.md section 8
    row f2).  The reference's nodes keep running between /compute calls
    (program.go:80-92); here each instance's ACC/BAK/ptr, ports, stacks and the
    master's inChan/outChan persist in HBM between calls, and :meth:`compute`
    performs one /compute (master.go:216-219) on every instance at once."""

    def __init__(self, net: "Network", n: int, *, device: int = 0, budget=None, stack_cap=None):
        o = make_opts(budget, stack_cap)
        h = C.c_void_p()
        N.check(N.lib().mk_session_create(net.handle, device, n, C.byref(o), C.byref(h)), "mk_session_create")
        self._h, self._net, self.n, self.device = h, net, n, device
        _LIVE.add(self)

    def compute(self, values, *, steps=True, busy_ok=False) -> BatchResult:
        """One /compute call per instance: ``values[i]`` goes to instance i.

        A call whose budget slice runs out stays open (status MK_ST_BUDGET):
        :meth:`resume` continues it, :meth:`cancel` abandons it.  While one is
        open a new call on that instance does nothing (MK_ST_CALL_OPEN) and
        this raises MkError(MK_EBUSY) unless ``busy_ok``."""
        v = np.ascontiguousarray(np.asarray(values, dtype=np.int64))
        if v.size != self.n:
            raise ValueError(f"expected {self.n} values, got {v.size}")
        return self._step(v.ctypes.data_as(C.c_void_p), steps, busy_ok, "mk_session_compute")

    def resume(self, *, steps=True) -> BatchResult:
        """One more budget slice of every instance's open call (instances
        without one report status 0) -- mk_session_step(in = NULL)."""
        return self._step(None, steps, False, "mk_session_step")

    def _step(self, vp, steps, busy_ok, what) -> BatchResult:
        out = np.zeros(self.n, np.int32)
        st = np.zeros(self.n, np.uint8)
        sp = np.zeros(self.n, np.uint32) if steps else None
        rc = N.lib().mk_session_step(self._h, vp, out.ctypes.data_as(C.c_void_p), st.ctypes.data_as(C.c_void_p),
                                     sp.ctypes.data_as(C.c_void_p) if sp is not None else None)
        if not (busy_ok and rc == N.MK_EBUSY):
            N.check(rc, what)
        return BatchResult(out, st, sp)

    def plan(self) -> str:
        """Which tier runs the sessions (mk_session_plan)."""
        buf = C.create_string_buffer(1024)
        N.check(N.lib().mk_session_plan(self._h, buf, len(buf)), "mk_session_plan")
        return buf.value.decode()

    def cancel(self):
        """Abandon every instance's open call (mk_session_cancel)."""
        N.check(N.lib().mk_session_cancel(self._h), "mk_session_cancel")

    def compute_seq(self, values, *, steps=True, busy_ok=False) -> BatchResult:
        """Sequential /compute calls in one launch: ``values`` has shape
        (ncalls, n) -- row c is call c on every instance -- or, for n == 1,
        a flat list of the calls.  Results have the shape of ``values``.  A
        call that stays open (MK_ST_BUDGET) makes the instance's later calls
        of the burst report MK_ST_CALL_OPEN without running."""
        v = np.ascontiguousarray(np.asarray(values, dtype=np.int64))
        shape = v.shape
        if v.ndim == 1 and self.n == 1:
            v = v.reshape(-1, 1)
        if v.ndim != 2 or v.shape[1] != self.n:
            raise ValueError(f"expected (ncalls, {self.n}) values, got {shape}")
        m = v.shape[0]
        out = np.zeros(v.shape, np.int32)
        st = np.zeros(v.shape, np.uint8)
        sp = np.zeros(v.shape, np.uint32) if steps else None
        if m:
            rc = N.lib().mk_session_compute_seq(self._h, v.ctypes.data_as(C.c_void_p), m,
                                                out.ctypes.data_as(C.c_void_p), st.ctypes.data_as(C.c_void_p),
                                                sp.ctypes.data_as(C.c_void_p) if sp is not None else None)
            if not (busy_ok and rc == N.MK_EBUSY):
                N.check(rc, "mk_session_compute_seq")
        return BatchResult(out.reshape(shape), st.reshape(shape), sp.reshape(shape) if sp is not None else None)

    def compute_device(self, in_ptr, out_ptr, status_ptr, steps_ptr=None, *, stream=None):
        N.check(N.lib().mk_session_compute_device(self._h, in_ptr, out_ptr, status_ptr, steps_ptr, stream),
                "mk_session_compute_device")

    def compute_seq_device(self, in_ptr, ncalls, out_ptr, status_ptr, steps_ptr=None, *, stream=None):
        """A burst of `ncalls` sequential calls per instance in one launch on
        device arrays laid out [call][instance] (mk_session_compute_seq_device)."""
        N.check(N.lib().mk_session_compute_seq_device(self._h, in_ptr, ncalls, out_ptr, status_ptr, steps_ptr, stream),
                "mk_session_compute_seq_device")

    def reset(self):
        """/reset (master.go:126-143): every instance back to its initial state."""
        N.check(N.lib().mk_session_reset(self._h), "mk_session_reset")

    def close(self):
        if getattr(self, "_h", None):
            N.lib().mk_session_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def generate_inputs_device(n, out_ptr, *, seed, gen_kind=N.MK_GEN_FULL, gen_mask=0, offset=0, device=0, stream=None):
    N.check(N.lib().mk_generate_inputs_device(device, seed, gen_kind, gen_mask, offset, n, out_ptr, stream))


def valu_probe_device(blocks, iters, *, device=0, stream=None) -> int:
    ops = C.c_uint64()
    N.check(N.lib().mk_valu_probe_device(device, blocks, iters, C.byref(ops), stream))
    return ops.value
