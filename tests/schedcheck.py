"""ctypes binding of lib/libmisaka_amd_check.so: the host model of the tier-2
superblock executor (misaka-net_amd/csrc/sched_check.cpp), used to test the
schedule compiler against the oracle without a GPU."""
import ctypes as C
import os

import numpy as np

import misaka_net_amd as mk
from misaka_net_amd import _native as N

LIB = os.path.join(os.path.dirname(mk._native.LIB_PATH), "libmisaka_amd_check.so")
# MK_CHECK_LIB: another build of the same sources (the ASan + UBSan one,
# __graft_entry__.build_check(sanitize=True), tests/test_sanitized.py)
SAN = os.environ.get("MK_CHECK_LIB")
_lib = None


def lib():
    global _lib
    if _lib is None:
        import __graft_entry__ as g

        if SAN:
            assert os.path.exists(SAN), SAN
        else:
            g.build_check()
        h = C.CDLL(SAN or LIB)
        h.mkc_load.restype = C.c_void_p
        h.mkc_load.argtypes = [C.POINTER(N.mk_node_desc), C.c_int, C.c_char_p, C.c_size_t]
        h.mkc_free.argtypes = [C.c_void_p]
        h.mkc_emulate.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_int, C.c_void_p, C.c_size_t, C.c_void_p,
                                  C.c_void_p, C.c_void_p, C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t]
        h.mkc_jit_lane.argtypes = [C.c_void_p, C.c_uint32, C.c_int, C.c_int, C.POINTER(C.c_uint32),
                                   C.POINTER(C.c_int), C.c_char_p, C.c_size_t]
        h.mkc_tier.argtypes = [C.c_void_p, C.c_uint32, C.c_int, C.c_char_p, C.c_size_t]
        h.mkc_tokenize.argtypes = [C.c_char_p, C.c_char_p, C.c_size_t]
        _lib = h
    return _lib


class NotCompiled(Exception):
    pass


def tokenize(program: str):
    """The check library's front end (sched_check.cpp mkc_tokenize): the
    token vectors of misaka_net_amd.tokenize, or TisParseError."""
    buf = C.create_string_buffer(max(4096, 64 * len(program) + 1024))
    rc = lib().mkc_tokenize(program.encode(), buf, len(buf))
    text = buf.value.decode(errors="surrogateescape")
    if rc == -2:
        raise mk.TisParseError(text)
    assert rc == 0, rc
    return [line.split("\x1f") for line in text.split("\n")]


def _load(nodes):
    rows = [(n.name, n.kind, n.program) if hasattr(n, "name") else tuple(n) for n in nodes]
    kinds = {"program": 0, "stack": 1, "master": 2}
    arr = (N.mk_node_desc * len(rows))()
    keep = []
    for i, (nm, kd, pg) in enumerate(rows):
        a, b = nm.encode(), (pg or "").encode()
        keep += [a, b]
        arr[i].name, arr[i].kind, arr[i].program = a, kinds[kd], b
    err = C.create_string_buffer(4096)
    h = lib().mkc_load(arr, len(rows), err, len(err))
    assert h, err.value
    return h, keep


SHAPES = {0: "stream", 1: "machine"}


def jit_lane(nodes, *, stack_cap=None, stop_on_output=False, machine=False, with_shape=False):
    """(source of the native tier's lane code, stack slots per lane[, shape]).
    ``machine``: force the machine shape (resumable lane) on acyclic networks too."""
    h, _keep = _load(nodes)
    try:
        ns = C.c_uint32()
        sh = C.c_int()
        buf = C.create_string_buffer(1 << 24)
        rc = lib().mkc_jit_lane(h, 1024 if stack_cap is None else stack_cap, 1 if stop_on_output else 0,
                                1 if machine else 0, C.byref(ns), C.byref(sh), buf, len(buf))
        if rc == 1:
            raise NotCompiled(buf.value.decode())
        assert rc == 0, rc
        if with_shape:
            return buf.value.decode(), ns.value, SHAPES[sh.value]
        return buf.value.decode(), ns.value
    finally:
        lib().mkc_free(h)


def emulate(nodes, xs, *, budget=None, stack_cap=None, stop_on_output=False, want_plan=False):
    h, _keep = _load(nodes)
    try:
        v = np.ascontiguousarray(np.asarray(xs, dtype=np.int64))
        out = np.zeros(v.size, np.int32)
        st = np.zeros(v.size, np.uint8)
        sp = np.zeros(v.size, np.uint32)
        why = C.create_string_buffer(512)
        plan = C.create_string_buffer(1 << 22) if want_plan else None
        rc = lib().mkc_emulate(h, budget or (1 << 20), 1024 if stack_cap is None else stack_cap,
                               1 if stop_on_output else 0, v.ctypes.data, v.size, out.ctypes.data, st.ctypes.data,
                               sp.ctypes.data, why, len(why), plan, len(plan) if plan is not None else 0)
        if rc == 1:
            raise NotCompiled(why.value.decode())
        assert rc == 0, f"emulator error {rc}"
        return (out, st, sp, plan.value.decode() if plan is not None else None)
    finally:
        lib().mkc_free(h)


TIERS = {3: "native", 2: "compiled", 1: "interp"}


def tier(nodes, *, stack_cap=None, stop_on_output=False):
    """(tier name, shape or fallback reason) as the product picks it for the default budget."""
    h, _keep = _load(nodes)
    try:
        why = C.create_string_buffer(1024)
        t = lib().mkc_tier(h, 1024 if stack_cap is None else stack_cap, 1 if stop_on_output else 0, why, len(why))
        return TIERS[t], why.value.decode()
    finally:
        lib().mkc_free(h)


# ---- stateful sessions on the host model (tis_sched.h compile_session_schedule)

HANDOFF = 0xFE


class OrcFlat(C.Structure):
    """oracle/orc_flat.h"""
    _fields_ = [("acc", C.c_int64 * 64), ("bak", C.c_int64 * 64), ("ip", C.c_int32 * 64), ("pendv", C.c_int32 * 64),
                ("port", C.c_int32 * 256), ("pfull", C.c_uint64), ("pend", C.c_uint32), ("hung", C.c_uint32),
                ("in_full", C.c_int32), ("out_full", C.c_int32), ("in_val", C.c_int32), ("out_val", C.c_int32),
                ("depth", C.c_uint32 * 64), ("entries", C.c_void_p), ("deposited", C.c_int32), ("pin", C.c_int32),
                ("pos", C.c_int32), ("changed", C.c_int32), ("csteps", C.c_uint32)]


class HostSessions:
    """n session instances executing the session schedule's device form
    (sched_check.cpp mkc_sess_*); ``call(values)`` is one /compute on each.
    Calls that hand off report HANDOFF; ``export(i)`` is the state the
    interpreter would continue from."""

    def __init__(self, nodes, n, *, stack_cap=None):
        h = lib()
        h.mkc_sess_new.restype = C.c_void_p
        h.mkc_sess_new.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_char_p, C.c_size_t]
        h.mkc_sess_free.argtypes = [C.c_void_p]
        h.mkc_sess_call.argtypes = [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p]
        h.mkc_sess_export.argtypes = [C.c_void_p, C.c_size_t, C.POINTER(OrcFlat), C.c_void_p]
        self.cap = 1024 if stack_cap is None else stack_cap
        self._net, self._keep = _load(nodes)
        why = C.create_string_buffer(1 << 20)
        self._h = h.mkc_sess_new(self._net, self.cap, n, why, len(why))
        if not self._h:
            lib().mkc_free(self._net)
            self._net = None
            raise NotCompiled(why.value.decode())
        self.plan = why.value.decode()
        self.n = n
        self.nstack = 0

    def call(self, values, *, budget=None):
        v = np.ascontiguousarray(np.asarray(values, dtype=np.int64))
        assert v.size == self.n
        out = np.zeros(self.n, np.int32)
        st = np.zeros(self.n, np.uint8)
        sp = np.zeros(self.n, np.uint32)
        rc = lib().mkc_sess_call(self._h, v.ctypes.data, budget or (1 << 20), out.ctypes.data, st.ctypes.data,
                                 sp.ctypes.data)
        assert rc == 0, f"emulator error {rc}"
        return out, st, sp

    def export(self, i, nstack):
        f = OrcFlat()
        ent = np.zeros(max(1, nstack) * self.cap, np.int32)
        rc = lib().mkc_sess_export(self._h, i, C.byref(f), ent.ctypes.data)
        assert rc == 0, f"export error {rc}"
        f.entries = ent.ctypes.data
        return f, ent

    def __del__(self):
        if getattr(self, "_h", None):
            lib().mkc_sess_free(self._h)
            self._h = None
        if getattr(self, "_net", None):
            lib().mkc_free(self._net)
            self._net = None


def session_lane(nodes, *, stack_cap=None):
    """(session lane source of the native tier, registers, stack slots)."""
    h, _keep = _load(nodes)
    try:
        lib().mkc_sess_lane.argtypes = [C.c_void_p, C.c_uint32, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32),
                                        C.c_char_p, C.c_size_t]
        nr, ns = C.c_uint32(), C.c_uint32()
        buf = C.create_string_buffer(1 << 24)
        rc = lib().mkc_sess_lane(h, 1024 if stack_cap is None else stack_cap, C.byref(nr), C.byref(ns), buf, len(buf))
        if rc == 1:
            raise NotCompiled(buf.value.decode())
        assert rc == 0, rc
        return buf.value.decode(), nr.value, ns.value
    finally:
        lib().mkc_free(h)


def session_max_call_steps(nodes, *, stack_cap=None):
    """Longest /compute call of the session schedule (None: unbounded)."""
    h, _keep = _load(nodes)
    try:
        lib().mkc_sess_call_steps.argtypes = [C.c_void_p, C.c_uint32, C.POINTER(C.c_uint64)]
        v = C.c_uint64()
        rc = lib().mkc_sess_call_steps(h, 1024 if stack_cap is None else stack_cap, C.byref(v))
        if rc == 1:
            raise NotCompiled("session schedule declined")
        assert rc == 0, rc
        return None if v.value == (1 << 64) - 1 else v.value
    finally:
        lib().mkc_free(h)


def session_module(nodes, *, stack_cap=None):
    """The native session module's full source (what hiprtc compiles)."""
    h, _keep = _load(nodes)
    try:
        lib().mkc_sess_module.argtypes = [C.c_void_p, C.c_uint32, C.c_char_p, C.c_size_t]
        buf = C.create_string_buffer(1 << 24)
        rc = lib().mkc_sess_module(h, 1024 if stack_cap is None else stack_cap, buf, len(buf))
        if rc == 1:
            raise NotCompiled(buf.value.decode())
        assert rc == 0, rc
        return buf.value.decode()
    finally:
        lib().mkc_free(h)


# ---- test tool: a standalone hiprtc compiler (tests/native/rtc_compile.cpp)

_TOOL_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "native")


def rtc_tool():
    """Path of the built test compiler (this ROCm's hiprtc in a process of its
    own that never loads PyTorch); rebuilt when its source changes."""
    import hashlib
    import subprocess

    src = os.path.join(_TOOL_DIR, "rtc_compile.cpp")
    out = os.path.join(_TOOL_DIR, "build", "rtc_compile")
    cmd = ["g++", "-O2", "-std=c++17", "-Wall", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include", src,
           "-L/opt/rocm/lib", "-lhiprtc", "-Wl,-rpath,/opt/rocm/lib"]
    with open(src, "rb") as f:
        stamp = hashlib.sha256(f.read() + " ".join(cmd).encode()).hexdigest()
    try:
        with open(out + ".stamp") as f:
            if f.read().strip() == stamp and os.path.exists(out):
                return out
    except OSError:
        pass
    os.makedirs(os.path.dirname(out), exist_ok=True)
    tmp = f"{out}.tmp{os.getpid()}"
    subprocess.check_call(cmd + ["-o", tmp])
    os.replace(tmp, out)
    with open(out + ".stamp", "w") as f:
        f.write(stamp + "\n")
    return out
