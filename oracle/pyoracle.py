"""ctypes binding of the C oracle (oracle/tis_oracle.c).

TEST INFRASTRUCTURE ONLY -- the parity checker.  Imported by tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg; never by the product
package (misaka-net_amd/).  See tis_oracle.c's header for what pins it.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
from typing import Optional, Sequence

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "tis_oracle.c")
LIB = os.path.join(HERE, "build", "liboracle_tis.so")

ST_QUIESCENT, ST_BUDGET, ST_STACK_OVERFLOW, ST_OUTPUT_STOP, ST_HAS_OUTPUT = 1, 2, 3, 4, 0x10
ST_CALL_OPEN = 6
KIND = {"program": 0, "stack": 1}


def build(force: bool = False) -> str:
    """Compile the oracle with gcc (no GPU needed)."""
    import hashlib

    h = hashlib.sha256()
    for src in (SRC, os.path.join(os.path.dirname(SRC), "orc_flat.h")):
        with open(src, "rb") as f:
            h.update(f.read())
    stamp = h.hexdigest()  # content, not mtime: the tree travels to the GPU box
    try:
        with open(LIB + ".stamp") as f:
            fresh = os.path.exists(LIB) and f.read().strip() == stamp
    except OSError:
        fresh = False
    if force or not fresh:
        os.makedirs(os.path.dirname(LIB), exist_ok=True)
        tmp = f"{LIB}.tmp{os.getpid()}"
        subprocess.check_call(["gcc", "-O2", "-std=c11", "-Wall", "-shared", "-fPIC", "-pthread", "-o", tmp, SRC])
        os.replace(tmp, LIB)
        with open(LIB + ".stamp", "w") as f:
            f.write(stamp + "\n")
    return LIB


_lib = None


def lib():
    global _lib
    if _lib is None:
        build()
        h = C.CDLL(LIB)
        h.orc_tokenize.argtypes = [C.c_char_p, C.c_char_p, C.c_size_t]
        h.orc_label_map.argtypes = [C.c_char_p, C.c_char_p, C.c_size_t]
        h.orc_net_load.restype = C.c_void_p
        h.orc_net_load.argtypes = [
            C.c_int,
            C.POINTER(C.c_char_p),
            C.POINTER(C.c_int),
            C.POINTER(C.c_char_p),
            C.c_char_p,
            C.c_char_p,
            C.c_size_t,
        ]
        h.orc_net_free.argtypes = [C.c_void_p]
        h.orc_compute_batch.argtypes = [
            C.c_void_p,
            C.c_void_p,
            C.c_size_t,
            C.c_void_p,
            C.c_void_p,
            C.c_void_p,
            C.c_uint32,
            C.c_uint32,
            C.c_int,
            C.c_int,
        ]
        h.orc_gen_inputs.argtypes = [C.c_uint64, C.c_int, C.c_uint32, C.c_uint64, C.c_size_t, C.c_void_p]
        h.orc_sessions_new.restype = C.c_void_p
        h.orc_sessions_new.argtypes = [C.c_void_p, C.c_size_t, C.c_uint32]
        h.orc_sessions_free.argtypes = [C.c_void_p]
        h.orc_sessions_reset.argtypes = [C.c_void_p]
        h.orc_sessions_cancel.argtypes = [C.c_void_p]
        h.orc_session_import.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p]
        h.orc_sessions_compute.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32,
                                           C.c_int]
        h.orc_go_atoi.argtypes = [C.c_char_p, C.c_size_t, C.POINTER(C.c_int64)]
        h.orc_trace_lane.argtypes = [C.c_void_p, C.c_int64, C.c_uint32, C.c_uint32, C.c_int, C.c_void_p, C.c_uint32,
                                     C.POINTER(C.c_uint32)]
        _lib = h
    return _lib


class OracleParseError(ValueError):
    pass


def tokenize(program: str) -> list[list[str]]:
    buf = C.create_string_buffer(max(4096, 64 * len(program) + 1024))
    rc = lib().orc_tokenize(program.encode(), buf, len(buf))
    text = buf.value.decode(errors="surrogateescape")
    if rc == -1:
        raise OracleParseError(text)
    assert rc == 0, "token buffer too small"
    return [line.split("\x1f") for line in text.split("\n")]


def label_map(program: str) -> dict:
    buf = C.create_string_buffer(1 << 16)
    rc = lib().orc_label_map(program.encode(), buf, len(buf))
    if rc == -1:
        raise OracleParseError(buf.value.decode())
    out = {}
    for line in buf.value.decode().splitlines():
        k, v = line.rsplit("=", 1)
        out[k] = int(v)
    return out


def go_atoi(s: str):
    """strconv.Atoi restatement: returns int or raises ValueError."""
    v = C.c_int64()
    b = s.encode()
    rc = lib().orc_go_atoi(b, len(b), C.byref(v))
    if rc:
        raise ValueError(f"strconv.Atoi: parsing {s!r}: {'invalid syntax' if rc == 1 else 'value out of range'}")
    return v.value


class OracleNet:
    """nodes: sequence of objects with .name/.kind/.program (or tuples)."""

    def __init__(self, nodes: Sequence):
        rows = [(n.name, n.kind, n.program) if hasattr(n, "name") else tuple(n) for n in nodes]
        master = [r[0] for r in rows if r[1] == "master"]
        rows = [r for r in rows if r[1] != "master"]
        n = len(rows)
        names = (C.c_char_p * n)(*[r[0].encode() for r in rows])
        kinds = (C.c_int * n)(*[KIND[r[1]] for r in rows])
        progs = (C.c_char_p * n)(*[(r[2] or "").encode() for r in rows])
        err = C.create_string_buffer(8192)
        h = lib().orc_net_load(n, names, kinds, progs, master[0].encode() if master else None, err, len(err))
        if not h:
            raise OracleParseError(err.value.decode(errors="surrogateescape"))
        self._h = h

    def __del__(self):
        if getattr(self, "_h", None):
            lib().orc_net_free(self._h)
            self._h = None

    def compute_batch(self, values, *, budget: Optional[int] = None, stack_cap: Optional[int] = None,
                      stop_on_output: bool = False, threads: int = 1):
        v = np.ascontiguousarray(np.asarray(values, dtype=np.int64))
        n = v.size
        out = np.zeros(n, np.int32)
        st = np.zeros(n, np.uint8)
        sp = np.zeros(n, np.uint32)
        rc = lib().orc_compute_batch(
            self._h,
            v.ctypes.data_as(C.c_void_p),
            n,
            out.ctypes.data_as(C.c_void_p),
            st.ctypes.data_as(C.c_void_p),
            sp.ctypes.data_as(C.c_void_p),
            budget or (1 << 20),
            1024 if stack_cap is None else stack_cap,
            1 if stop_on_output else 0,
            threads,
        )
        assert rc == 0
        return out, st, sp


TRACE_DTYPE = np.dtype([("round", "<u4"), ("node", "<u2"), ("ip", "<u2"), ("acc", "<i8"), ("bak", "<i8")])


def trace_lane(net: "OracleNet", x: int, *, max_entries: int = 4096, budget: Optional[int] = None,
               stack_cap: Optional[int] = None, stop_on_output: bool = False):
    """Every retired instruction of the lane for input x (round, node, ip,
    acc, bak after it), first max_entries of them, and the lane's status."""
    out = np.zeros(max_entries, TRACE_DTYPE)
    cnt = C.c_uint32()
    st = lib().orc_trace_lane(net._h, int(x), budget or (1 << 20), 1024 if stack_cap is None else stack_cap,
                              1 if stop_on_output else 0, out.ctypes.data_as(C.c_void_p), max_entries, C.byref(cnt))
    return out[: cnt.value], st


class OracleSessions:
    """n stateful network instances (row f2): each compute() is one /compute
    call on every instance; state persists between calls (see tis_oracle.c)."""

    def __init__(self, net: OracleNet, n: int, *, stack_cap: Optional[int] = None):
        self._net = net  # keeps the network alive
        self.n = n
        self._h = lib().orc_sessions_new(net._h, n, 1024 if stack_cap is None else stack_cap)

    def __del__(self):
        if getattr(self, "_h", None):
            lib().orc_sessions_free(self._h)
            self._h = None

    def reset(self):
        lib().orc_sessions_reset(self._h)

    def compute(self, values, *, budget: Optional[int] = None, threads: int = 1):
        """One /compute call per instance (``values`` None: one more slice
        of every open call, tis_oracle.c session_step)."""
        if values is None:
            vp = None
        else:
            v = np.ascontiguousarray(np.asarray(values, dtype=np.int64))
            assert v.size == self.n
            vp = v.ctypes.data_as(C.c_void_p)
        out = np.zeros(self.n, np.int32)
        st = np.zeros(self.n, np.uint8)
        sp = np.zeros(self.n, np.uint32)
        rc = lib().orc_sessions_compute(self._h, vp, out.ctypes.data_as(C.c_void_p),
                                        st.ctypes.data_as(C.c_void_p), sp.ctypes.data_as(C.c_void_p),
                                        budget or (1 << 20), threads)
        assert rc == 0
        return out, st, sp

    def resume(self, *, budget: Optional[int] = None, threads: int = 1):
        return self.compute(None, budget=budget, threads=threads)

    def cancel(self):
        """Abandon every open call (the master answered it 504)."""
        lib().orc_sessions_cancel(self._h)

    def import_state(self, i, flat):
        """Instance i takes a handed-off state (orc_flat.h: a ctypes
        structure, its entries buffer kept alive by the caller) with its
        call open; the next resume() finishes that call."""
        assert lib().orc_session_import(self._h, i, C.addressof(flat)) == 0


def gen_inputs(seed: int, n: int, *, kind: int = 0, mask: int = 0, offset: int = 0) -> np.ndarray:
    out = np.zeros(n, np.int64)
    lib().orc_gen_inputs(seed, kind, mask, offset, n, out.ctypes.data_as(C.c_void_p))
    return out
