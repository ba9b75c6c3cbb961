"""ctypes binding of the C ABI declared in include/mk.h.

The shared library is built in-tree (``misaka-net_amd/lib/libmisaka_amd.so``,
see ``__graft_entry__.build``).  There is no fallback: if the library is
missing every entry point raises, so a GPU run can never silently take a
CPU path.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libmisaka_amd.so")

MK_OK = 0
MK_EINVAL = -1
MK_EPARSE = -2
MK_ELIMIT = -3
MK_EDEVICE = -4
MK_ENOMEM = -5
MK_EBUSY = -6

MK_ST_QUIESCENT = 1
MK_ST_BUDGET = 2
MK_ST_STACK_OVERFLOW = 3
MK_ST_OUTPUT_STOP = 4
MK_ST_REMOTE_WAIT = 5
MK_ST_CALL_OPEN = 6
MK_ST_REASON_MASK = 0x0F
MK_ST_HAS_OUTPUT = 0x10

MK_NODE_PROGRAM = 0
MK_NODE_STACK = 1
MK_NODE_MASTER = 2
MK_NODE_REMOTE_PROGRAM = 3
MK_NODE_REMOTE_STACK = 4
MK_REMOTE_SEND = 0
MK_REMOTE_PUSH = 1
MK_REMOTE_POP = 2

MK_FLAG_STOP_ON_OUTPUT = 1
MK_FLAG_FORCE_INTERP = 2
MK_FLAG_TILE = 4
MK_FLAG_REFILL = 8
MK_FLAG_JIT = 16
MK_FLAG_DEFER_STATS = 32

MK_IN_I64 = 0
MK_IN_I32 = 1
MK_IN_GEN = 2
MK_GEN_FULL = 0
MK_GEN_MASKED = 1
MK_STATS_LEN = 8

ERROR_NAMES = {
    MK_EINVAL: "MK_EINVAL",
    MK_EPARSE: "MK_EPARSE",
    MK_ELIMIT: "MK_ELIMIT",
    MK_EDEVICE: "MK_EDEVICE",
    MK_ENOMEM: "MK_ENOMEM",
    MK_EBUSY: "MK_EBUSY",
}


class mk_node_desc(C.Structure):
    _fields_ = [("name", C.c_char_p), ("kind", C.c_int), ("program", C.c_char_p)]


class mk_opts(C.Structure):
    _fields_ = [
        ("budget", C.c_uint32),
        ("stack_cap", C.c_uint32),
        ("flags", C.c_uint32),
        ("device_mask", C.c_uint32),
    ]


class mk_remote_req(C.Structure):
    _fields_ = [("node", C.c_uint32), ("op", C.c_uint32), ("remote", C.c_uint32), ("reg", C.c_uint32),
                ("value", C.c_int32)]


class mk_input(C.Structure):
    _fields_ = [
        ("kind", C.c_int),
        ("data", C.c_void_p),
        ("seed", C.c_uint64),
        ("gen_kind", C.c_uint32),
        ("gen_mask", C.c_uint32),
        ("offset", C.c_uint64),
    ]


# name -> (restype, argtypes); every symbol include/mk.h declares.
SIGNATURES = {
    "mk_net_load": (C.c_int, [C.POINTER(mk_node_desc), C.c_int, C.POINTER(C.c_void_p), C.c_char_p, C.c_size_t]),
    "mk_net_free": (None, [C.c_void_p]),
    "mk_compute_batch": (
        C.c_int,
        [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p, C.c_void_p, C.POINTER(mk_opts)],
    ),
    "mk_compute_device": (
        C.c_int,
        [
            C.c_void_p,
            C.c_int,
            C.POINTER(mk_input),
            C.c_size_t,
            C.c_void_p,
            C.c_void_p,
            C.c_void_p,
            C.c_void_p,
            C.POINTER(mk_opts),
            C.c_void_p,
        ],
    ),
    "mk_stats_fold": (C.c_int, [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]),
    "mk_session_create": (C.c_int, [C.c_void_p, C.c_int, C.c_size_t, C.POINTER(mk_opts), C.POINTER(C.c_void_p)]),
    "mk_session_compute": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "mk_session_compute_seq": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p, C.c_void_p]),
    "mk_session_compute_device": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "mk_session_compute_seq_device": (
        C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "mk_session_reset": (C.c_int, [C.c_void_p]),
    "mk_session_cancel": (C.c_int, [C.c_void_p]),
    "mk_session_plan": (C.c_int, [C.c_void_p, C.c_char_p, C.c_size_t]),
    "mk_session_free": (None, [C.c_void_p]),
    "mk_generate_inputs_device": (
        C.c_int,
        [C.c_int, C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint64, C.c_size_t, C.c_void_p, C.c_void_p],
    ),
    "mk_tokenize": (C.c_int, [C.c_char_p, C.c_char_p, C.c_size_t]),
    "mk_net_disasm": (C.c_int, [C.c_void_p, C.c_char_p, C.c_size_t]),
    "mk_net_info": (C.c_int, [C.c_void_p, C.POINTER(C.c_int)]),
    "mk_net_plan": (C.c_int, [C.c_void_p, C.POINTER(mk_opts), C.c_char_p, C.c_size_t]),
    "mk_net_sched_disasm": (C.c_int, [C.c_void_p, C.POINTER(mk_opts), C.c_char_p, C.c_size_t]),
    "mk_net_prepare": (C.c_int, [C.c_void_p, C.POINTER(mk_opts), C.c_int]),
    "mk_net_jit_source": (C.c_int, [C.c_void_p, C.POINTER(mk_opts), C.c_char_p, C.c_size_t]),
    "mk_valu_probe_device": (C.c_int, [C.c_int, C.c_int, C.c_int, C.POINTER(C.c_uint64), C.c_void_p]),
    "mk_session_step": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "mk_session_remote_poll": (C.c_int, [C.c_void_p, C.c_size_t, C.POINTER(mk_remote_req), C.c_int,
                                         C.POINTER(C.c_int)]),
    "mk_session_remote_done": (C.c_int, [C.c_void_p, C.c_size_t, C.c_uint32, C.c_int32]),
    "mk_session_port_put": (C.c_int, [C.c_void_p, C.c_size_t, C.c_uint32, C.c_uint32, C.c_int32]),
    "mk_session_stack_push": (C.c_int, [C.c_void_p, C.c_size_t, C.c_uint32, C.c_int32]),
    "mk_session_stack_pop": (C.c_int, [C.c_void_p, C.c_size_t, C.c_uint32, C.POINTER(C.c_int32)]),
    "mk_session_input_take": (C.c_int, [C.c_void_p, C.c_size_t, C.POINTER(C.c_int32)]),
    "mk_session_output_put": (C.c_int, [C.c_void_p, C.c_size_t, C.c_int32]),
    "mk_net_node_index": (C.c_int, [C.c_void_p, C.c_char_p, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "mk_trace_lane": (C.c_int, [C.c_void_p, C.c_int, C.c_int64, C.POINTER(mk_opts), C.c_void_p, C.c_uint32,
                                C.POINTER(C.c_uint32), C.POINTER(C.c_uint8)]),
    "mk_version": (C.c_char_p, []),
}

_lib = None
_lock = threading.Lock()


class NativeLibraryMissing(RuntimeError):
    pass


def lib() -> C.CDLL:
    """Load libmisaka_amd.so (raises NativeLibraryMissing if it was not built)."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise NativeLibraryMissing(
                    f"{LIB_PATH} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'`"
                )
            h = C.CDLL(LIB_PATH)
            for name, (res, args) in SIGNATURES.items():
                fn = getattr(h, name)
                fn.restype = res
                fn.argtypes = args
            _lib = h
        return _lib


class MkError(RuntimeError):
    def __init__(self, code: int, msg: str = ""):
        self.code = code
        super().__init__(f"{ERROR_NAMES.get(code, code)}: {msg}" if msg else ERROR_NAMES.get(code, str(code)))


def check(rc: int, what: str = "") -> None:
    if rc != MK_OK:
        raise MkError(rc, what)
