"""Stateful sessions compiled by the schedule compiler (row f2 on the native
tier; tis_sched.h compile_session_schedule), executed by the host model of
its device form (sched_check.cpp mkc_sess_*) and checked, call by call,
against the oracle's session restatement (tis_oracle.c session_step).

A call that would reach its budget slice inside a superblock is handed off
(U_HANDOFF): the host model exports the instance's state in the
interpreter's terms (sess_convert.h) and the oracle, importing it, must
finish that call and every later one exactly as the oracle's own run does.
CPU only."""
import os

import numpy as np
import pytest

import misaka_net_amd as mk
from oracle import pyoracle as po
import schedcheck as sc
from misaka_net_amd import _native as N
from schedcheck import HANDOFF, HostSessions, NotCompiled
from tisgen import random_network, stack_loop_network

CALLS = 6


def _nstack(nodes):
    return sum(1 for n in nodes if (n.kind if hasattr(n, "name") else n[1]) == "stack")


def run_pair(nodes, n, *, budget=None, stack_cap=None, seed=1, calls=CALLS, resumes=3, kind=0, mask=0):
    """Returns (calls checked, hand-offs seen)."""
    host = HostSessions(nodes, n, stack_cap=stack_cap)
    ref = po.OracleSessions(po.OracleNet(nodes), n, stack_cap=stack_cap)
    probes = {}  # lane -> (oracle instance finishing it, keep-alive)
    checked = handoffs = 0
    b = budget or (1 << 20)
    for k in range(calls):
        row = po.gen_inputs(seed * 7919 + k, n, kind=kind, mask=mask)
        ho, hs, hp = host.call(row, budget=b)
        ro, rs, rp = ref.compute(row, budget=b)
        for i in range(n):
            if i in probes:
                po_, _keep = probes[i]
                got = tuple(int(a[0]) for a in po_.compute([row[i]], budget=b))
            elif hs[i] == HANDOFF:
                flat, ent = host.export(i, _nstack(nodes))
                po_ = po.OracleSessions(po.OracleNet(nodes), 1, stack_cap=stack_cap)
                po_.import_state(0, flat)
                probes[i] = (po_, (flat, ent))
                got = tuple(int(a[0]) for a in po_.resume(budget=b))
                handoffs += 1
            else:
                got = (int(ho[i]), int(hs[i]), int(hp[i]))
            assert got == (int(ro[i]), int(rs[i]), int(rp[i])), (k, i, int(row[i]), got, (ro[i], rs[i], rp[i]))
            checked += 1
        # open calls (handed-off lanes only) get more slices, then are cancelled
        for _ in range(resumes):
            ro, rs, rp = ref.resume(budget=b)
            for i, (po_, _keep) in probes.items():
                got = tuple(int(a[0]) for a in po_.resume(budget=b))
                assert got == (int(ro[i]), int(rs[i]), int(rp[i])), ("resume", k, i, got)
            for i in range(n):
                if i not in probes:
                    assert rs[i] in (0, po.ST_STACK_OVERFLOW), ("a native lane left a call open", k, i)
        ref.cancel()
        for po_, _keep in probes.values():
            po_.cancel()
    return checked, handoffs


def test_example_network_sessions():
    nodes = mk.networks.example_network()
    host = HostSessions(nodes, 4)
    out, st, sp = host.call([5, 2147483647, -3, 4294967301])
    assert out.tolist() == [7, -2147483647, -1, 7] and (st == 0x10).all() and (sp == 11).all()
    out, st, sp = host.call([1, 2, 3, 4])
    assert out.tolist() == [3, 4, 5, 6] and (sp == 12).all()
    run_pair(nodes, 64)


@pytest.mark.parametrize("name", ["sample", "countdown", "pipeline8"])
def test_config_networks(name):
    nodes = {"sample": mk.networks.sample_network, "countdown": mk.networks.countdown_network,
             "pipeline8": lambda: mk.networks.pipeline_network(8)}[name]()
    kind, mask = (1, 1023) if name == "countdown" else (0, 0)
    run_pair(nodes, 48, kind=kind, mask=mask)
    # small budget slices: the long calls hand off and the oracle finishes them
    _, h = run_pair(nodes, 48, budget=60, kind=kind, mask=mask)
    if name == "countdown":
        assert h > 0


def test_state_that_persists():
    # running sum, second output returned by the next call, quiescent calls
    run_pair([("n", "program", "IN NIL\nADD 10\nOUT ACC")], 8)
    run_pair([("n", "program", "IN ACC\nOUT ACC\nOUT ACC")], 8)
    run_pair([("n", "program", "IN ACC\nJEZ Z\nOUT ACC\nZ: NOP")], 16, kind=1, mask=3)
    run_pair([("n", "program", "IN ACC\nPUSH ACC, s\nPOP s, ACC\nPUSH ACC, s\nOUT ACC"), ("s", "stack", "")], 8,
             stack_cap=3)


def test_long_call_hands_off_mid_loop():
    nodes = [("n", "program", "IN ACC\nL: SUB 1\nJGZ L\nOUT ACC")]
    host = HostSessions(nodes, 2)
    out, st, sp = host.call([3, 5000], budget=1000)
    assert st[0] == 0x10 and st[1] == HANDOFF
    checked, h = run_pair(nodes, 32, budget=500, kind=1, mask=1023)
    assert h > 0


@pytest.mark.parametrize("seed", range(150))
def test_random_networks(seed):
    nodes = random_network(seed)
    cap = [1, 3, 8, 16, 17, 40, 1024][seed % 7]
    try:
        run_pair(nodes, 24, budget=[37, 200, 1000, 5000][seed % 4], stack_cap=cap, seed=seed)
    except NotCompiled:
        pytest.skip("not compilable")


@pytest.mark.parametrize("seed", range(60))
def test_stack_loop_networks(seed):
    nodes, gen = stack_loop_network(seed)
    try:
        run_pair(nodes, 24, budget=[100, 2000, 6000][seed % 3], stack_cap=[16, 40, 1024][seed % 3], seed=seed,
                 kind=gen.get("kind", 0), mask=gen.get("mask", 0))
    except NotCompiled:
        pytest.skip("not compilable")


# ---- the generated session lane (tis_jit.cpp, machine shape) compiled with g++,
# driven like mk_sess_exec drives it, against the host model call by call

SESS_HEADER = """#include <cstdint>
#include <cstddef>
#define MK_FN static inline
#define MK_LOOP_NEED(pol) 0u
#define MK_KEEP(m, need) (m)
#define MK_ALL(p) (p)
#define MK_SLOT_ST(b, ss, s, v) ((b)[(uint64_t)(s) * (ss)] = (v))
#define MK_SLOT_LD(b, ss, s) ((b)[(uint64_t)(s) * (ss)])
#define MK_SLOT_STX(b, ss, s, v) ((b)[(uint64_t)(s) * (ss)] = (v))
#define MK_SLOT_LDX(b, ss, s) ((b)[(uint64_t)(s) * (ss)])
#define MK_FLAG_GT(x) ((int32_t)((x) > 0))
#define MK_FLAG_LT(x) ((int32_t)((x) < 0))
#define MK_FLAG_NZ(x) ((int32_t)((x) != 0))
#define MK_FLAG_MIN(x, f) ((int32_t)((uint32_t)(x) < (uint32_t)(f) ? (uint32_t)(x) : (uint32_t)(f)))
#define MK_MAD24(f, k, x) ((int32_t)((uint32_t)(x) + (uint32_t)(f) * (uint32_t)(k)))
#define MK_SATDEC(x) ((int32_t)((uint32_t)(x) ? (uint32_t)(x) - 1u : 0u))
#define MK_OPAQUE1() 1u
#define MK_SATSUB(x, o) ((int32_t)((uint32_t)(x) >= (o) ? (uint32_t)(x) - (o) : 0u))
"""

SESS_DRIVER = """
extern "C" void sessrun{i}(size_t n, uint32_t budget, const int64_t *in, int32_t *out, uint8_t *st, uint32_t *sp,
                          uint32_t *sb, int64_t *regs, int32_t *slots) {{
    using namespace n{i};
    for (size_t s = 0; s < n; s++) {{
        MkLane L;
        mk_sess_load(L, regs, s, n, sb[s] < MK_SS_DEAD);
        out[s] = 0; sp[s] = 0;
        if (sb[s] == MK_SS_DEAD) {{ st[s] = 3; continue; }}
        if (sb[s] >= MK_SS_DEAD) {{ st[s] = 0xFE; continue; }}
        L.sb = sb[s]; L.steps = 0; L.st = 0; L.outv = 0; L.next = MK_SS_DEAD;
        mk_sess_input(L, (int64_t)(int32_t)in[s]);
        while (L.sb < MK_SB_DONE) mk_run(L.sb, L, budget, slots + s, n, 0u, L.steps);
        if (L.st == MK_SS_HANDOFF) {{ st[s] = 0xFE; sp[s] = L.steps; sb[s] = MK_SS_HAND; }}
        else {{ out[s] = (L.st & 0x10) ? L.outv : 0; st[s] = (uint8_t)L.st; sp[s] = L.steps; sb[s] = L.next; }}
        mk_sess_store(L, regs, s, n);
    }}
}}
"""


def _build_sessions(cases, path):
    import ctypes as C
    import subprocess

    parts = [SESS_HEADER]
    for i, (src, _nr, _ns) in enumerate(cases):
        parts.append(f"namespace n{i} {{\n{src}\n}}\n")
        parts.append(SESS_DRIVER.format(i=i))
    with open(path + ".cpp", "w") as f:
        f.write("".join(parts))
    subprocess.check_call(["g++", "-O1", "-std=c++17", "-shared", "-fPIC", "-w", "-o", path + ".so", path + ".cpp"])
    return C.CDLL(path + ".so")


def test_generated_session_lane(tmp_path):
    import schedcheck as sc

    nets = [("example", mk.networks.example_network(), {}, (0, 0)),
            ("sample", mk.networks.sample_network(), {}, (0, 0)),
            ("countdown", mk.networks.countdown_network(), {"budget": 700}, (1, 1023)),
            ("pipeline8", mk.networks.pipeline_network(8), {}, (0, 0)),
            ("sum", [("n", "program", "IN NIL\nADD 10\nOUT ACC")], {}, (0, 0)),
            ("twice", [("n", "program", "IN ACC\nOUT ACC\nOUT ACC")], {}, (0, 0)),
            ("ovf", [("n", "program", "IN ACC\nPUSH ACC, s\nPOP s, ACC\nPUSH ACC, s\nOUT ACC"), ("s", "stack", "")],
             {"stack_cap": 3}, (0, 0))]
    for seed in range(30):
        nets.append((f"rand{seed}", random_network(seed), {"budget": [37, 200, 1000][seed % 3],
                                                          "stack_cap": [1, 3, 8, 16, 17, 40, 1024][seed % 7]}, (0, 0)))
    for seed in range(12):
        rows, gen = stack_loop_network(seed)
        nets.append((f"stk{seed}", rows, {"budget": [100, 2000][seed % 2]}, (gen["kind"], gen["mask"])))
    cases, keep = [], []
    for label, nodes, kw, gen in nets:
        try:
            cases.append(sc.session_lane(nodes, stack_cap=kw.get("stack_cap")))
            keep.append((label, nodes, kw, gen))
        except NotCompiled:
            pass
    lib = _build_sessions(cases, str(tmp_path / "sess"))
    import ctypes as C

    n = 16
    for i, ((label, nodes, kw, gen), (src, nr, ns)) in enumerate(zip(keep, cases)):
        host = HostSessions(nodes, n, stack_cap=kw.get("stack_cap"))
        sb = np.zeros(n, np.uint32)
        regs = np.zeros(max(1, nr) * n, np.int64)
        slots = np.full(max(1, ns) * n, 0x5A5A5A5A, np.int32)
        b = kw.get("budget") or (1 << 20)
        for k in range(5):
            row = po.gen_inputs(k * 31 + i, n, kind=gen[0], mask=gen[1])
            ref = host.call(row, budget=b)
            out, st, sp = np.zeros(n, np.int32), np.zeros(n, np.uint8), np.zeros(n, np.uint32)
            getattr(lib, f"sessrun{i}")(C.c_size_t(n), C.c_uint32(b), C.c_void_p(row.ctypes.data),
                                        C.c_void_p(out.ctypes.data), C.c_void_p(st.ctypes.data),
                                        C.c_void_p(sp.ctypes.data), C.c_void_p(sb.ctypes.data),
                                        C.c_void_p(regs.ctypes.data), C.c_void_p(slots.ctypes.data))
            for a, r in zip((out, st, sp), ref):
                bad = np.nonzero(a != r)[0]
                assert not bad.size, (label, k, int(bad[0]), int(a[bad[0]]), int(r[bad[0]]))


def test_session_modules_compile_for_gfx950(tmp_path):
    # the whole module (lane + mk_sess_exec) through this ROCm's hiprtc, as
    # the loader compiles it (the standalone test compiler; no GPU needed)
    import subprocess

    import schedcheck as sc

    rtc = sc.rtc_tool()
    for name, nodes in [("example", mk.networks.example_network()), ("countdown", mk.networks.countdown_network()),
                        ("pipeline64", mk.networks.pipeline_network(64)), ("rand3", random_network(3))]:
        src = sc.session_module(nodes)
        p = tmp_path / f"{name}.hip"
        p.write_text(src)
        r = subprocess.run([rtc, str(p), str(tmp_path / f"{name}.co")], capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, (name, r.stdout[-2000:])
        assert (tmp_path / f"{name}.co").stat().st_size > 0


def test_session_call_bound_covers_every_call():
    """jit_session_max_call_steps (tis_jit.cpp): a network whose calls cannot
    loop gets a bound on any call's retired steps, which the session
    launches use to skip the interpreter pass (no call can hand off below
    it).  Every emulated call -- sequential calls on 64 instances, full-range
    inputs -- retires at most the bound; networks with data-dependent loops
    are unbounded."""
    bounded = {"example": mk.networks.example_network(), "sample": mk.networks.sample_network(),
               "pipeline4": mk.networks.pipeline_network(4)}
    for seed in range(12):
        bounded[f"rand{seed}"] = random_network(seed)
    seen_bounded = 0
    for name, nodes in bounded.items():
        try:
            bound = sc.session_max_call_steps(nodes)
        except sc.NotCompiled:
            continue
        if bound is None:
            continue
        seen_bounded += 1
        emu = sc.HostSessions(nodes, 64)
        for call in range(6):
            _, _, sp = emu.call(po.gen_inputs(0x4D49534B41 + call, 64))
            assert int(sp.max()) <= bound, (name, call, int(sp.max()), bound)
        # the condition the one-launch shortcut relies on (mk_exec.hip session
        # launch: call_steps < budget): at budget = bound + 1 neither the
        # budget guard nor a round end fires, so no call hands off to the
        # interpreter or stops on the budget
        tight = sc.HostSessions(nodes, 64)
        for call in range(6):
            _, st, sp = tight.call(po.gen_inputs(0x4D49534B41 + call, 64), budget=bound + 1)
            assert not (st == sc.HANDOFF).any(), (name, call, "handed off below the bound")
            assert not ((st & N.MK_ST_REASON_MASK) == N.MK_ST_BUDGET).any(), (name, call, "budget stop")
            assert int(sp.max()) <= bound
    assert seen_bounded >= 3
    assert sc.session_max_call_steps(mk.networks.countdown_network()) is None
    assert sc.session_max_call_steps(mk.networks.example_network()) is not None
