"""Tier 3 (native kernel per network, misaka-net_amd/csrc/tis_jit.cpp) on CPU.

The generator emits the lane function as portable C++; here it is compiled
with g++ (all networks of a case list into one shared object) and run lane by
lane against the oracle -- bit-exact out/status/steps.  The GPU runs the same
function inside the hiprtc-compiled kernel (tests/test_gpu_parity.py, mode
"jit"); that the full module compiles for gfx950 is checked here too (hiprtc
needs no GPU)."""
import ctypes as C
import os
import subprocess

import numpy as np
import pytest

import misaka_net_amd as mk
from misaka_net_amd.network import NodeSpec
from oracle import pyoracle as po
import schedcheck as sc
from tisgen import census_classes, stack_loop_network, loop_cases, random_network

SEED = 0x4D49534B41

HEADER = """#include <cstdint>
#include <cstddef>
#include <vector>
#define MK_FN static inline
#define MK_LANE_CHECKED 1
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


def build_lanes(cases, path):
    """cases: [(lane source, nslots)] -> CDLL exporting run<i>(in, n, budget, out, st, steps)."""
    parts = [HEADER]
    for i, (src, nslots) in enumerate(cases):
        parts.append(f"namespace n{i} {{\n{src}\n}}\n")
        parts.append(
            f'extern "C" void run{i}(const int64_t *in, size_t n, uint32_t budget, int32_t *out, uint8_t *st,'
            f" uint32_t *sp) {{\n"
            f"    std::vector<int32_t> slots({nslots} + 1, 0x5A5A5A5A);\n"
            f"    for (size_t i = 0; i < n; i++) {{\n"
            f"        uint32_t s, t;\n"
            f"#if MK_JIT_MACHINE == 0\n"  # the kernel's dispatch: unguarded lane when no path reaches the budget
            f"        const int32_t o = budget > MK_MAX_STEPS ? n{i}::mk_lane_ng(in[i], budget, slots.data(), 1, &s, &t)\n"
            f"                                                : n{i}::mk_lane(in[i], budget, slots.data(), 1, &s, &t);\n"
            f"#else\n"
            f"        const int32_t o = n{i}::mk_lane(in[i], budget, slots.data(), 1, &s, &t);\n"
            f"#endif\n"
            f"        out[i] = (t & 0x10) ? o : 0; st[i] = (uint8_t)t; sp[i] = s;\n"
            f"    }}\n}}\n")
    src = path + ".cpp"
    with open(src, "w") as f:
        f.write("".join(parts))
    so = path + ".so"
    subprocess.check_call(["g++", "-O1", "-std=c++17", "-shared", "-fPIC", "-w", "-o", so, src])
    return C.CDLL(so)


def run_lane(lib, i, xs, budget):
    v = np.ascontiguousarray(np.asarray(xs, dtype=np.int64))
    out = np.zeros(v.size, np.int32)
    st = np.zeros(v.size, np.uint8)
    sp = np.zeros(v.size, np.uint32)
    getattr(lib, f"run{i}")(C.c_void_p(v.ctypes.data), C.c_size_t(v.size), C.c_uint32(budget),
                            C.c_void_p(out.ctypes.data), C.c_void_p(st.ctypes.data), C.c_void_p(sp.ctypes.data))
    return out, st, sp


def check_cases(tmp_path, cases, machine=False):
    """cases: [(label, nodes, xs, kw)] -- every case compiled and compared.
    ``machine``: the resumable (machine-shape) lane for every case."""
    srcs, keep = [], []
    for label, nodes, xs, kw in cases:
        try:
            src, ns = sc.jit_lane(nodes, stack_cap=kw.get("stack_cap"), stop_on_output=kw.get("stop_on_output", False),
                                  machine=machine)
        except sc.NotCompiled:
            continue  # tier 1 handles it; covered elsewhere
        srcs.append((src, ns))
        keep.append((label, nodes, xs, kw))
    assert keep, "no case compiled"
    lib = build_lanes(srcs, str(tmp_path / "lanes"))
    for i, (label, nodes, xs, kw) in enumerate(keep):
        got = run_lane(lib, i, xs, kw.get("budget") or (1 << 20))
        ref = po.OracleNet(nodes).compute_batch(xs, **kw)
        bad = np.nonzero((got[0] != ref[0]) | (got[1] != ref[1]) | (got[2] != ref[2]))[0]
        assert not bad.size, (label, int(bad[0]), [g[bad[0]] for g in got], [r[bad[0]] for r in ref])
    return [k[0] for k in keep]


@pytest.mark.parametrize("machine", [False, True])
def test_configs(tmp_path, machine):
    cases = []
    for name in sorted(mk.networks.CONFIGS):
        kind = 1 if name.startswith("c5") else 0
        cases.append((name, mk.networks.CONFIGS[name](), po.gen_inputs(SEED, 2000, kind=kind, mask=1023), {}))
    cases.append(("c4_d1024", mk.networks.pipeline_network(1024), po.gen_inputs(SEED, 40), {}))
    for d in (64, 256):  # every node's stack order reaches the output (networks.pipeline_program)
        cases.append((f"c4_observe_d{d}", mk.networks.pipeline_network(d, observe=True), po.gen_inputs(SEED, 200), {}))
    cases.append(("c5_all_trips", mk.networks.countdown_network(), np.arange(0, 1024, dtype=np.int64), {}))
    for b in (1, 11, 12, 13):
        cases.append((f"c2_budget{b}", mk.networks.example_network(), po.gen_inputs(SEED, 300), {"budget": b}))
        cases.append((f"c5_budget{b}", mk.networks.countdown_network(),
                      po.gen_inputs(SEED, 300, kind=1, mask=1023), {"budget": b * 37}))
    done = check_cases(tmp_path, cases, machine)
    # every config fits the native tier (the deep pipelines once their
    # constant-bound PUSH/POP loops are rolled back into loops)
    assert set(c[0] for c in cases) == set(done)


@pytest.mark.parametrize("machine", [False, True])
def test_wide_immediates_and_stop(tmp_path, machine):
    prog = ("IN ACC\nADD 2147483648\nADD 4294967295\nSUB 2147483649\nADD -4294967296\n"
            "ADD 9223372036854775807\nSUB -9223372036854775808\nMOV ACC, n:R1\nMOV R1, ACC\n"
            "JRO 2147483648\nNOP\nOUT ACC\nJLZ L\nOUT 1\nL: OUT 2")
    loop = [("a", "program", "JRO 0"), ("b", "program", "OUT 3\nJRO 0")]
    cases = [("wide", [("n", "program", prog)], po.gen_inputs(SEED, 2048), {}),
             ("budget", loop, [0] * 8, {"budget": 11}),
             ("stop", loop, [0] * 8, {"stop_on_output": True})]
    assert len(check_cases(tmp_path, cases, machine)) == 3


def test_paired_dispatch_marker(monkeypatch):
    # Two lanes per thread in the tile-sorted kernel (round 6, MK_PAIR in
    # kMachineSortKernel): networks without stack slots, one sweep pass for
    # two sorted chunks; the lanes' own code is the one-lane form, so every
    # machine-shape parity test here and on the GPU covers it.  Stack slots
    # (one column per thread) and MK_JIT_PAIR=0 keep one lane per thread.
    src, ns = sc.jit_lane(mk.networks.countdown_network(), machine=True)
    assert ns == 0 and "#define MK_PAIR 1" in src
    src, ns = sc.jit_lane(mk.networks.pipeline_network(64), machine=True)
    assert ns > 0 and "#define MK_PAIR 1" not in src
    monkeypatch.setenv("MK_JIT_PAIR", "0")
    src, _ = sc.jit_lane(mk.networks.countdown_network(), machine=True)
    assert "#define MK_PAIR 1" not in src


def test_loop_phases(tmp_path):
    # every path of the machine shape's self-loops (tisgen.loop_cases)
    cases = [(lbl, nodes, np.asarray(xs, np.int64), kw) for lbl, nodes, xs, kw in loop_cases()]
    assert len(check_cases(tmp_path, cases, machine=True)) == len(cases)


# The countdown's saturating decrements in asm blocks of MK_JIT_SAT_BLOCK
# (default 4) and the counter form of countdowns by other steps
# (MK_JIT_SAT_COUNT, default on; "count0" turns it off): every loop path, and
# C5 over all trip counts and at budgets inside its loops.
@pytest.mark.parametrize("mode", ["count0", "b8", "b32", "default"])
def test_countdown_forms(tmp_path, monkeypatch, mode):
    if mode == "count0":
        monkeypatch.setenv("MK_JIT_SAT_COUNT", "0")
    elif mode.startswith("b"):  # other asm block sizes
        monkeypatch.setenv("MK_JIT_SAT_BLOCK", mode[1:])
    cases = [(lbl, nodes, np.asarray(xs, np.int64), kw) for lbl, nodes, xs, kw in loop_cases()]
    cases.append(("c5_all_trips", mk.networks.countdown_network(), np.arange(-3, 1024, dtype=np.int64), {}))
    for b in (1, 2, 3, 37, 400, 1500):
        cases.append((f"c5_budget{b}", mk.networks.countdown_network(),
                      po.gen_inputs(SEED, 300, kind=1, mask=1023), {"budget": b}))
    assert len(check_cases(tmp_path, cases, machine=True)) == len(cases)


@pytest.mark.parametrize("machine", [False, True])
@pytest.mark.parametrize("block", range(4))
def test_random_networks(tmp_path, block, machine):
    cases = []
    for seed in range(block * 40, block * 40 + 40):
        kw = dict(budget=[37, 200, 1000][seed % 3], stack_cap=[1, 3, 8, 16, 17, 40, 1024][seed % 7],
                  stop_on_output=(seed % 5 == 4))
        cases.append((f"seed{seed}", random_network(seed), po.gen_inputs(seed * 7919 + 1, 256), kw))
    assert len(check_cases(tmp_path, cases, machine)) >= 30


@pytest.mark.parametrize("machine", [False, True])
@pytest.mark.parametrize("block", range(3))
def test_dynamic_stack_networks(tmp_path, block, machine):
    # stack depths that follow the data (tisgen.stack_loop_network): dynamic
    # stacks (STX/LDX, in-line OVF, the empty-check branch), capacities and
    # budgets that end lanes inside pushes and pops
    cases = []
    for seed in range(block * 30, block * 30 + 30):
        rows, gen = stack_loop_network(seed)
        kw = dict(budget=[None, 57, 300, 2000][seed % 4], stack_cap=[None, 3, 17, 64, 200][seed % 5])
        kw = {k: v for k, v in kw.items() if v is not None}
        cases.append((f"seed{seed}", rows, po.gen_inputs(seed + 5, 96, **gen), kw))
    for cls in ("data_dependent_stack_depth", "two_stacks_independent_depths"):
        nodes = census_classes()[cls][0][1]
        for cap in (None, 5, 200):
            xs = po.gen_inputs(3, 256, kind=1, mask=255)
            cases.append((f"{cls}_{cap}", nodes, xs, {"stack_cap": cap} if cap else {}))
    assert len(check_cases(tmp_path, cases, machine)) >= 24


def test_shapes():
    # acyclic schedules stream; data-dependent loops get the machine shape
    assert sc.jit_lane(mk.networks.example_network(), with_shape=True)[2] == "stream"
    assert sc.jit_lane(mk.networks.sample_network(), with_shape=True)[2] == "stream"
    src, _, shape = sc.jit_lane(mk.networks.countdown_network(), with_shape=True)
    assert shape == "machine" and "do {" in src


@pytest.mark.parametrize("which", ["countdown", "example", "sample"])
def test_module_compiles_for_gfx950(which):
    # hiprtc in-process, no GPU: the product library reports the native tier
    # for both shapes (machine: countdown; light stream: example, sample)
    net = mk.Network(getattr(mk.networks, f"{which}_network")())
    plan = net.plan(mode="jit")
    assert plan.startswith("tier=native "), plan
    src = net.jit_source()
    assert "mk_jit_exec" in src and "mk_lane" in src


# The machine shape of the deep pipelines (C4) used to hand hiprtc a 1.4 MB
# function whose checked variant had one early exit per round end (5,643 at
# D=64); it now looks the budget exit up after the body (tis_jit.cpp
# emit_budget_exit) and every C4 depth compiles well inside the bound, with
# the pipelined POP loops on.
COMPILE_BOUND_S = 60


@pytest.mark.parametrize("depth", [64, 256, 1024])
def test_machine_shape_pipeline_compiles_in_bound(depth, monkeypatch):
    monkeypatch.setenv("MK_JIT_SHAPE", "machine")
    net = mk.Network(mk.networks.pipeline_network(depth))
    plan = net.plan(mode="jit")
    assert plan.startswith("tier=native ") and "shape=machine" in plan, plan
    secs = float(plan.split("compile=")[1].split("s")[0])
    assert secs < COMPILE_BOUND_S, plan
    src = net.jit_source()
    assert len(src) < (1 << 20) and "mk_jit_exec" in src


def test_pipeline_stacks_share_slots(monkeypatch):
    # node k drains its stack before node k+1 pushes: the eight stacks share
    # one slot range (tis_sched.cpp share_slots); MK_SCHED_SHARE=0 gives each
    # its own.  D=64's shared range fits LDS: the heavy kernel keeps it there
    # (its default plan: round 6 also plans eight waves per SIMD, with 16
    # slots -- test_lds_occupancy_tunes_register_count).
    for depth, shared, own in ((64, 41, 328), (256, 233, 1864), (1024, 1001, 8008)):
        assert sc.jit_lane(mk.networks.pipeline_network(depth))[1] == shared
        monkeypatch.setenv("MK_SCHED_SHARE", "0")
        assert sc.jit_lane(mk.networks.pipeline_network(depth))[1] == own
        monkeypatch.delenv("MK_SCHED_SHARE")
    monkeypatch.setenv("MK_JIT_VGPR_FILE", "256")  # the eight-wave plan rejected: the default
    plan = mk.Network(mk.networks.pipeline_network(64)).plan(mode="jit")
    assert "slots=41 " in plan and "shape=stream-heavy-lds " in plan, plan
    monkeypatch.delenv("MK_JIT_VGPR_FILE")
    monkeypatch.setenv("MK_JIT_LDS_SLOTS", "0")
    plan = mk.Network(mk.networks.pipeline_network(64)).plan(mode="jit")
    assert "shape=stream-heavy " in plan, plan


def test_lds_occupancy_tunes_register_count(monkeypatch):
    # The loader's policy for heavy networks (mk_exec.hip tune_lds_auto):
    # D=64's 41 slots fit LDS at four waves per CU, yet eight per SIMD take
    # 49 registers (16 slots in a 5 KiB share, round 6); D=256
    # gets eight waves per SIMD (more_waves): 241 registers leave 16 slots,
    # all in a 5 KiB LDS share, and the compiled module holds eight waves
    # (its VGPRs are checked: stack_plans=w8:...); D=300 cannot reach eight
    # within 256 registers and gets two (80 slots in 20 KiB); D=400 reaches
    # neither and keeps 64 registers, four waves per CU, 160 of 337 slots in
    # LDS; D=1024 (961 slots at 64 registers) stays in HBM
    def fields(depth):
        plan = mk.Network(mk.networks.pipeline_network(depth)).plan(mode="jit")
        return dict(w.split("=", 1) for w in plan.split() if "=" in w)

    f = fields(64)  # round 6: eight waves per SIMD too (49 registers, 16 slots in a 5 KiB share)
    assert f["shape"] == "stream-heavy-lds" and f["regs"] == "49" and f["slots"] == "16", f
    assert f["stack_plans"].startswith("w8:") and "rejected" not in f["stack_plans"], f
    f = fields(256)
    assert f["shape"] == "stream-heavy-lds" and f["regs"] == "241" and f["slots"] == "16", f
    assert f["stack_plans"].startswith("w8:") and "rejected" not in f["stack_plans"], f
    assert f["waves_per_simd"] == "8" if "waves_per_simd" in f else True
    f = fields(300)
    assert f["shape"] == "stream-heavy-lds" and int(f["slots"]) <= 80 and f["stack_plans"].startswith("w2:"), f
    f = fields(400)
    assert f["shape"] == "stream-heavy-split" and f["regs"] == "64" and f["slots"] == "337", f
    f = fields(1024)
    assert f["shape"] == "stream-heavy" and f["regs"] == "64" and f["slots"] == "961", f
    # a fixed LDS budget (MK_JIT_LDS_SLOTS): registers for the most waves
    # with every slot in LDS -- D=256 reaches three (<= 208 slots of 256 B in
    # 2-KiB granules)
    monkeypatch.setenv("MK_JIT_LDS_SLOTS", "81920")
    f = fields(256)
    assert f["shape"] == "stream-heavy-lds" and int(f["slots"]) <= 208 and int(f["regs"]) > 24, f
    monkeypatch.setenv("MK_JIT_TUNE_REGS", "0")
    f = fields(256)
    assert f["slots"] == "233" and f["regs"] == "24", f


def test_stack_plan_rejection_falls_back(monkeypatch):
    # The plan-rejection path of jit_compile: a more_waves plan
    # whose module cannot hold its waves gives way to the next plan, and last
    # to the default.  MK_JIT_VGPR_FILE lowers the register file the check
    # prices against, so the path runs on purpose: at 256 VGPRs D=256's
    # eight-wave module (38 VGPRs x 8 = 304) is rejected and the two-wave
    # plan (80 slots in LDS) compiles and holds; at 128 both are rejected and
    # the default (64 registers, 160 of 193 slots in LDS) runs.
    def fields(depth, mode="jit"):
        plan = mk.Network(mk.networks.pipeline_network(depth)).plan(mode=mode)
        return dict(w.split("=", 1) for w in plan.split() if "=" in w)

    monkeypatch.setenv("MK_JIT_VGPR_FILE", "256")
    f = fields(256)
    assert f["stack_plans"].startswith("w8:") and f["stack_plans"].split(";")[0].endswith("-rejected"), f
    assert f["stack_plans"].split(";")[1].startswith("w2:") and "rejected" not in f["stack_plans"].split(";")[1], f
    assert int(f["slots"]) <= 80 and f["shape"] == "stream-heavy-lds", f
    monkeypatch.setenv("MK_JIT_VGPR_FILE", "128")
    f = fields(256)
    assert f["stack_plans"].count("-rejected") == 2, f
    assert f["regs"] == "64" and f["slots"] == "193" and f["shape"] == "stream-heavy-split", f
    f = fields(64)  # D=64's eight-wave plan rejected: the 24-register default (41 slots, 15 waves per CU)
    assert f["stack_plans"].endswith("-rejected") and f["regs"] == "24" and f["slots"] == "41", f
    # tier 2 keeps the default plan whichever plan the native tier runs: its
    # LDS register file would hold one block per CU at 241 registers
    monkeypatch.delenv("MK_JIT_VGPR_FILE")
    assert fields(256)["regs"] == "241"
    t2 = fields(256, mode="tile")
    assert t2["regs"] == "64" and t2["slots"] == "193" and t2["B"] == "64", t2


def test_compile_bounds_fall_back_with_reason(monkeypatch):
    # over the source bound: tier 2 runs it, mk_net_plan names the bound
    monkeypatch.setenv("MK_JIT_MAX_SRC", "1000")
    net = mk.Network(mk.networks.pipeline_network(64))
    plan = net.plan()
    assert plan.startswith("tier=compiled ") and "compile bound" in plan, plan
    assert mk.Network(mk.networks.pipeline_network(64)).plan(mode="jit").startswith("tier=none"), plan
    # over the time bound: the compile is abandoned, tier 2 runs it
    monkeypatch.delenv("MK_JIT_MAX_SRC")
    monkeypatch.setenv("MK_JIT_COMPILE_S", "0.001")
    # (one bound for all its stack plans' compiles together: the first one
    # abandoned, none is started for the next)
    plan = mk.Network(mk.networks.pipeline_network(256)).plan()
    assert plan.startswith("tier=compiled ") and "did not finish" in plan, plan
    assert "no time left for the next stack plan" in plan and "regs=64" in plan, plan


@pytest.mark.parametrize("cls", ["data_dependent_stack_depth", "two_stacks_independent_depths"])
@pytest.mark.parametrize("heavy", [False, True])
def test_dynamic_stack_module_compiles_for_gfx950(cls, heavy, monkeypatch):
    # the census classes whose stack depths follow the data run natively
    # (machine shape; forced stream + heavy: the buffer-op form of the
    # per-lane slot numbers, MK_SLOT_STX/LDX)
    if heavy:
        monkeypatch.setenv("MK_JIT_SHAPE", "stream")
        monkeypatch.setenv("MK_JIT_HEAVY_OPS", "1")
    net = mk.Network(mk.networks.census_classes()[cls][0][1])
    plan = net.plan(mode="jit")
    assert plan.startswith("tier=native "), plan
    src = net.jit_source()
    assert "MK_SLOT_STX" in src and "MK_SLOT_LDX" in src


def test_knobs_are_snapshotted_per_network(monkeypatch):
    # a network keeps the knobs of its load: plan, source and module agree
    monkeypatch.setenv("MK_JIT_SHAPE", "machine")
    net = mk.Network(mk.networks.example_network())
    monkeypatch.setenv("MK_JIT_SHAPE", "stream")
    assert "shape=machine" in net.plan(mode="jit")
    assert "#define MK_JIT_MACHINE 1" in net.jit_source()
    assert "knobs=shape=machine" in net.plan(mode="jit")


# The native tier's modules are code object v5 whichever hiprtc builds them
# (mk_exec.hip kCodeObjectVersion, mk_rtc.cpp): ROCm 7.2's default v6 modules
# corrupted the host heap inside PyTorch's bundled HIP runtime (r03c-r03k).
# The module of a dynamic-stack network (the shape that showed it), dumped by
# MK_JIT_DUMP, read with llvm-readelf: ELF ABI version 3 = code object v5.
def test_modules_are_code_object_v5(tmp_path, monkeypatch):
    readelf = "/opt/rocm/lib/llvm/bin/llvm-readelf"
    if not os.path.exists(readelf):
        pytest.skip("llvm-readelf not installed")
    rows, _ = stack_loop_network(6)  # two dynamic stacks, machine shape
    co = str(tmp_path / "m.co")
    monkeypatch.setenv("MK_JIT_DUMP", co)
    plan = mk.Network(rows).plan()
    assert plan.startswith("tier=native"), plan
    hdr = subprocess.run([readelf, "-h", co], capture_output=True, text=True, check=True).stdout
    assert any(l.split() == ["ABI", "Version:", "3"] for l in hdr.splitlines()), hdr


def _pop_chain_program(accum: str, depth: int, tail: str = "SWP\nOUT ACC") -> str:
    """One node: push x + 7k (k = 1..depth), then pop every value into an
    accumulator kept in BAK through `accum` (ACC holds the running value, R2
    the popped one), the loop counter in the node's own port R1."""
    return "\n".join([
        "IN ACC", "SAV", f"MOV {depth}, ACC",
        "L: SWP", "ADD 7", "PUSH ACC, s", "SWP", "SUB 1", "JGZ L",
        "MOV 0, ACC", "SAV", f"MOV {depth}, ACC", "MOV ACC, a:R1",
        "Q: POP s, ACC", "MOV ACC, a:R2", "SWP", accum, "SAV",
        "MOV R1, ACC", "SUB 1", "MOV ACC, a:R1", "JGZ Q",
        "MOV R1, NIL", tail, ""])


POP_CHAINS = {
    "mul3": "MOV ACC, a:R3\nADD ACC\nADD R3\nADD R2",      # C4's sum = 3 * sum + v
    "add": "ADD R2",                                       # sum + v
    "sub": "SUB R2",                                       # sum - v
    "mul2": "ADD ACC\nADD R2",                             # 2 * sum + v
    "mul4c": "ADD ACC\nADD ACC\nADD R2\nADD 5",            # 4 * sum + v + 5
    "neg": "NEG\nADD R2",                                  # v - sum
    "mul5": "MOV ACC, a:R3\nADD ACC\nADD ACC\nADD R3\nSUB R2",  # 5 * sum - v
}


@pytest.mark.parametrize("tail", ["out", "sign"])
def test_pop_chains(tmp_path, tail):
    """Pipelined pop runs (emit_prefetched_run) feeding linear accumulations,
    read through hops (narrow registers) or by a sign test (wide), bit-exact
    against the oracle on full-range inputs (INT32_MIN/MAX included)."""
    t = "SWP\nOUT ACC" if tail == "out" else "SWP\nJGZ P\nOUT 1\nJMP E\nP: OUT ACC\nE: NOP"
    cases = []
    for name, accum in POP_CHAINS.items():
        nodes = [NodeSpec("a", "program", _pop_chain_program(accum, 100, t)), NodeSpec("s", "stack", "")]
        cases.append((f"{name}-{tail}", nodes, po.gen_inputs(SEED, 300), {}))
    check_cases(tmp_path, cases)
