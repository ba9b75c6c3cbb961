"""GPU executor (HIP, via the C ABI) against the CPU oracle: bit-exact
out/status/steps on seeded inputs, plus size-independent properties at the
BASELINE.json sizes."""
import os
import re
import threading

import numpy as np
import pytest

import misaka_net_amd as mk
from misaka_net_amd import _native as N
from oracle import pyoracle as po
from tisgen import loop_cases, random_network, stack_loop_network

pytestmark = pytest.mark.gpu

SEED = 0x4D49534B41
THREADS = min(16, os.cpu_count() or 1)


def _m(mode):
    return None if mode == "auto" else mode


def oracle(nodes, xs, **kw):
    return po.OracleNet(nodes).compute_batch(xs, threads=THREADS, **kw)


def assert_same(got, ref, ctx=""):
    out, st, sp = ref
    bad = np.nonzero((got.out != out) | (got.status != st) | (got.steps != sp))[0]
    if bad.size:
        i = int(bad[0])
        raise AssertionError(
            f"{ctx}: {bad.size} lanes differ; lane {i}: gpu (out={got.out[i]}, st={got.status[i]:#x}, "
            f"steps={got.steps[i]}) oracle (out={out[i]}, st={st[i]:#x}, steps={sp[i]})"
        )


def test_readme_kat_on_gpu(gpu):
    net = mk.Network(mk.networks.example_network())
    r = net.compute_batch([5, 0, -7, 2147483646, 2147483647, -2147483648, 4294967301, -4294967296])
    assert r.out.tolist() == [7, 2, -5, -2147483648, -2147483647, -2147483646, 7, 2]
    assert (r.status == 0x11).all() and (r.steps == 12).all()


# "auto": the default path (the native per-network kernel when the schedule
# fits its limits, else tier 2); tier 2 with both lane schedulings; tier 1
MODES = ["auto", "tile", "refill", "interp"]
NATIVE = {"c2_example", "c3_sample", "c4_pipeline_d64", "c5_countdown"}  # default path: the native tier


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize(
    "name,nodes,n,gen",
    [
        ("c2_example", mk.networks.example_network(), 1 << 17, (N.MK_GEN_FULL, 0)),
        ("c3_sample", mk.networks.sample_network(), 1 << 17, (N.MK_GEN_FULL, 0)),
        ("c4_pipeline_d64", mk.networks.pipeline_network(64), 1 << 12, (N.MK_GEN_FULL, 0)),
        ("c5_countdown", mk.networks.countdown_network(), 1 << 15, (N.MK_GEN_MASKED, 1023)),
    ],
)
def test_configs_bit_exact(gpu, name, nodes, n, gen, mode):
    xs = po.gen_inputs(SEED, n, kind=gen[0], mask=gen[1])
    net = mk.Network(nodes)
    mode = None if mode == "auto" else mode
    plan = net.plan(mode=mode)
    if mode is None:
        assert plan.startswith("tier=native" if name in NATIVE else "tier=compiled"), plan
    elif mode != "interp":
        assert plan.startswith("tier=compiled"), plan
    got = net.compute_batch(xs, mode=mode)
    assert_same(got, oracle(nodes, xs), name)


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("depth", [256, 1024])
def test_c4_deep_stacks_spill_to_hbm(gpu, mode, depth):
    nodes = mk.networks.pipeline_network(depth)
    xs = po.gen_inputs(SEED, 600)
    got = mk.Network(nodes).compute_batch(xs, mode=_m(mode))
    ref = oracle(nodes, xs)
    assert_same(got, ref, f"c4 D={depth}")
    assert (got.status == 0x11).all()


# Every path of the machine shape's self-loops (tisgen.loop_cases: 32-bit
# and 64-bit phases, range checks at +-2^30, step counters, budget-ended
# loops), once on the default path and once with the machine shape and a
# policy that leaves loops early (so groups re-enter loops with smaller
# and mixed step counts).
@pytest.mark.parametrize("variant", ["auto", "machine-early-exit", "pool64", "k2"])
def test_loop_phases_bit_exact(gpu, monkeypatch, variant):
    if variant == "machine-early-exit":  # the pool-less kernel, leaving loops early
        monkeypatch.setenv("MK_JIT_SHAPE", "machine")
        monkeypatch.setenv("MK_JIT_POLICY", "8,12,16")
    if variant == "pool64":  # the smallest LDS lane pool: groups refill from few parked lanes
        monkeypatch.setenv("MK_JIT_SHAPE", "machine")
        monkeypatch.setenv("MK_JIT_POOL", "64")
    if variant == "k2":  # two lanes per thread
        monkeypatch.setenv("MK_JIT_SHAPE", "machine")
        monkeypatch.setenv("MK_JIT_POOL", "2")
    for label, nodes, xs, kw in loop_cases(n=4096):
        xs = np.asarray(xs, np.int64)
        assert_same(mk.Network(nodes).compute_batch(xs, **kw), oracle(nodes, xs, **kw), f"{label} {variant}")


# Both stack-slot layouts of the heavy kernel (wave-blocked / lane-major),
# whichever the slot count would pick.
@pytest.mark.parametrize("layout", ["blocked", "lane"])
@pytest.mark.parametrize("depth", [64, 1024])
def test_heavy_kernel_slot_layouts(gpu, monkeypatch, layout, depth):
    monkeypatch.setenv("MK_JIT_SLOT_LAYOUT", layout)
    nodes = mk.networks.pipeline_network(depth)
    net = mk.Network(nodes)
    assert "shape=stream-heavy" in net.plan(), net.plan()
    xs = po.gen_inputs(SEED + depth, 1000)
    assert_same(net.compute_batch(xs), oracle(nodes, xs), f"c4 D={depth} {layout}")


# Stack slots in LDS (the heavy kernel's wave owns nslots x 64 words) against
# HBM, and split between them: by default (tune_lds_auto) D=64 in LDS; D=256
# (241 registers, 16 slots: eight waves per SIMD) and D=300 (two waves) in
# LDS with most stack entries in registers (more_waves); D=400 / 480 split
# (the first 160 / 320 slots in LDS), D=1024 in HBM; MK_JIT_LDS_SLOTS=0 keeps
# every slot in HBM, 81920 every slot of D=256 in LDS (three waves per CU).
# The pipelined POP loops read LDS.
@pytest.mark.parametrize("lds,depth,shape", [("auto", 64, "lds"), ("0", 64, "heavy"), ("auto", 256, "lds"),
                                             ("auto", 300, "lds"), ("0", 256, "heavy"), ("81920", 256, "lds"),
                                             ("auto", 400, "split"), ("auto", 480, "split")])
def test_heavy_kernel_slots_in_lds(gpu, monkeypatch, lds, depth, shape):
    if lds != "auto":
        monkeypatch.setenv("MK_JIT_LDS_SLOTS", lds)
    nodes = mk.networks.pipeline_network(depth)
    net = mk.Network(nodes)
    want = {"heavy": "shape=stream-heavy ", "split": "shape=stream-heavy-split ", "lds": "shape=stream-heavy-lds "}
    assert want[shape] in net.plan(), net.plan()
    xs = po.gen_inputs(SEED + 5 * depth, 4100)
    assert_same(net.compute_batch(xs), oracle(nodes, xs), f"c4 D={depth} lds={lds}")


def signed_pop_network(depth):
    """Pushes x - 7i (int32), pops them into an int64 sum and branches on its
    sign: a popped value that were zero-extended instead of sign-extended
    (stack.go:113 -> program.go:163 round trip) would flip the branch."""
    prog = "\n".join(
        ["IN ACC", "SAV", f"MOV {depth}, ACC", "PL: SWP", "SUB 7", "PUSH ACC, s0", "SWP", "SUB 1", "JGZ PL",
         "MOV 0, ACC", "SAV", f"MOV {depth}, ACC", "MOV ACC, p0:R1", "QL: POP s0, ACC", "MOV ACC, p0:R2", "SWP",
         "ADD R2", "SAV", "MOV R1, ACC", "SUB 1", "MOV ACC, p0:R1", "JGZ QL", "SWP", "JLZ NEG", "OUT 1", "JMP E",
         "NEG: OUT -1", "E: NOP", ""]
    )
    return [mk.networks.NodeSpec("p0", "program", prog), mk.networks.NodeSpec("s0", "stack")]


# Popped values are sign-extended in every slot layout of the heavy kernel
# (the wave-blocked one reads slots with unsigned 32-bit buffer loads; "lds"
# keeps them in LDS, "blocked" / "lane" in HBM).
@pytest.mark.parametrize("layout", ["blocked", "lane", "lds"])
@pytest.mark.parametrize("depth", [64, 300])
def test_heavy_kernel_pops_sign_extend(gpu, monkeypatch, layout, depth):
    monkeypatch.setenv("MK_JIT_SLOT_LAYOUT", "lane" if layout == "lane" else "blocked")
    monkeypatch.setenv("MK_JIT_LDS_SLOTS", "163840" if layout == "lds" else "0")
    monkeypatch.setenv("MK_JIT_HEAVY_OPS", "16")
    nodes = signed_pop_network(depth)
    net = mk.Network(nodes)
    want = "shape=stream-heavy-lds " if layout == "lds" else "shape=stream-heavy "
    assert want in net.plan(), net.plan()
    xs = po.gen_inputs(SEED + 7 * depth, 1000)
    ref = oracle(nodes, xs)
    assert {1, -1} <= set(ref[0].tolist())
    assert_same(net.compute_batch(xs), ref, f"signed pops D={depth} {layout}")


# Pipelined POP loops (emit_prefetched_run: reps >= 64) in every kernel: the
# light stream one (4 lanes per thread, lane-major slots), the heavy one
# (wave-blocked buffer slots) and the machine shape (lane registers in a
# struct).  The 8-node pipeline on the machine shape used to be a 1.4 MB
# module that took hiprtc minutes (one early exit per round end in its
# checked variant); with the budget-exit lookup it compiles in seconds.
@pytest.mark.parametrize("shape", ["light", "heavy", "machine"])
def test_pipelined_pops_every_shape(gpu, monkeypatch, shape):
    if shape == "heavy":
        monkeypatch.setenv("MK_JIT_HEAVY_OPS", "16")
    if shape == "machine":
        monkeypatch.setenv("MK_JIT_SHAPE", "machine")
    cases = [signed_pop_network(300), mk.networks.pipeline_network(256)]
    for nodes in cases:
        net = mk.Network(nodes)
        plan = net.plan()
        want = {"light": "shape=stream ", "heavy": "shape=stream-heavy", "machine": "shape=machine"}[shape]
        if shape == "light" and "shape=stream-heavy" in plan:
            continue  # the 8-node pipeline is heavy by size
        assert want in plan + " ", plan
        xs = po.gen_inputs(SEED + 3, 777)
        assert_same(net.compute_batch(xs), oracle(nodes, xs), f"pipelined pops {shape}")


# Heavy stream kernels run one thread per input, several launches per batch
# when the stack slots of the whole batch exceed the slot-memory cap
# (MK_JIT_SLOT_BYTES=1: 64 inputs per launch); counters included.
def test_heavy_kernel_chunked_launches(gpu, monkeypatch):
    import torch

    monkeypatch.setenv("MK_JIT_SLOT_BYTES", "1")
    nodes = mk.networks.pipeline_network(1024)
    net = mk.Network(nodes)
    assert "shape=stream-heavy" in net.plan(), net.plan()
    n = 1000
    xs = po.gen_inputs(SEED, n)
    assert_same(net.compute_batch(xs), oracle(nodes, xs), "c4 D=1024 in 16 launches")
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    st = torch.empty(n, dtype=torch.uint8, device="cuda")
    stats = torch.zeros(N.MK_STATS_LEN, dtype=torch.int64, device="cuda")
    net.compute_device(n, out_ptr=out.data_ptr(), status_ptr=st.data_ptr(), stats_ptr=stats.data_ptr(),
                       gen_kind=N.MK_GEN_FULL, seed=SEED, stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    ref = oracle(nodes, po.gen_inputs(SEED, n))
    assert out.cpu().numpy().tolist() == ref[0].tolist()
    assert stats[0].item() == int(ref[2].sum()) and stats[2].item() == n


@pytest.mark.parametrize("mode", MODES)
def test_c5_zero_trip_and_maximum_trip(gpu, mode):
    nodes = mk.networks.countdown_network()
    xs = np.arange(0, 1024, dtype=np.int64)
    assert_same(mk.Network(nodes).compute_batch(xs, mode=_m(mode)), oracle(nodes, xs), "c5 all trip counts")


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("seed", range(0, 240, 1))
def test_random_networks_bit_exact(gpu, seed, mode):
    rows = random_network(seed)
    xs = po.gen_inputs(seed * 7919 + 1, 256)
    cap = [1, 3, 8, 16, 17, 40, 1024][seed % 7]
    kw = dict(budget=[37, 200, 1000][seed % 3], stack_cap=cap, stop_on_output=(seed % 5 == 4))
    net = mk.Network(rows)
    got = net.compute_batch(xs, mode=_m(mode), **kw)
    if mode == "auto":  # the default path is the native tier unless a limit sends it down a tier, with a reason
        plan = net.plan(stack_cap=kw["stack_cap"], stop_on_output=kw["stop_on_output"])
        assert plan.startswith(("tier=native", "tier=interp")) or " native=" in plan, plan
    assert_same(got, oracle(rows, xs, **kw), f"seed {seed}")


# Stack depths that follow the data (the schedule compiler's dynamic stacks:
# STX/LDX at base + depth register, in-line OVF, the empty-check branch):
# tisgen.stack_loop_network on every tier, capacities and budgets that end
# lanes inside pushes and pops (stack.go:95-155, program.go:475-566).
@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("seed", range(0, 60))
def test_dynamic_stack_networks_bit_exact(gpu, seed, mode):
    rows, gen = stack_loop_network(seed)
    xs = po.gen_inputs(seed + 5, 2048, **gen)
    kw = dict(budget=[None, 57, 300, 2000][seed % 4], stack_cap=[None, 3, 17, 64, 200][seed % 5])
    kw = {k: v for k, v in kw.items() if v is not None}
    got = mk.Network(rows).compute_batch(xs, mode=_m(mode), **kw)
    assert_same(got, oracle(rows, xs, **kw), f"seed {seed}")


# The census classes whose depths follow the data, at their bench size
# (1,048,576 lanes, inputs 0..255) on the default path, now the native tier:
# every lane exact against an oracle table over all 256 inputs.
@pytest.mark.parametrize("cls", ["data_dependent_stack_depth", "two_stacks_independent_depths"])
@pytest.mark.parametrize("mode", ["auto", "tile"])
def test_dynamic_stack_census_full_size(gpu, cls, mode):
    n = 1 << 20
    nodes = mk.networks.census_classes()[cls][0][1]
    net = mk.Network(nodes)
    if mode == "auto":
        assert net.plan().startswith("tier=native"), net.plan()
    out, st, sp, stats = _device_run(net, n, gen=(N.MK_GEN_MASKED, 255), mode=_m(mode))
    x = po.gen_inputs(SEED, n, kind=N.MK_GEN_MASKED, mask=255)
    t_out, t_st, t_sp = oracle(nodes, np.arange(256, dtype=np.int64))
    assert np.array_equal(out, t_out[x]) and np.array_equal(st, t_st[x]) and np.array_equal(sp, t_sp[x])
    assert stats[0] == int(sp.astype(np.int64).sum()) and stats[2] == n


# The tile-sorted kernel's measured grid (mk_exec.hip GridTune, round 6):
# the first three launches at a batch size run 3/4, 1/2 and all of the
# resident grid, a later one keeps the fastest.  Every launch of the tuning
# sequence, and the ones after it, is exact; the plan reports the choice.
@pytest.mark.parametrize("cls", ["data_dependent_stack_depth", "two_stacks_independent_depths"])
def test_grid_tuning_launches_exact(gpu, cls):
    n = (1 << 18) + 333  # a tuned size, with a partial last tile
    nodes = mk.networks.census_classes()[cls][0][1]
    net = mk.Network(nodes)
    assert net.plan().startswith("tier=native") and "grid_tuned=" not in net.plan()
    x = po.gen_inputs(SEED, n, kind=N.MK_GEN_MASKED, mask=255)
    t_out, t_st, t_sp = oracle(nodes, np.arange(256, dtype=np.int64))
    for k in range(6):
        out, st, sp, stats = _device_run(net, n, gen=(N.MK_GEN_MASKED, 255))
        assert np.array_equal(out, t_out[x]) and np.array_equal(st, t_st[x]) and np.array_equal(sp, t_sp[x]), k
        assert stats[0] == int(sp.astype(np.int64).sum()) and stats[2] == n
    m = re.search(r"grid_tuned=(\d+)/(\d+)", net.plan())
    assert m and 0 < int(m.group(1)) <= int(m.group(2)), net.plan()


# The tile-sorted kernel's end-reason counters (stats[2..6]): the other
# three reasons are counted only when some lane of a chunk did not end
# quiescent (round 6), so every reason is driven here -- budgets inside the
# loops, stop-on-output, and stack overflows on a dynamic-stack class.
@pytest.mark.parametrize("case", ["plain", "budget", "stop", "overflow"])
def test_machine_reason_counters(gpu, case):
    import torch

    n = 300000
    if case == "overflow":
        nodes = mk.networks.census_classes()["data_dependent_stack_depth"][0][1]
        kw, mask = {"stack_cap": 100}, 255
    else:
        nodes = mk.networks.countdown_network()
        kw = {"budget": 700} if case == "budget" else {"stop_on_output": True} if case == "stop" else {}
        mask = 1023
    net = mk.Network(nodes)
    assert "shape=machine" in net.plan(**({"stack_cap": kw["stack_cap"]} if "stack_cap" in kw else {}))
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    st = torch.empty(n, dtype=torch.uint8, device="cuda")
    sp = torch.empty(n, dtype=torch.int32, device="cuda")
    stats = torch.zeros(N.MK_STATS_LEN, dtype=torch.int64, device="cuda")
    net.compute_device(n, out_ptr=out.data_ptr(), status_ptr=st.data_ptr(), steps_ptr=sp.data_ptr(),
                       stats_ptr=stats.data_ptr(), seed=SEED, gen_kind=N.MK_GEN_MASKED, gen_mask=mask,
                       stream=torch.cuda.current_stream().cuda_stream, **kw)
    torch.cuda.synchronize()
    s_ = st.cpu().numpy()
    r = s_ & N.MK_ST_REASON_MASK
    got = stats.cpu().numpy()
    want = [int((s_ & N.MK_ST_HAS_OUTPUT).astype(bool).sum()), n] + [int((r == k).sum()) for k in (1, 2, 3, 4)]
    assert list(got[1:7]) == want, (case, list(got), want)
    assert got[0] == int(sp.cpu().numpy().view(np.uint32).astype(np.int64).sum())
    if case != "plain":
        assert want[2 + {"budget": 1, "overflow": 2, "stop": 3}[case]] > 0, (case, want)


@pytest.mark.parametrize("mode", MODES)
def test_budget_and_stop_on_output(gpu, mode):
    nodes = [("a", "program", "JRO 0"), ("b", "program", "OUT 3\nJRO 0")]
    got = mk.Network(nodes).compute_batch([0] * 70, budget=11, mode=_m(mode))
    assert (got.steps == 12).all() and (got.status == (N.MK_ST_BUDGET | N.MK_ST_HAS_OUTPUT)).all()
    got = mk.Network(nodes).compute_batch([0] * 70, stop_on_output=True, mode=_m(mode))
    assert (got.steps == 2).all() and (got.status == (N.MK_ST_OUTPUT_STOP | N.MK_ST_HAS_OUTPUT)).all()


@pytest.mark.parametrize("mode", ["auto", "tile", "refill"])
@pytest.mark.parametrize("budget", [1, 11, 12, 13, 5000])
def test_compiled_budget_boundaries(gpu, budget, mode):
    for nodes, kind in ((mk.networks.example_network(), 0), (mk.networks.countdown_network(), 1)):
        xs = po.gen_inputs(SEED, 3000, kind=kind, mask=1023)
        got = mk.Network(nodes).compute_batch(xs, budget=budget, mode=_m(mode))
        assert_same(got, oracle(nodes, xs, budget=budget), str(budget))


def test_empty_batch(gpu):
    got = mk.Network(mk.networks.example_network()).compute_batch([])
    assert got.out.size == 0


@pytest.mark.parametrize("mode", MODES)
def test_ragged_sizes(gpu, mode):
    nodes = mk.networks.sample_network()
    net = mk.Network(nodes)
    for n in [1, 2, 3, 5, 63, 64, 65, 255, 257, 1000, 1023, 1025, 4097]:
        xs = po.gen_inputs(n, n)
        assert_same(net.compute_batch(xs, mode=_m(mode)), oracle(nodes, xs), f"n={n}")


def test_concurrent_host_calls(gpu):
    nodes = mk.networks.example_network()
    net = mk.Network(nodes)
    xs = [po.gen_inputs(s, 50000) for s in range(4)]
    res = [None] * 4

    def work(i):
        res[i] = net.compute_batch(xs[i])

    ts = [threading.Thread(target=work, args=(i,)) for i in range(4)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    for i in range(4):
        assert_same(res[i], oracle(nodes, xs[i]), f"thread {i}")


def test_device_generator_matches_oracle(gpu):
    import torch

    n = 1 << 20
    d = torch.empty(n, dtype=torch.int32, device="cuda")
    mk.generate_inputs_device(n, d.data_ptr(), seed=SEED, offset=12345,
                              stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert np.array_equal(d.cpu().numpy(), po.gen_inputs(SEED, n, offset=12345).astype(np.int32))


def _device_run(net, n, *, in_tensor=None, in_kind=N.MK_IN_I32, gen=(N.MK_GEN_FULL, 0), offset=0, mode=None):
    import torch

    out = torch.empty(n, dtype=torch.int32, device="cuda")
    st = torch.empty(n, dtype=torch.uint8, device="cuda")
    sp = torch.empty(n, dtype=torch.int32, device="cuda")
    stats = torch.zeros(N.MK_STATS_LEN, dtype=torch.int64, device="cuda")
    net.compute_device(n, out_ptr=out.data_ptr(), status_ptr=st.data_ptr(), steps_ptr=sp.data_ptr(),
                       stats_ptr=stats.data_ptr(), in_ptr=None if in_tensor is None else in_tensor.data_ptr(),
                       in_kind=in_kind, seed=SEED, gen_kind=gen[0], gen_mask=gen[1], offset=offset,
                       stream=torch.cuda.current_stream().cuda_stream, mode=_m(mode))
    torch.cuda.synchronize()
    return out.cpu().numpy(), st.cpu().numpy(), sp.cpu().numpy().view(np.uint32), stats.cpu().numpy()


@pytest.mark.parametrize("mode", MODES)
def test_device_api_input_kinds_agree(gpu, mode):
    import torch

    nodes = mk.networks.sample_network()
    net = mk.Network(nodes)
    n = 100003
    x64 = po.gen_inputs(SEED, n, offset=777)
    a = _device_run(net, n, offset=777, mode=_m(mode))
    b = _device_run(net, n, in_tensor=torch.from_numpy(x64.astype(np.int32)).cuda(), in_kind=N.MK_IN_I32, mode=_m(mode))
    c = _device_run(net, n, in_tensor=torch.from_numpy(x64).cuda(), in_kind=N.MK_IN_I64, mode=_m(mode))
    # misaligned int32 input / output views take the scalar tile path
    xt = torch.from_numpy(x64.astype(np.int32)).cuda()
    xo = torch.empty(n + 1, dtype=torch.int32, device="cuda")
    xo[1:] = xt
    d = _device_run(net, n, in_tensor=xo[1:], in_kind=N.MK_IN_I32, mode=_m(mode))
    ref = oracle(nodes, x64)
    for r in (a, b, c, d):
        for u, v in zip(r[:3], ref):
            assert np.array_equal(u, v)
        assert r[3][0] == int(ref[2].sum()) and r[3][2] == n
        assert r[3][1] == int(((ref[1] & 0x10) != 0).sum())


@pytest.mark.parametrize("mode", MODES)
def test_c2_full_size_properties(gpu, mode):
    # BASELINE config 2: 16,777,216 lanes; size-independent checks:
    # out == int32(x + 2) (README.md:39-44), 12 retired instrs, quiescent + output.
    import torch

    n = 1 << 24
    net = mk.Network(mk.networks.example_network())
    x = torch.empty(n, dtype=torch.int32, device="cuda")
    mk.generate_inputs_device(n, x.data_ptr(), seed=SEED, stream=torch.cuda.current_stream().cuda_stream)
    out, st, sp, stats = _device_run(net, n, in_tensor=x, mode=_m(mode))
    xe = x.cpu().numpy().astype(np.int64)
    assert np.array_equal(out, ((xe + 2 + 2**31) % 2**32 - 2**31).astype(np.int32))
    assert (st == 0x11).all() and (sp == 12).all()
    assert stats[0] == 12 * n and stats[1] == n and stats[2] == n and stats[3] == n
    # a seeded slice bit-exact against the oracle, edge lanes included
    sl = slice(n - 4096, n)
    ref = oracle(mk.networks.example_network(), xe[sl])
    assert np.array_equal(out[sl], ref[0]) and np.array_equal(st[sl], ref[1]) and np.array_equal(sp[sl], ref[2])


@pytest.mark.parametrize("mode", MODES)
def test_c3_64m_shard_properties(gpu, mode):
    # BASELINE config 3 shards 67,108,864 lanes over 8 GPUs; one shard here
    # (lanes [7*8M, 8*8M)) with the global lane offset of rank 7.
    n = 1 << 23
    off = 7 * n
    nodes = mk.networks.sample_network()
    net = mk.Network(nodes)
    out, st, sp, stats = _device_run(net, n, offset=off, mode=_m(mode))
    x = po.gen_inputs(SEED, n, offset=off)
    x32 = x.astype(np.int32).astype(np.int64)
    want = ((2 * x32 + 2**31) % 2**32 - 2**31).astype(np.int32)
    nz = x32 != 0
    assert np.array_equal(out[nz], want[nz]) and (out[~nz] == 0).all()
    assert (st[nz] == 0x11).all() and (st[~nz] == N.MK_ST_QUIESCENT).all()
    # steps depend only on the sign class; pin each class with the oracle
    for cls in (x32 > 0, x32 < 0, x32 == 0):
        if cls.any():
            i = int(np.nonzero(cls)[0][0])
            assert (sp[cls] == oracle(nodes, x[i:i + 1])[2][0]).all()


@pytest.mark.parametrize("mode", ["auto", "interp"])
def test_c3_full_64m_equals_eight_shards(gpu, mode):
    # BASELINE config 3 end to end: one launch over all 67,108,864 global
    # lanes equals the concatenation of the 8 rank shards (8,388,608 lanes at
    # offsets r * 8,388,608, inputs generated from the global lane index) --
    # the order bench.py's RCCL gather to rank 0 must reproduce
    # (misaka_net_amd.dist.shard / timed_gather).  out, status and steps
    # bit-exact; the retired-instruction counters add up.
    shard, world = 1 << 23, 8
    net = mk.Network(mk.networks.sample_network())
    full = _device_run(net, world * shard, offset=0, mode=_m(mode))
    tot = np.zeros(N.MK_STATS_LEN, np.int64)
    for r in range(world):
        lo, hi = mk.dist.shard(r, shard)
        part = _device_run(net, shard, offset=lo, mode=_m(mode))
        for a, b, what in zip(full[:3], part[:3], ("out", "status", "steps")):
            bad = np.nonzero(a[lo:hi] != b)[0]
            assert not bad.size, f"rank {r} shard: {what} differs at global lane {lo + int(bad[0])}"
        tot += part[3]
    assert tot[0] == full[3][0] and tot[1] == full[3][1] and tot[2] == full[3][2] == world * shard


@pytest.mark.parametrize("mode", MODES)
def test_c5_full_size_properties(gpu, mode):
    # the C5 bench workload: 4,194,304 lanes, masked inputs 0..1023.  The
    # network is a function of x alone, so every lane is checked exactly
    # against an oracle table over all 1024 inputs; out also in closed form:
    # x <= 0 -> -1, else r = (x - 1) % 3 + 1 selects 112 / 13 / 4 by JRO.
    n = 1 << 22
    nodes = mk.networks.countdown_network()
    out, st, sp, stats = _device_run(mk.Network(nodes), n, gen=(N.MK_GEN_MASKED, 1023), mode=_m(mode))
    x = po.gen_inputs(SEED, n, kind=N.MK_GEN_MASKED, mask=1023)
    t_out, t_st, t_sp = oracle(nodes, np.arange(1024, dtype=np.int64))
    assert np.array_equal(out, t_out[x]) and np.array_equal(st, t_st[x]) and np.array_equal(sp, t_sp[x])
    r = (x - 1) % 3 + 1
    assert np.array_equal(out, np.where(x <= 0, -1, np.choose(r - 1, [112, 13, 4])))
    assert stats[0] == int(sp.astype(np.int64).sum()) and stats[2] == n


def _affine(nodes):
    """(A, B) with out(x) = int32(A*x + B) for the pipeline networks: every
    hop truncates to int32 and the control flow does not depend on x, so
    the int32 output is affine in x mod 2^32 (stack.go:95-155,
    intStack.go:20-38, program.go:284-311); A and B from two oracle lanes."""
    f = oracle(nodes, np.array([0, 1], np.int64))[0].astype(np.int64)
    return (int(f[1]) - int(f[0])) % 2**32, int(f[0]) % 2**32


def _assert_affine_every_lane(out, x, A, B):
    want = ((A * (x.astype(np.int64) % 2**32) + B) % 2**32).astype(np.uint32).view(np.int32)
    bad = np.nonzero(out != want)[0]
    assert not bad.size, f"{bad.size} lanes off the affine map; lane {bad[0]}: x={x[bad[0]]} out={out[bad[0]]}"


# The C4 bench workloads at their bench sizes: d64 (1,048,576 lanes), d256
# (524,288; the default heavy kernel: 193 shared slots, the first 160 in LDS
# and the rest in the wave's HBM block) and d1024 (262,144; 961 shared slots
# in HBM, wave-blocked buffer slots, launches of at most 69,824 inputs whose
# slot blocks fit the Infinity Cache -- tis_jit.h kJitSlotBytes).  Every
# lane is checked exactly: status and steps equal the oracle's (the control
# flow does not depend on x) and out equals the oracle's affine map.  The
# bench network's map has A = 0 (networks.pipeline_program: its x
# coefficient vanishes after 8 nodes), so its every-lane check sees the last
# nodes' stacks; the observe variant below carries every node's.
@pytest.mark.parametrize("depth,n", [(64, 1 << 20), (256, 1 << 19), (1024, 1 << 18)])
def test_c4_full_size_every_lane(gpu, depth, n):
    nodes = mk.networks.pipeline_network(depth)
    net = mk.Network(nodes)
    if depth > 64:
        assert "shape=stream-heavy" in net.plan(), net.plan()
    out, st, sp, stats = _device_run(net, n)
    x = po.gen_inputs(SEED, n)
    A, B = _affine(nodes)
    assert A == 0
    _assert_affine_every_lane(out, x, A, B)
    ref = oracle(nodes, x[-512:])
    assert np.array_equal(out[-512:], ref[0]) and np.array_equal(sp[-512:], ref[2])
    assert (st == 0x11).all() and (sp == ref[2][0]).all() and stats[0] == int(ref[2][0]) * n


# The same workloads with pipeline_network(observe=True): each node adds its
# input back at the end, so the x coefficient is odd and a wrong pop order,
# a lost push or a slot mix-up in any node changes every lane's output.
@pytest.mark.parametrize("depth,n", [(64, 1 << 20), (256, 1 << 19), (1024, 1 << 18)])
def test_c4_observe_full_size_every_lane(gpu, depth, n):
    nodes = mk.networks.pipeline_network(depth, observe=True)
    bench = mk.Network(mk.networks.pipeline_network(depth)).plan().split("shape=")[1].split()[0]
    net = mk.Network(nodes)
    assert net.plan().split("shape=")[1].split()[0] == bench, net.plan()  # the bench network's kernel shape
    out, st, sp, stats = _device_run(net, n)
    x = po.gen_inputs(SEED, n)
    A, B = _affine(nodes)
    assert A % 2 == 1
    _assert_affine_every_lane(out, x, A, B)
    ref = oracle(nodes, x[:512])
    assert np.array_equal(out[:512], ref[0]) and np.array_equal(sp[:512], ref[2])
    assert (st == 0x11).all() and (sp == ref[2][0]).all() and stats[0] == int(ref[2][0]) * n


# The stack plans the loader falls back to: with the register
# file the check prices against lowered (MK_JIT_VGPR_FILE), D=256 runs its
# two-wave plan (256) or the default one-wave plan (128) -- every lane at the
# bench size, as test_c4_observe_full_size_every_lane -- and tier 2 runs the
# default plan's schedule while the native tier runs a more_waves plan.
@pytest.mark.parametrize("vfile,plans", [(256, "w2:"), (128, "-rejected;w2:")])
def test_c4_stack_plan_fallbacks_every_lane(gpu, monkeypatch, vfile, plans):
    monkeypatch.setenv("MK_JIT_VGPR_FILE", str(vfile))
    nodes = mk.networks.pipeline_network(256, observe=True)
    net = mk.Network(nodes)
    plan = net.plan()
    assert plans in plan and ("regs=64" in plan) == (vfile == 128), plan
    n = 1 << 19
    out, st, sp, stats = _device_run(net, n)
    x = po.gen_inputs(SEED, n)
    A, B = _affine(nodes)
    _assert_affine_every_lane(out, x, A, B)
    ref = oracle(nodes, x[:512])
    assert np.array_equal(out[:512], ref[0]) and np.array_equal(sp[:512], ref[2])
    assert (st == 0x11).all() and stats[0] == int(ref[2][0]) * n


def test_tier2_keeps_the_default_stack_plan(gpu):
    nodes = mk.networks.pipeline_network(256, observe=True)
    net = mk.Network(nodes)
    regs = lambda plan: int(plan.split("regs=")[1].split()[0])  # noqa: E731
    assert regs(net.plan()) > 200 and regs(net.plan(mode="tile")) == 64, (net.plan(), net.plan(mode="tile"))
    xs = po.gen_inputs(SEED, 20000)
    ref = oracle(nodes, xs)
    for mode in ("tile", "refill", None):
        assert_same(net.compute_batch(xs, mode=mode), ref, f"C4 d256 {mode}")


@pytest.mark.parametrize("mode", MODES)
def test_wide_immediates_on_symbolic_acc(gpu, mode):
    # immediates whose low 32-bit word has bit 31 set, applied to a data-dependent ACC
    prog = ("IN ACC\nADD 2147483648\nADD 4294967295\nSUB 2147483649\nADD -4294967296\n"
            "ADD 9223372036854775807\nSUB -9223372036854775808\nMOV ACC, n:R1\nMOV R1, ACC\n"
            "JRO 2147483648\nNOP\nOUT ACC\nJLZ L\nOUT 1\nL: OUT 2")
    nodes = [("n", "program", prog)]
    xs = po.gen_inputs(SEED, 4096)
    assert_same(mk.Network(nodes).compute_batch(xs, mode=_m(mode)), oracle(nodes, xs), "wide imm")


# The native tier's two kernel shapes (tis_jit.h): acyclic schedules stream,
# cyclic ones run as per-lane state machines.  Force the machine shape on
# every network (the knobs are read when a network is loaded) and run each of
# its kernels: the pool-less one under several wave policies (MK_JIT_POLICY,
# compiled into each new network's kernel) and the two lane-compaction
# kernels (MK_JIT_POOL: K lanes per thread, or an LDS pool per wave).
@pytest.mark.parametrize("policy", ["k2", "k4", "pool64", "pool256", "8,12,16", "1,0,64", "64,16,1", "16,8,4"])
def test_machine_shape_and_policies(gpu, monkeypatch, policy):
    monkeypatch.setenv("MK_JIT_SHAPE", "machine")
    if policy.startswith("pool") or policy.startswith("k"):
        monkeypatch.setenv("MK_JIT_POOL", policy.lstrip("pokl"))
    else:
        monkeypatch.setenv("MK_JIT_POLICY", policy)
    cases = [("c2", mk.networks.example_network(), po.gen_inputs(SEED, 5000), {}),
             ("c3", mk.networks.sample_network(), po.gen_inputs(SEED, 5000), {}),
             ("c5", mk.networks.countdown_network(), po.gen_inputs(SEED, 5000, kind=1, mask=1023), {}),
             ("c5b", mk.networks.countdown_network(), po.gen_inputs(SEED, 3000, kind=1, mask=1023), {"budget": 700})]
    for seed in range(0, 240, 7):
        kw = dict(budget=[37, 200, 1000][seed % 3], stack_cap=[1, 3, 8, 16, 17, 40, 1024][seed % 7],
                  stop_on_output=(seed % 5 == 4))
        cases.append((f"seed{seed}", random_network(seed), po.gen_inputs(seed * 7919 + 1, 777), kw))
    for label, nodes, xs, kw in cases:
        net = mk.Network(nodes)
        got = net.compute_batch(xs, **kw)
        plan = net.plan(stack_cap=kw.get("stack_cap"), stop_on_output=kw.get("stop_on_output", False))
        if label.startswith("c"):
            assert "shape=machine" in plan, plan
            assert ("-pool" in plan) == policy.startswith("pool"), plan
            assert ("machine-k" in plan) == policy.startswith("k"), plan
        assert_same(got, oracle(nodes, xs, **kw), f"{label} policy {policy}")


# Deferred counters (MK_FLAG_DEFER_STATS + mk_stats_fold) add up to the same
# totals as per-launch folding, and to the oracle's, on every tier.
@pytest.mark.parametrize("mode", ["auto", "tile", "interp"])
def test_deferred_stats_fold(gpu, mode):
    import torch

    nodes = mk.networks.countdown_network()
    net = mk.Network(nodes)
    n = 5000
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    st = torch.empty(n, dtype=torch.uint8, device="cuda")
    s_imm = torch.zeros(N.MK_STATS_LEN, dtype=torch.int64, device="cuda")
    s_def = torch.zeros(N.MK_STATS_LEN, dtype=torch.int64, device="cuda")
    sh = torch.cuda.current_stream().cuda_stream
    kw = dict(out_ptr=out.data_ptr(), status_ptr=st.data_ptr(), gen_kind=N.MK_GEN_MASKED, gen_mask=1023,
              stream=sh, mode=_m(mode))
    for seed in (1, 2, 3):
        net.compute_device(n, stats_ptr=s_imm.data_ptr(), seed=seed, **kw)
    for seed in (1, 2, 3):
        net.compute_device(n, stats_ptr=None, seed=seed, defer_stats=True, **kw)
    net.stats_fold(s_def.data_ptr(), stream=sh)
    torch.cuda.synchronize()
    assert s_imm.tolist() == s_def.tolist()
    steps = sum(int(oracle(nodes, po.gen_inputs(seed, n, kind=1, mask=1023))[2].sum()) for seed in (1, 2, 3))
    assert s_def[0].item() == steps and s_def[2].item() == 3 * n


# ---- stateful sessions (row f2): GPU vs the oracle's session restatement ----
def _session_pair(nodes, n, **kw):
    cap = kw.get("stack_cap")
    g = mk.Network(nodes).sessions(n, budget=kw.get("budget"), stack_cap=cap)
    o = po.OracleSessions(po.OracleNet(nodes), n, stack_cap=cap)
    return g, o


def _session_calls(nodes, seqs, resumes=2, **kw):
    """Every row is one call on every instance; calls left open by their
    budget slice are resumed ``resumes`` times, then the rest are cancelled,
    on both sides (mk_session_step(NULL) / mk_session_cancel vs the oracle's
    session_step / orc_sessions_cancel)."""
    g, o = _session_pair(nodes, seqs.shape[1], **kw)
    b = kw.get("budget")
    for k, row in enumerate(seqs):
        got = g.compute(row)
        assert_same(got, o.compute(row, budget=b, threads=THREADS), f"call {k}")
        for j in range(resumes):
            if not ((got.status & N.MK_ST_REASON_MASK) == N.MK_ST_BUDGET).any():
                break
            got = g.resume()
            assert_same(got, o.resume(budget=b, threads=THREADS), f"call {k} resume {j}")
        g.cancel()
        o.cancel()
    return g, o


def test_sessions_example_network(gpu):
    seqs = po.gen_inputs(SEED, 6 * 3000).reshape(6, 3000)
    g, _ = _session_calls(mk.networks.example_network(), seqs)
    r = g.compute(np.full(3000, 5))
    assert (r.out == 7).all() and (r.status == N.MK_ST_HAS_OUTPUT).all()


def test_sessions_countdown_and_reset(gpu):
    nodes = mk.networks.countdown_network()
    seqs = po.gen_inputs(SEED, 4 * 2000, kind=1, mask=1023).reshape(4, 2000)
    g, o = _session_calls(nodes, seqs, budget=3000)
    g.reset()
    o.reset()
    row = po.gen_inputs(7, 2000, kind=1, mask=1023)
    assert_same(g.compute(row), o.compute(row, budget=3000), "after reset")


@pytest.mark.parametrize("seed", range(0, 60))
def test_sessions_random_networks(gpu, seed):
    rows = random_network(seed)
    cap = [1, 3, 8, 16, 17, 40, 1024][seed % 7]
    seqs = po.gen_inputs(seed * 131 + 5, 5 * 300).reshape(5, 300)
    _session_calls(rows, seqs, budget=[37, 200, 1000][seed % 3], stack_cap=cap)


def test_sessions_deep_stacks(gpu):
    nodes = mk.networks.pipeline_network(64)
    seqs = po.gen_inputs(SEED, 3 * 500).reshape(3, 500)
    _session_calls(nodes, seqs)


# Sequential calls in one launch (mk_session_compute_seq): identical to the
# same calls made one launch each, and to the oracle's session restatement.
@pytest.mark.parametrize("seed", range(0, 24))
def test_session_seq_matches_single_calls(gpu, seed):
    rows = random_network(seed) if seed else mk.networks.countdown_network()
    cap = [1, 3, 8, 16, 17, 40, 1024][seed % 7]
    budget = [37, 200, 1000][seed % 3]
    seqs = po.gen_inputs(seed * 977 + 3, 7 * 200, kind=1 if not seed else 0, mask=1023).reshape(7, 200)
    g, o = _session_pair(rows, 200, budget=budget, stack_cap=cap)
    got = g.compute_seq(seqs)
    for k, row in enumerate(seqs):
        ref = o.compute(row, budget=budget, threads=THREADS)
        assert_same(mk.network.BatchResult(got.out[k], got.status[k], got.steps[k]), ref, f"seq call {k}")
    # the state after the burst continues like the oracle's: calls still open
    # report MK_ST_CALL_OPEN (MK_EBUSY), then resume; cancelled, a new call runs
    row = po.gen_inputs(seed + 11, 200)
    assert_same(g.compute(row, busy_ok=True), o.compute(row, budget=budget, threads=THREADS), "after burst")
    assert_same(g.resume(), o.resume(budget=budget, threads=THREADS), "resumed after burst")
    g.cancel()
    o.cancel()
    assert_same(g.compute(row), o.compute(row, budget=budget, threads=THREADS), "after cancel")


def test_session_seq_single_instance_long_burst(gpu):
    # the master's stateful mode: one instance, a burst of 4,096 calls
    nodes = [("acc", "program", "IN ACC\nADD R0\nMOV ACC, acc:R0\nOUT ACC\nMOV R0, ACC\nMOV ACC, acc:R0")]
    g = mk.Network(nodes).sessions(1)
    xs = po.gen_inputs(SEED, 4096)
    r = g.compute_seq(xs)
    o = po.OracleSessions(po.OracleNet(nodes), 1)
    ref = [o.compute([x]) for x in xs.tolist()]
    assert r.out.tolist() == [int(x[0][0]) for x in ref] and r.status.tolist() == [int(x[1][0]) for x in ref]


# The device API on a caller's stream and the host API on the handle's own
# stream share the handle's stack slots and counters: the library orders
# them (mk_exec.hip order_on), so interleaved launches stay exact.
def test_device_and_host_api_interleaved_streams(gpu):
    import torch

    nodes = mk.networks.pipeline_network(64)
    net = mk.Network(nodes)
    n = 1 << 16
    side = torch.cuda.Stream()
    outs = []
    for rep in range(3):
        out = torch.empty(n, dtype=torch.int32, device="cuda")
        st = torch.empty(n, dtype=torch.uint8, device="cuda")
        net.compute_device(n, out_ptr=out.data_ptr(), status_ptr=st.data_ptr(), seed=SEED + rep,
                           stream=side.cuda_stream)
        xs = po.gen_inputs(SEED + 100 + rep, 2048)
        host = net.compute_batch(xs)  # enqueued while the side-stream launch may still run
        outs.append((out, st, xs, host, rep))
    torch.cuda.synchronize()
    for out, st, xs, host, rep in outs:
        assert_same(host, oracle(nodes, xs), f"host API rep {rep}")
        tail = po.gen_inputs(SEED + rep, n)[-1024:]
        ref = oracle(nodes, tail)
        assert np.array_equal(out.cpu().numpy()[-1024:], ref[0]) and np.array_equal(st.cpu().numpy()[-1024:], ref[1])


# Lane trace (mk_trace_lane): the interpreter's record
# of every retired instruction of one lane equals the oracle's
# (orc_trace_lane) -- round, node, ptr, ACC and BAK after each instruction.
@pytest.mark.parametrize("seed", range(0, 40))
def test_lane_trace_matches_oracle(gpu, seed):
    if seed < 4:
        nodes = [mk.networks.example_network, mk.networks.sample_network, mk.networks.countdown_network,
                 lambda: mk.networks.pipeline_network(8)][seed]()
    else:
        nodes = random_network(seed)
    onet = po.OracleNet(nodes)
    net = mk.Network(nodes)
    for x in po.gen_inputs(seed + 17, 3).tolist() + [0, 7]:
        kw = dict(budget=[37, 200, 5000][seed % 3], stack_cap=[3, 16, 1024][seed % 3])
        got, st = net.trace(x, max_entries=512, **kw)
        ref, rst = po.trace_lane(onet, x, max_entries=512, **kw)
        assert st == rst, (seed, x, st, rst)
        assert got.tobytes() == ref.tobytes(), (seed, x, got[:8], ref[:8])


# The host API stages calls of up to MK_HOST_CHUNK inputs through pinned
# memory and larger ones straight from the caller's buffers: both paths,
# alternating on one handle (buffers are re-sized), steps on and off.
@pytest.mark.parametrize("chunk", [1000, 4096])
def test_host_api_chunks(gpu, monkeypatch, chunk):
    monkeypatch.setenv("MK_HOST_CHUNK", str(chunk))
    for (nodes, gen), n in zip([(mk.networks.countdown_network(), dict(kind=1, mask=1023)),
                                (mk.networks.pipeline_network(16), {}), (mk.networks.sample_network(), {}),
                                (mk.networks.countdown_network(), dict(kind=1, mask=1023))],
                               [10007, chunk, 977, 10007]):
        net = mk.Network(nodes)
        xs = po.gen_inputs(SEED + chunk + n, n, **gen)
        ref = oracle(nodes, xs)
        assert_same(net.compute_batch(xs), ref, f"chunk {chunk}")
        got = net.compute_batch(xs, steps=False)
        assert np.array_equal(got.out, ref[0]) and np.array_equal(got.status, ref[1]) and got.steps is None


def test_host_api_device_mask(gpu):
    # device_mask selects the GPUs of an in-process shard; naming a GPU that
    # does not exist is an error (never a silent fallback)
    import torch

    net = mk.Network(mk.networks.example_network())
    xs = po.gen_inputs(SEED, 3000)
    ndev = torch.cuda.device_count()
    assert_same(net.compute_batch(xs, devices=range(ndev)), oracle(mk.networks.example_network(), xs), "all GPUs")
    with pytest.raises(N.MkError) as e:
        net.compute_batch(xs, devices=[ndev])
    assert e.value.code == N.MK_EINVAL


# Machine-shape launches of >= 64K inputs run the inputs grouped by value
# (order_* kernels, lane j answers input order[j]); every input is answered
# at its own index, identically to the input-order launch (MK_JIT_ORDER=0).
@pytest.mark.parametrize("kind", ["gen", "i32", "i64"])
def test_machine_input_order_is_transparent(gpu, monkeypatch, kind):
    import torch

    n = 200_003
    cases = [("c5", mk.networks.countdown_network(), (N.MK_GEN_MASKED, 1023))]
    for seed in (3, 17, 41):
        rows = random_network(seed)
        cases.append((f"seed{seed}", rows, (N.MK_GEN_FULL, 0)))
    # "1": global order by value (MK_JIT_ORDER); "0": the default tile-sorted
    # kernel; "dyn" / "snake": the tile-sorted kernel with its chunks taken by
    # free waves / in snake order (MK_JIT_TS_DYN); "plain": input order
    # (MK_JIT_TILE_SORT=0)
    variants = {"1": ("1", "1", None), "0": ("0", "1", None), "dyn": ("0", "1", "1"), "snake": ("0", "1", "0"),
                "plain": ("0", "0", None)}
    for label, nodes, gen in cases:
        res = {}
        for order, (o, ts, dyn) in variants.items():
            monkeypatch.setenv("MK_JIT_ORDER", o)
            monkeypatch.setenv("MK_JIT_TILE_SORT", ts)
            if dyn is None:
                monkeypatch.delenv("MK_JIT_TS_DYN", raising=False)
            else:
                monkeypatch.setenv("MK_JIT_TS_DYN", dyn)
            net = mk.Network(nodes)
            if "shape=machine" not in net.plan():
                monkeypatch.setenv("MK_JIT_SHAPE", "machine")
                net = mk.Network(nodes)
                monkeypatch.delenv("MK_JIT_SHAPE")
            xs = torch.from_numpy(po.gen_inputs(SEED, n, kind=gen[0], mask=gen[1]))
            if kind == "gen":
                res[order] = _device_run(net, n, gen=gen)
            elif kind == "i32":
                res[order] = _device_run(net, n, in_tensor=xs.to(torch.int32).cuda(), in_kind=N.MK_IN_I32)
            else:
                res[order] = _device_run(net, n, in_tensor=xs.cuda(), in_kind=N.MK_IN_I64)
        for k in ("0", "dyn", "snake", "plain"):
            for a, b in zip(res["1"], res[k]):
                assert np.array_equal(a, b), (label, k)
        ref = oracle(nodes, po.gen_inputs(SEED, n, kind=gen[0], mask=gen[1])[-3000:])
        out, st, sp, _ = res["1"]
        assert np.array_equal(out[-3000:], ref[0]) and np.array_equal(st[-3000:], ref[1]) and \
            np.array_equal(sp[-3000:], ref[2]), label


# ---- native-tier sessions (tis_jit.h mk_sess_exec) ------
# The session tests above run on the native tier whenever the network
# compiles (a call that reaches its budget slice inside a superblock is
# handed to the interpreter mid-call).  Here: which tier, both tiers against
# each other and the oracle, and hand-offs inside bursts.

def test_sessions_native_tier_plans(gpu):
    for nodes in (mk.networks.example_network(), mk.networks.countdown_network(), mk.networks.sample_network(),
                  mk.networks.pipeline_network(64)):
        s = mk.Network(nodes).sessions(4)
        assert s.plan().startswith("tier=native"), s.plan()
        s.close()


def test_sessions_interp_when_disabled(gpu, monkeypatch):
    monkeypatch.setenv("MK_SESSION_NATIVE", "0")
    s = mk.Network(mk.networks.example_network()).sessions(4)
    assert s.plan().startswith("tier=interp reason=disabled"), s.plan()
    r = s.compute([5, 6, 7, 8])
    assert r.out.tolist() == [7, 8, 9, 10]


@pytest.mark.parametrize("seed", range(0, 16))
def test_sessions_native_handoff_bursts(gpu, seed):
    # countdowns whose long calls cross the budget inside a burst: the native
    # kernel answers the calls before the hand-off, the interpreter the rest
    nodes = mk.networks.countdown_network() if seed % 2 == 0 else random_network(seed)
    budget = [150, 400, 1000, 3000][seed % 4]
    g, o = _session_pair(nodes, 256, budget=budget)
    seqs = po.gen_inputs(seed * 5 + 1, 5 * 256, kind=1, mask=1023).reshape(5, 256)
    got = g.compute_seq(seqs)
    for k, row in enumerate(seqs):
        assert_same(mk.network.BatchResult(got.out[k], got.status[k], got.steps[k]),
                    o.compute(row, budget=budget, threads=THREADS), f"burst call {k}")
    for j in range(3):
        assert_same(g.resume(), o.resume(budget=budget, threads=THREADS), f"resume {j}")
    g.cancel()
    o.cancel()
    row = po.gen_inputs(seed + 99, 256, kind=1, mask=1023)
    assert_same(g.compute(row), o.compute(row, budget=budget, threads=THREADS), "after burst")


def test_sessions_native_vs_interp_large(gpu, monkeypatch):
    # the C2 network at 65,536 instances x 6 calls: native and interpreter agree
    nodes = mk.networks.example_network()
    xs = po.gen_inputs(SEED, 6 * 65536).reshape(6, 65536)
    a = mk.Network(nodes).sessions(65536)
    assert a.plan().startswith("tier=native")
    monkeypatch.setenv("MK_SESSION_NATIVE", "0")
    b = mk.Network(nodes).sessions(65536)
    for row in xs:
        ra, rb = a.compute(row), b.compute(row)
        assert np.array_equal(ra.out, rb.out) and np.array_equal(ra.status, rb.status)
        assert np.array_equal(ra.steps, rb.steps)


# Device-array session APIs (mk_session_compute_device on a caller stream,
# mk_session_compute_seq_device bursts; bench.py's sessions leg) against the
# oracle's sessions: the same calls in the same order, one launch per call or
# one launch per burst, with budget slices that hand calls off mid-burst.
@pytest.mark.parametrize("seed", [0, 3, 7, 12])
def test_session_device_bursts_match_oracle(gpu, seed):
    import torch

    nodes = mk.networks.example_network() if seed == 0 else random_network(seed)
    n, calls = 1000, 5
    budget = None if seed == 0 else [300, 1000, 5000][seed % 3]
    xs = po.gen_inputs(seed * 31 + 7, calls * n, kind=0 if seed == 0 else 1, mask=1023).reshape(calls, n)
    o = po.OracleSessions(po.OracleNet(nodes), n)
    refs = [o.compute(row, budget=budget, threads=THREADS) for row in xs]
    s = torch.cuda.Stream()
    x = torch.from_numpy(xs).cuda()
    for burst in (False, True):
        g = mk.Network(nodes).sessions(n, budget=budget)
        out = torch.empty((calls, n), dtype=torch.int32, device="cuda")
        st = torch.empty((calls, n), dtype=torch.uint8, device="cuda")
        sp = torch.empty((calls, n), dtype=torch.int32, device="cuda")
        torch.cuda.synchronize()
        if burst:
            g.compute_seq_device(x.data_ptr(), calls, out.data_ptr(), st.data_ptr(), sp.data_ptr(),
                                 stream=s.cuda_stream)
        else:
            for c in range(calls):
                g.compute_device(x[c].data_ptr(), out[c].data_ptr(), st[c].data_ptr(), sp[c].data_ptr(),
                                 stream=s.cuda_stream)
        s.synchronize()
        for c in range(calls):
            got = mk.network.BatchResult(out[c].cpu().numpy(), st[c].cpu().numpy(),
                                         sp[c].cpu().numpy().astype(np.uint32))
            assert_same(got, refs[c], f"burst={burst} call {c}")
        g.close()


# Consecutive calls of one session set on different streams, with no host
# synchronisation between the device calls: two caller streams, the null
# stream (the session's own) and the host API.  Each call needs the state the
# previous one left, so the library's cross-stream ordering (mk_exec.hip
# session_wait_last / session_mark) is what keeps the results exact.  C5's
# countdown network: long kernels, and machine modules dispatching by sweeps.
def test_session_calls_across_streams_match_oracle(gpu):
    import torch

    nodes = mk.networks.countdown_network()
    n, calls = 1 << 15, 7
    xs = po.gen_inputs(77, calls * n, kind=1, mask=1023).reshape(calls, n)
    o = po.OracleSessions(po.OracleNet(nodes), n)
    refs = [o.compute(row, threads=THREADS) for row in xs]
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    x = torch.from_numpy(xs).cuda()
    torch.cuda.synchronize()
    g = mk.Network(nodes).sessions(n)
    out = torch.empty((calls, n), dtype=torch.int32, device="cuda")
    st = torch.empty((calls, n), dtype=torch.uint8, device="cuda")
    sp = torch.empty((calls, n), dtype=torch.int32, device="cuda")
    host = {}
    for c, where in enumerate(["s1", "s2", "null", "s1", "host", "s2", "s2"]):
        if where == "host":
            host[c] = g.compute(xs[c])
            continue
        stream = {"s1": s1.cuda_stream, "s2": s2.cuda_stream, "null": None}[where]
        g.compute_device(x[c].data_ptr(), out[c].data_ptr(), st[c].data_ptr(), sp[c].data_ptr(), stream=stream)
    torch.cuda.synchronize()
    for c in range(calls):
        got = host[c] if c in host else mk.network.BatchResult(out[c].cpu().numpy(), st[c].cpu().numpy(),
                                                               sp[c].cpu().numpy().astype(np.uint32))
        assert_same(got, refs[c], f"call {c}")
    g.close()


@pytest.mark.gpu
@pytest.mark.parametrize("fill", ["zeros", "sevens", "halves"])
def test_machine_tiles_of_equal_inputs(gpu, fill):
    """The tile-sorted machine kernel skips its histogram when a tile holds
    one value (tis_jit.cpp kMachineSortKernel, span 0): C5 over all-equal
    tiles, a partial last tile, and tiles mixing one repeated value with
    ordinary inputs, bit-exact against the oracle with the counters."""
    import torch

    n = 3 * 1024 + 517  # three whole tiles of 1,024 and a partial one
    xs = np.zeros(n, np.int64)
    if fill == "sevens":
        xs[:] = 7
    elif fill == "halves":  # every other tile one value, the others random
        xs[:] = po.gen_inputs(SEED, n, kind=N.MK_GEN_MASKED, mask=1023)
        for t in range(0, n, 2048):
            xs[t:t + 1024] = 300
    nodes = mk.networks.countdown_network()
    net = mk.Network(nodes)
    assert "shape=machine" in net.plan()
    got = _device_run(net, n, in_tensor=torch.from_numpy(xs.astype(np.int32)).cuda(), in_kind=N.MK_IN_I32)
    ref = po.OracleNet(nodes).compute_batch(xs)
    for g_, r_ in zip(got[:3], ref[:3]):
        np.testing.assert_array_equal(g_, r_)
    assert int(got[3][0]) == int(np.asarray(ref[2], np.uint64).sum())  # retired steps
