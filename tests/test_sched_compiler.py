"""Schedule compiler (tier 2, misaka-net_amd/csrc/tis_sched.cpp) against the
oracle, executed by the host model of the superblock kernel
(lib/libmisaka_amd_check.so) -- no GPU needed.  The GPU runs the same
micro-op streams in tests/test_gpu_parity.py."""
import numpy as np
import pytest

import misaka_net_amd as mk
from oracle import pyoracle as po
import schedcheck as sc
from tisgen import random_network, stack_loop_network

SEED = 0x4D49534B41


def same(nodes, xs, **kw):
    o, s, p, _ = sc.emulate(nodes, xs, **kw)
    ro, rs, rp = po.OracleNet(nodes).compute_batch(xs, **kw)
    bad = np.nonzero((o != ro) | (s != rs) | (p != rp))[0]
    assert not bad.size, (int(bad[0]), (o[bad[0]], s[bad[0]], p[bad[0]]), (ro[bad[0]], rs[bad[0]], rp[bad[0]]))


@pytest.mark.parametrize("name", sorted(mk.networks.CONFIGS))
def test_configs(name):
    nodes = mk.networks.CONFIGS[name]()
    kind = 1 if name.startswith("c5") else 0
    xs = po.gen_inputs(SEED, 3000, kind=kind, mask=1023)
    same(nodes, xs)


def test_example_compiles_to_straight_line():
    o, s, p, plan = sc.emulate(mk.networks.example_network(), [5], want_plan=True)
    assert plan.splitlines()[0].startswith("superblocks=1 ")
    fast = plan.split("(checked)")[0]
    ops = [l.split()[1] for l in fast.splitlines()[2:] if l.startswith("  ") and not l.strip().startswith("ext")]
    assert ops == ["GUARD", "ADDI", "ADDI", "END"], ops


def test_deep_pipeline_d1024():
    same(mk.networks.pipeline_network(1024), po.gen_inputs(SEED, 40))


@pytest.mark.parametrize("depth", [64, 1024])
def test_observe_pipeline(depth):
    same(mk.networks.pipeline_network(depth, observe=True), po.gen_inputs(SEED, 40))


@pytest.mark.parametrize("budget", [1, 5, 11, 12, 13, 100])
def test_budget_boundaries(budget):
    same(mk.networks.example_network(), po.gen_inputs(SEED, 64), budget=budget)
    same(mk.networks.countdown_network(), po.gen_inputs(SEED, 64, kind=1, mask=1023), budget=budget * 37)


def test_stop_on_output_and_overflow():
    same(mk.networks.sample_network(), po.gen_inputs(SEED, 200), stop_on_output=True)
    same(mk.networks.pipeline_network(64), po.gen_inputs(SEED, 20), stack_cap=63)


def test_constant_spin_loops_generalise():
    nodes = [("a", "program", "L: ADD 1\nJMP L"), ("b", "program", "IN ACC\nJRO 0")]
    same(nodes, [1, 2, 3], budget=5000)


def test_random_networks():
    declined = 0
    for seed in range(0, 600):
        rows = random_network(seed)
        xs = po.gen_inputs(seed * 7919 + 1, 48)
        kw = dict(budget=[37, 200, 1000][seed % 3], stack_cap=[1, 3, 8, 16, 17, 40, 1024][seed % 7],
                  stop_on_output=(seed % 5 == 4))
        try:
            same(rows, xs, **kw)
        except sc.NotCompiled:
            declined += 1
    assert declined < 30


def test_wide_immediates_on_symbolic_acc():
    prog = ("IN ACC\nADD 2147483648\nADD 4294967295\nSUB 2147483649\nADD -4294967296\n"
            "ADD 9223372036854775807\nSUB -9223372036854775808\nMOV ACC, n:R1\nMOV R1, ACC\n"
            "JRO 2147483648\nNOP\nOUT ACC\nJLZ L\nOUT 1\nL: OUT 2")
    same([("n", "program", prog)], po.gen_inputs(SEED, 500))


def test_dynamic_stack_networks():
    # stack depths that follow the data: the compiler's dynamic stacks
    # (tisgen.stack_loop_network), host model vs oracle over capacities and
    # budgets; every one of them compiles now
    for seed in range(300):
        rows, gen = stack_loop_network(seed)
        xs = po.gen_inputs(seed + 5, 64, **gen)
        for cap, budget in ((None, None), (3, 200), (17, 1000), (64, 57)):
            kw = {k: v for k, v in (("stack_cap", cap), ("budget", budget)) if v is not None}
            same(rows, xs, **kw)


def test_exit_moves_keep_the_branch_operand():
    # regressions of canonicalize: a SWP-driven swap of two homes (a move
    # cycle) at a branch on ACC, and a cycle temp that took a home written by
    # an earlier move of the same exit
    a = "IN ACC\nL0: PUSH 4, s0\nSUB 2\nJGZ L0\nL1: SWP\nSWP\nSWP\nPUSH ACC, s1\nPOP s0, ACC\nSWP\nJGZ L1"
    rows = [("b", "program", "C: POP s0, ACC\nADD 1\nSWP\nJMP C"), ("s0", "stack", ""), ("s1", "stack", ""),
            ("a", "program", a)]
    same(rows, np.arange(0, 64))
    a = "IN ACC\nSAV\nL2: NOP\nPUSH ACC, s0\nSWP\nSUB 1\nJGZ L2\nPUSH -1, s0\nMOV R0, ACC\nOUT ACC"
    b = "C: POP s0, ACC\nJLZ E\nSWP\nADD 1\nSWP\nJMP C\nE: SWP\nMOV ACC, a:R0"
    same([("s0", "stack", ""), ("a", "program", a), ("b", "program", b)], np.arange(0, 80))


def _push_pop(stk, depth, tag):
    """PUSH depth values (a+1, a+2, ... for a = ACC) onto `stk`, POP them folding sum = 2*sum + v
    into ACC."""
    return ["SAV", f"MOV {depth}, ACC", f"{tag}P: SWP", "ADD 1", f"PUSH ACC, {stk}", "SWP", "SUB 1", f"JGZ {tag}P",
            "MOV 0, ACC", "SAV", f"MOV {depth}, ACC", f"{tag}Q: SWP", "MOV ACC, a:R3", f"POP {stk}, ACC",
            "MOV ACC, a:R2", "MOV R3, ACC", "ADD ACC", "ADD R2", "SWP", "SUB 1", f"JGZ {tag}Q", "SWP"]


# Stacks share slots only when their windows of slot accesses cannot overlap
# on any lane (tis_sched.cpp share_slots): used one after the other they
# share -- also behind a data-dependent branch whose two arms use them in
# opposite orders, or when only one arm uses one of them -- and interleaved
# they do not.  Every network is checked against the oracle on the host model.
@pytest.mark.parametrize("shape", ["sequential", "interleaved", "branch_orders", "branch_one_arm"])
def test_slot_sharing_is_safe(shape):
    D = 40
    S = lambda n: (n, "stack", "")  # noqa: E731
    if shape == "sequential":
        body = ["IN ACC"] + _push_pop("s0", D, "A") + _push_pop("s1", D, "B") + ["OUT ACC"]
    elif shape == "interleaved":
        push = lambda s, t: [f"MOV {D}, ACC", f"{t}: SWP", "ADD 1", f"PUSH ACC, {s}", "SWP", "SUB 1", f"JGZ {t}"]  # noqa
        body = (["IN ACC", "SAV"] + push("s0", "P0") + push("s1", "P1") + ["MOV 0, ACC", "SAV"] +
                [f"MOV {D}, ACC", "L: SWP", "MOV ACC, a:R3", "POP s0, ACC", "MOV ACC, a:R2", "POP s1, ACC",
                 "ADD R2", "ADD R3", "ADD R3", "ADD R3", "SWP", "SUB 1", "JGZ L", "SWP", "OUT ACC"])
    elif shape == "branch_orders":
        body = (["IN ACC", "JGZ POS"] + _push_pop("s0", D, "A") + _push_pop("s1", D, "B") +
                ["OUT ACC", "JMP E", "POS: NOP"] + _push_pop("s1", D, "C") + _push_pop("s0", D, "F") +
                ["OUT ACC", "E: NOP"])
    else:
        body = (["IN ACC", "JGZ POS"] + _push_pop("s0", D, "A") + ["POS: NOP"] + _push_pop("s1", D, "B") +
                ["OUT ACC"])
    nodes = [("a", "program", "\n".join(body)), S("s0"), S("s1")]
    xs = po.gen_inputs(SEED, 300)
    xs[:4] = [0, 1, -1, 2147483647]
    same(nodes, xs)
    slots = sc.jit_lane(nodes)[1]
    own = (D - 23) * 2  # each stack's spilled depths, unshared
    assert (slots < own) == (shape != "interleaved"), (shape, slots)
