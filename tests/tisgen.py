"""Seeded random TIS programs / networks for parity fuzzing.

Two generators:
  * ``random_network`` -- loadable networks exercising every instruction
    form, every source, edge immediates (int32/int64 bounds, Atoi range
    errors), ports, stacks, unknown hosts, wrong-service targets and the
    master name.  Used for oracle-vs-GPU bit-exact tests.
  * ``mutated_line`` -- text-level mutations of valid lines (whitespace
    classes incl. \\v and \\f, case, commas, signs, labels, comments) for
    parser accept/reject/error-text parity.
"""
from __future__ import annotations

import random

IMM_EDGES = [
    "0", "1", "-1", "2", "-2", "7", "100", "-100", "1000",
    "2147483647", "-2147483648", "2147483648", "-2147483649", "4294967296", "4294967301",
    "9223372036854775807", "-9223372036854775808",
    "9223372036854775808", "-9223372036854775809", "99999999999999999999",  # Atoi range errors
    "007", "-0",
]
SRCS = ["ACC", "NIL", "R0", "R1", "R2", "R3"]
REGS = ["R0", "R1", "R2", "R3"]


def rand_imm(r: random.Random) -> str:
    if r.random() < 0.6:
        return str(r.randint(-20, 20))
    return r.choice(IMM_EDGES)


def random_program(r: random.Random, progs, stacks, others, nlines=None, allow_in=True, allow_out=True):
    nlines = nlines or r.randint(1, 12)
    labels = [f"L{i}" for i in range(r.randint(0, 3))]
    label_lines = r.sample(range(nlines), min(len(labels), nlines))
    labels = labels[: len(label_lines)]
    lines = []
    for i in range(nlines):
        kind = r.random()
        targets_prog = progs + others
        targets_stack = stacks + others + progs[:1]
        if kind < 0.05:
            body = ""
        elif kind < 0.08:
            body = "# comment " + str(r.randint(0, 9))
        else:
            f = r.choice(
                ["NOP", "SWP", "SAV", "NEG", "MOVL", "MOVL", "MOVN", "MOVN", "ADD", "ADD", "SUB", "JMP", "JCC",
                 "JCC", "JRO", "PUSH", "POP", "IN", "OUT", "OUT"]
            )
            if f in ("NOP", "SWP", "SAV", "NEG"):
                body = f
            elif f == "MOVL":
                src = rand_imm(r) if r.random() < 0.4 else r.choice(SRCS)
                body = f"MOV {src}, {r.choice(['ACC', 'NIL'])}"
            elif f == "MOVN":
                src = rand_imm(r) if r.random() < 0.3 else r.choice(SRCS)
                body = f"MOV {src}, {r.choice(targets_prog)}:{r.choice(REGS)}"
            elif f in ("ADD", "SUB"):
                src = rand_imm(r) if r.random() < 0.5 else r.choice(SRCS)
                body = f"{f} {src}"
            elif f in ("JMP", "JCC"):
                if not labels:
                    body = "NOP"
                else:
                    op = "JMP" if f == "JMP" else r.choice(["JEZ", "JNZ", "JGZ", "JLZ"])
                    lab = r.choice(labels)
                    body = f"{op} {lab.lower() if r.random() < 0.2 else lab}"
            elif f == "JRO":
                src = str(r.randint(-4, 4)) if r.random() < 0.4 else (rand_imm(r) if r.random() < 0.2 else r.choice(SRCS))
                body = f"JRO {src}"
            elif f == "PUSH":
                src = rand_imm(r) if r.random() < 0.3 else r.choice(SRCS)
                body = f"PUSH {src}, {r.choice(targets_stack)}"
            elif f == "POP":
                body = f"POP {r.choice(targets_stack)}, {r.choice(['ACC', 'NIL'])}"
            elif f == "IN":
                body = f"IN {r.choice(['ACC', 'NIL'])}" if allow_in else "NOP"
            else:
                src = rand_imm(r) if r.random() < 0.3 else r.choice(SRCS)
                body = f"OUT {src}" if allow_out else "NOP"
        if i in label_lines:
            lab = labels[label_lines.index(i)]
            sep = r.choice([" ", "", "  ", "\t"])
            body = f"{lab}:{sep}{body}"
        if r.random() < 0.15:
            body = r.choice([" ", "\t", "  "]) + body
        lines.append(body)
    text = "\n".join(lines)
    if r.random() < 0.5:
        text += "\n"
    return text


def random_network(seed: int, max_prog=5, max_stack=3):
    """Returns a list of (name, kind, program) rows."""
    r = random.Random(seed)
    pool = ["a", "b", "c", "node1", "node2", "Z9", "x_y", "misaka1", "misaka2", "p", "q", "ACC", "R0"]
    r.shuffle(pool)
    nprog = r.randint(1, max_prog)
    nstack = r.randint(0, max_stack)
    progs = pool[:nprog]
    stacks = pool[nprog: nprog + nstack]
    master = "master" if r.random() < 0.5 else None
    others = ["ghost"] + ([master] if master else [])
    rows = []
    in_node = r.choice(progs)
    for p in progs:
        text = random_program(r, progs, stacks, others, allow_in=(p == in_node or r.random() < 0.3))
        rows.append((p, "program", text))
    for s in stacks:
        rows.append((s, "stack", ""))
    if master:
        rows.append((master, "master", ""))
    r.shuffle(rows)
    return rows


WS = [" ", "\t", "  ", "\f", "\r", "\v", ""]


def mutated_line(r: random.Random) -> str:
    base = r.choice(
        [
            "NOP", "SWP", "SAV", "NEG", "MOV 1, ACC", "MOV -5, NIL", "MOV 3, a:R0", "MOV ACC, a:R1",
            "MOV R2, ACC", "MOV R3, b:R3", "ADD 1", "SUB -2", "ADD ACC", "SUB R1", "JMP L", "JEZ l", "JNZ L",
            "JGZ M", "JLZ L", "JRO 2", "JRO -1", "JRO R0", "PUSH 5, s", "PUSH ACC, s", "POP s, ACC",
            "POP s, NIL", "IN ACC", "IN NIL", "OUT 1", "OUT ACC", "OUT R2", "L:", "L: NOP", "# c", "",
            "MOV ACC, ACC", "MOV NIL, NIL", "MOV 9223372036854775808, ACC",
        ]
    )
    ops = r.randint(0, 3)
    s = base
    for _ in range(ops):
        m = r.random()
        if m < 0.2 and " " in s:  # change a whitespace run
            i = s.index(" ")
            s = s[:i] + r.choice(WS) + s[i + 1:]
        elif m < 0.3 and ", " in s:
            s = s.replace(", ", r.choice([",", " ,", " , ", ",\t", ",  ", ",\v"]), 1)
        elif m < 0.4:
            s = s.lower() if r.random() < 0.5 else s.capitalize()
        elif m < 0.5:
            s = r.choice(WS) + s
        elif m < 0.6:
            s = s + r.choice(WS + ["#", " # c", "x", ","])
        elif m < 0.7:
            s = r.choice(["L:", "L: ", "l:", "  L:\t", "M:", "1:", "_:"]) + s
        elif m < 0.8:
            s = s.replace("1", r.choice(["+1", "--1", "1a", "01", "- 1", "1 2"]), 1)
        elif m < 0.9:
            s = s.replace("R", r.choice(["R", "r", "R4", "RR"]), 1)
        else:
            s = s.replace("a:", r.choice(["a :", "a: ", ":", "a::", "a-b:"]), 1)
    return s


def mutated_program(seed: int) -> str:
    r = random.Random(seed)
    lines = [mutated_line(r) for _ in range(r.randint(1, 6))]
    if r.random() < 0.3:
        lines.append("L:")
    return "\n".join(lines)


# ---- self-loop shapes of the native machine kernel -----------------------------
# Each targets one path of the generated loop (tis_jit.cpp emit_self_loop):
# the 32-bit induction phase and its range check (values near +-2^30, steps
# of 1 and of ~2^30), the 64-bit phase (int64 wrap), loops with no induction
# register (step counter), JMP-only loops that only the budget ends, and
# budgets that end inside a loop (guarded phase).
def _edge_inputs(rng: random.Random, n: int, lo: int, hi: int) -> list:
    edges = [0, 1, -1, 2**30, -(2**30), 2**30 + 1, -(2**30) - 1, 2**31 - 1, -(2**31), 2**31 - 2, -(2**31) + 1]
    return [rng.choice(edges) if rng.random() < 0.2 else rng.randint(lo, hi) for _ in range(n)]


def loop_cases(n: int = 512, seed: int = 7):
    """[(label, nodes, inputs, kwargs)] for the oracle-vs-native loop tests."""
    rng = random.Random(seed)
    P = lambda text: [("n", "program", text)]  # noqa: E731
    return [
        ("up_by_1", P("IN ACC\nL: ADD 1\nJLZ L\nOUT ACC"), _edge_inputs(rng, n, -3000, 50), {}),
        ("up_by_1_budget", P("IN ACC\nL: ADD 1\nJLZ L\nOUT ACC"), _edge_inputs(rng, n, -3000, 50),
         {"budget": 2500}),
        ("down_by_7", P("IN ACC\nL: SUB 7\nJGZ L\nOUT ACC"), _edge_inputs(rng, n, -50, 20000), {"budget": 5000}),
        ("down_by_2pow30", P("IN ACC\nL: SUB 1073741823\nJGZ L\nOUT ACC"), _edge_inputs(rng, n, -5, 2**31 - 1), {}),
        ("swap_loop", P("IN ACC\nSAV\nL: SWP\nADD 1\nSWP\nSUB 1\nJGZ L\nSWP\nOUT ACC"),
         _edge_inputs(rng, n, -5, 900), {"budget": 6000}),
        ("jmp_forever", P("IN ACC\nL: ADD 3\nJMP L"), _edge_inputs(rng, n, -100, 100), {"budget": 999}),
        ("int64_wrap", P("IN ACC\nADD 9223372036854775000\nL: ADD 100\nJGZ L\nOUT ACC"),
         _edge_inputs(rng, n, -2000, 2000), {}),
        ("two_loops", [("a", "program", "IN ACC\nL: SUB 1\nJGZ L\nMOV 500, ACC\nM: SUB 2\nJGZ M\nOUT ACC")],
         _edge_inputs(rng, n, -10, 3000), {}),
        ("down_nz", P("IN ACC\nL: SUB 1\nJNZ L\nOUT ACC"), _edge_inputs(rng, n, -20, 2000), {"budget": 3000}),
        ("up_to_zero_jez", P("IN ACC\nL: ADD 2\nJEZ E\nJMP L\nE: OUT ACC"), _edge_inputs(rng, n, -2000, 20),
         {"budget": 3000}),
        ("doubling", P("IN ACC\nL: ADD ACC\nJGZ L\nOUT ACC"), _edge_inputs(rng, n, -5, 2**31 - 1), {}),
        ("neg_sub", P("IN ACC\nL: NEG\nSUB 1\nJLZ L\nOUT ACC"), _edge_inputs(rng, n, -99, 99), {"budget": 777}),
        ("loop_with_stack", [("a", "program", "IN ACC\nL: PUSH ACC, s\nSUB 1\nJGZ L\nPOP s, ACC\nOUT ACC"),
                             ("s", "stack", "")], _edge_inputs(rng, n, -3, 40), {"stack_cap": 64}),
    ]


# ---- census classes: network shapes that stress the schedule compiler -----------
from misaka_net_amd.networks import census_classes  # noqa: E402,F401  (defined with the bench workloads)


def stack_loop_network(seed: int):
    """Networks whose stack depths follow the data (the schedule compiler's
    dynamic stacks): loops with input-dependent trip counts that push and pop
    on 1-3 stacks, pops that may outnumber pushes (the POP then blocks), a
    second node popping what the first pushes (cross-node blocking), and
    values that reach the output (sums of popped values).  Returns
    (rows, gen kwargs for oracle.gen_inputs)."""
    r = random.Random(seed)
    ns = r.randint(1, 3)
    stacks = [f"s{k}" for k in range(ns)]
    lines = ["IN ACC"]
    if r.random() < 0.5:
        lines.append(f"ADD {r.randint(-3, 3)}")
    lines.append("SAV")
    consumer = r.random() < 0.35
    for k in range(r.randint(1, 3)):
        s = r.choice(stacks)
        lab = f"L{k}"
        body = []
        for _ in range(r.randint(1, 3)):
            c = r.random()
            if c < 0.45:
                body.append(f"PUSH ACC, {r.choice(stacks)}")
            elif c < 0.6:
                body.append(f"PUSH {r.randint(-5, 5)}, {r.choice(stacks)}")
            elif c < 0.8 and not consumer:
                body.append(f"POP {r.choice(stacks)}, NIL")
            else:
                # accumulate a popped value into BAK (ACC is the counter)
                body += ["SWP", f"PUSH ACC, {s}", f"POP {r.choice(stacks)}, ACC", "SWP"]
        step = r.choice([1, 1, 2, 3])
        jump = r.choice(["JGZ", "JGZ", "JNZ"]) if step == 1 else "JGZ"
        lines += [f"{lab}: " + body[0]] + body[1:] + [f"SUB {step}", f"{jump} {lab}"]
        if r.random() < 0.5:
            lines += ["SWP", "SAV"]  # the next loop counts from the running value
    if consumer:
        lines += [f"PUSH -1, {stacks[0]}", "MOV R0, ACC", "OUT ACC"]
        cons = (f"MOV 0, ACC\nSAV\nC: POP {stacks[0]}, ACC\nJLZ E\nSWP\nADD 1\nSWP\nJMP C\n"
                f"E: SWP\nMOV ACC, a:R0")
        rows = [("a", "program", "\n".join(lines)), ("b", "program", cons)]
    else:
        tail = r.choice(["SWP\nOUT ACC", "OUT ACC", f"POP {stacks[-1]}, ACC\nOUT ACC", "MOV 9, ACC\nOUT ACC"])
        rows = [("a", "program", "\n".join(lines) + "\n" + tail)]
    rows += [(s, "stack", "") for s in stacks]
    r.shuffle(rows)
    return rows, dict(kind=1, mask=r.choice([15, 63, 255]))
