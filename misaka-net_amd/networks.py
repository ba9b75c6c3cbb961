"""The networks of BASELINE.json's five configs.

C1/C2  docker-compose example network (docker-compose.yml:35-40,54-59): the
       YAML ``|`` block keeps one trailing newline, so each program has a
       sixth, empty line that executes as NOP.  README.md:39-44: result x+2.
C3     network built around docs/sample.txt "Example 2" (sample.txt:20-29),
       which is not loadable verbatim: ``entry`` feeds the
       input to ``router`` (sample.txt:20-29 verbatim, comp1:R1 -> pos:R3 and
       comp1:R3 -> neg:R3); ``pos``/``neg`` run sample.txt:2-3 without the
       ``//`` comments (MOV R3, ACC / ADD ACC) then OUT ACC.  Zero input ->
       no output (quiescent); otherwise int32(2x).
C4     8-program-node pipeline; node k pushes D values to its own stack,
       pops them back folding sum = 3*sum + v (ports used as scratch), and forwards the
       int32 sum to node k+1; the last node outputs.
C5     data-dependent countdown (``L: SUB 1 / JGZ L``) feeding a JRO-dispatched
       digit loop: trip counts follow the input, lanes diverge.
"""
from __future__ import annotations

from .network import NodeSpec

EXAMPLE_MISAKA1 = "IN ACC\nADD 1\nMOV ACC, misaka2:R0\nMOV R0, ACC\nOUT ACC\n"
EXAMPLE_MISAKA2 = "MOV R0, ACC\nADD 1\nPUSH ACC, misaka3\nPOP misaka3, ACC\nMOV ACC, misaka1:R0\n"


def example_network():
    """docker-compose.yml: master last_order, programs misaka1/misaka2, stack misaka3."""
    return [
        NodeSpec("misaka1", "program", EXAMPLE_MISAKA1),
        NodeSpec("misaka2", "program", EXAMPLE_MISAKA2),
        NodeSpec("misaka3", "stack"),
        NodeSpec("last_order", "master"),
    ]


SAMPLE_ROUTER = (
    "START:\n"
    "    MOV R0, ACC\n"
    "    JGZ POSITIVE\n"
    "    JLZ NEGATIVE\n"
    "    JMP START\n"
    "POSITIVE: MOV ACC, pos:R3\n"
    "    JMP START\n"
    "NEGATIVE:\n"
    "    MOV ACC, neg:R3\n"
    "    JMP START\n"
)
SAMPLE_DOUBLER = "MOV R3, ACC\nADD ACC\nOUT ACC\n"


def sample_network():
    return [
        NodeSpec("entry", "program", "IN ACC\nMOV ACC, router:R0\n"),
        NodeSpec("router", "program", SAMPLE_ROUTER),
        NodeSpec("pos", "program", SAMPLE_DOUBLER),
        NodeSpec("neg", "program", SAMPLE_DOUBLER),
        NodeSpec("master", "master"),
    ]


def pipeline_program(k: int, nodes: int, depth: int, observe: bool = False) -> str:
    """Node k of the C4 pipeline.  The bench network (observe=False) maps a
    node's input y to c*y + d with c = (3^depth - 1)/2, which is even: after
    8 nodes c^8 = 0 mod 2^32, so its int32 output is the same for every
    input and only the last nodes' stack contents reach it.  observe=True
    keeps y in the node's own port R0 and adds it back at the end (c + 1 =
    (3^depth + 1)/2, odd): every node's stack order then reaches the output
    of every lane, which is what the full-size parity tests check."""
    me, stk = f"p{k}", f"s{k}"
    first = "IN ACC" if k == 0 else "MOV R0, ACC"
    last = "OUT ACC" if k == nodes - 1 else f"MOV ACC, p{k + 1}:R0"
    keep = [f"MOV ACC, {me}:R0"] if observe else []  # y into the node's own (drained) R0
    add = ["ADD R0"] if observe else []
    return "\n".join(
        [
            first,
            *keep,
            "SAV",  # BAK = x
            f"MOV {depth}, ACC",
            "PL: SWP",  # ACC = x+i, BAK = counter
            "ADD 1",
            f"PUSH ACC, {stk}",
            "SWP",
            "SUB 1",
            "JGZ PL",
            "MOV 0, ACC",
            "SAV",  # BAK = running sum
            f"MOV {depth}, ACC",
            f"MOV ACC, {me}:R1",  # counter kept in own port R1
            f"QL: POP {stk}, ACC",
            f"MOV ACC, {me}:R2",
            "SWP",
            # sum = 3*sum + v: order dependent, so LIFO order is checked, and
            # with an odd multiplier (invertible mod 2^32) every popped value
            # reaches the int32 output.  (4*sum + v, used before, left only
            # the last 16 pops live in the low 32 bits, and a compiler may
            # drop the others' loads.)
            f"MOV ACC, {me}:R3",
            "ADD ACC",
            "ADD R3",
            "ADD R2",
            "SAV",
            "MOV R1, ACC",
            "SUB 1",
            f"MOV ACC, {me}:R1",
            "JGZ QL",
            "MOV R1, NIL",  # drain the counter port
            "SWP",
            *add,
            last,
            "",
        ]
    )


def pipeline_network(depth: int = 64, nodes: int = 8, observe: bool = False):
    out = [NodeSpec(f"p{k}", "program", pipeline_program(k, nodes, depth, observe)) for k in range(nodes)]
    out += [NodeSpec(f"s{k}", "stack") for k in range(nodes)]
    return out


COUNTDOWN = "IN ACC\nSAV\nL: SUB 1\nJGZ L\nSWP\nMOV ACC, digits:R0\n"
# Repeatedly subtract 3; the remainder (1..3) selects one of three ADDs via JRO.
DIGITS = (
    "MOV R0, ACC\n"
    "JEZ Z\n"
    "JLZ Z\n"
    "L: SUB 3\n"
    "JGZ L\n"
    "ADD 3\n"
    "JRO ACC\n"
    "ADD 100\n"
    "ADD 10\n"
    "ADD 1\n"
    "OUT ACC\n"
    "JMP E\n"
    "Z: OUT -1\n"
    "E: NOP\n"
)


def countdown_network():
    return [
        NodeSpec("count", "program", COUNTDOWN),
        NodeSpec("digits", "program", DIGITS),
    ]


# ---- census classes (tests/test_tier_census.py, bench.py --config t_*) ---------
# Network shapes that stress the schedule compiler: control state that
# depends on the data through stack depths, many JRO arms, many nodes.
def census_classes():
    """{class: [(label, nodes, input kwargs for oracle.gen_inputs)]} -- shapes
    whose control state the schedule compiler may not bound (tests/
    test_tier_census.py; bench.py --config t_*)."""
    P = lambda name, text: NodeSpec(name, "program", text)  # noqa: E731
    S = lambda name: NodeSpec(name, "stack", "")  # noqa: E731
    # push x (0..255) values then pop them all: stack depth follows the data
    dyn_depth = [P("a", "IN ACC\nSAV\nJEZ E\nL: PUSH ACC, s\nSUB 1\nJGZ L\nSWP\nM: POP s, NIL\nSUB 1\nJGZ M\n"
                      "E: MOV 7, ACC\nOUT ACC"), S("s")]
    # two stacks, depths x & 15 and (x >> 4) & 15, popped into a sum
    two_stacks = [P("a", "IN ACC\nSAV\nMOV 0, ACC\nMOV ACC, a:R1\nSWP\nSAV\n"
                       "A: JEZ B\nPUSH ACC, s\nSUB 1\nJMP A\n"
                       "B: SWP\nSAV\nC: JEZ D\nPUSH ACC, t\nSUB 1\nJMP C\n"
                       "D: MOV R1, ACC\nOUT ACC"), S("s"), S("t")]
    # JRO-heavy: a loop whose body dispatches through JRO into one of 8 arms;
    # SAV after ADD 3 reloads the counter each round, so the loop never ends
    # and every lane runs to the budget (12 node-instructions per round)
    arms = "\n".join(f"ADD {k + 1}\nJMP N" for k in range(8))
    jro_heavy = [P("a", "IN ACC\nSAV\nL: SWP\nJEZ E\nSUB 1\nSWP\nADD 3\nSAV\nJRO 2\n" + arms +
                   "\nN: SWP\nSAV\nSWP\nJMP L\nE: SWP\nOUT ACC")]
    # 16 program nodes in a ring: each adds its index and forwards; node 0 outputs
    ring = []
    for k in range(16):
        nxt = f"n{(k + 1) % 16:02d}"
        if k == 0:
            ring.append(P("n00", f"IN ACC\nMOV ACC, {nxt}:R0\nMOV R1, ACC\nOUT ACC"))
        elif k == 15:
            ring.append(P(f"n{k:02d}", f"MOV R0, ACC\nADD {k}\nMOV ACC, n00:R1"))
        else:
            ring.append(P(f"n{k:02d}", f"MOV R0, ACC\nADD {k}\nMOV ACC, {nxt}:R0"))
    return {
        "data_dependent_stack_depth": [("dyn_depth", dyn_depth, dict(kind=1, mask=255))],
        "two_stacks_independent_depths": [("two_stacks", two_stacks, dict(kind=1, mask=255))],
        "jro_heavy": [("jro_heavy", jro_heavy, dict(kind=1, mask=1023))],
        "sixteen_nodes": [("ring16", ring, dict(kind=0))],
    }


CONFIGS = {
    "c1_example_cpu": example_network,
    "c2_example": example_network,
    "c3_sample": sample_network,
    "c4_pipeline": pipeline_network,
    "c5_countdown": countdown_network,
}
