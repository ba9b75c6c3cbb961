"""Golden vectors for the front end, pinned to the reference's own regexes.

    python tests/golden/make_tokenizer_golden.py [/root/reference]

The Go reference cannot run here (no Go toolchain), but its tokenizer is a
table of RE2 patterns.  This script reads that table out of
internal/tis/tokenizer.go at generation time -- the label pattern
(tokenizer.go:12), the prefix pattern (:34) and, in source order, every
(pattern, token vector) branch of Tokenize (:40-101) -- evaluates the
patterns with Python's `re` after translating RE2's ASCII classes exactly
(`\\s` = [\\t\\n\\f\\r ], `\\w` = [0-9A-Za-z_], `\\d` = [0-9]; `$` = end of text,
RE2 has no line mode here), and drives them with a restatement of
GenerateLabelMap / Tokenize / LoadProgram's split (tokenizer.go:11-106,
program.go:178-193).  It commits only data: each program and the result
the reference's patterns give it (token vectors, or the Go error text).
tests/test_tokenizer_golden.py checks the product front end
(csrc/tis_front.cpp) and the oracle against it on every CPU run."""
import json
import os
import random
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.dirname(os.path.dirname(HERE)), os.path.dirname(HERE)]

REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
SRC = open(os.path.join(REF, "internal", "tis", "tokenizer.go")).read()


def rx(go: str) -> "re.Pattern":
    """RE2 (Perl syntax, no flags) -> Python, exact for the classes used."""
    out, i = [], 0
    while i < len(go):
        c = go[i]
        if c == "\\" and i + 1 < len(go):
            e = go[i + 1]
            out.append({"s": "[\\t\\n\\f\\r ]", "w": "[0-9A-Za-z_]", "d": "[0-9]"}.get(e, "\\" + e))
            i += 2
            continue
        out.append("\\Z" if c == "$" else c)
        i += 1
    return re.compile("".join(out))


LABEL = rx(re.search(r"labelRe := regexp\.MustCompile\(`([^`]*)`\)", SRC).group(1))
PREFIX = rx(re.search(r"prefixRe := regexp\.MustCompile\(`([^`]*)`\)", SRC).group(1))
# each branch: the pattern and what it appends (a []string literal, or the jump form)
BRANCHES = []
for m in re.finditer(r"regexp\.MustCompile\(`([^`]*)`\)\.FindStringSubmatch\(instr\); len\(m\) > 0 \{(.*?)\n\t\t\}",
                     SRC, re.S):
    body = m.group(2)
    lit = re.search(r"asm\[i\] = \[\]string\{(.*)\}", body)
    jump = "labelMap[label]" in body
    elems = []
    for e in [x.strip() for x in lit.group(1).split(",")] if lit else []:
        if e.startswith('"'):
            elems.append(("lit", e.strip('"')))
        elif re.fullmatch(r"m\[(\d)\]", e):
            elems.append(("grp", int(e[2])))
        elif re.fullmatch(r'fmt\.Sprintf\("%s_(\w+)"', e):
            elems.append(("suffix", re.fullmatch(r'fmt\.Sprintf\("%s_(\w+)"', e).group(1)))
        elif re.fullmatch(r"m\[(\d)\]\)", e):  # the Sprintf's argument, split off by the comma
            elems[-1] = ("sprintf", int(e[2]), elems[-1][1])
        elif e == "label":
            elems.append(("label",))
        else:
            raise SystemExit(f"unknown token element {e!r}")
    BRANCHES.append((rx(m.group(1)), "jump" if jump else "list", elems))
assert len(BRANCHES) == 17, len(BRANCHES)  # `^#.*$` and the 16 instruction forms


class GoError(Exception):
    pass


def generate_label_map(lines):  # tokenizer.go:11-26
    lm = {}
    for i, line in enumerate(lines):
        mm = LABEL.match(line)
        if mm:
            label = mm.group(1).upper()
            if label in lm:
                raise GoError("Cannot repeat label")
            lm[label] = i
    return lm


def tokenize(lines, lm):  # tokenizer.go:29-106
    asm = []
    for i, instr in enumerate(lines):
        pm = PREFIX.match(instr)
        if pm:
            instr = instr[pm.end():]
        if len(instr) == 0:
            asm.append(["NOP"])
            continue
        for pat, kind, elems in BRANCHES:
            mm = pat.match(instr)
            if not mm:
                continue
            if kind == "jump":
                label = mm.group(2).upper()
                if label not in lm:
                    raise GoError(f"line {i}, label '{label}' was not declared")
                asm.append([mm.group(1), label])
            elif not elems:  # the comment branch
                asm.append(["NOP"])
            else:
                toks = []
                for e in elems:
                    if e[0] == "lit":
                        toks.append(e[1])
                    elif e[0] == "grp":
                        toks.append(mm.group(e[1]))
                    elif e[0] == "sprintf":
                        toks.append(f"{mm.group(e[1])}_{e[2]}")
                asm.append(toks)
            break
        else:
            raise GoError(f"line {i}, '{instr}' not a valid instruction")
    return asm


def load_program(text):  # program.go:178-193: split, label map, tokenize
    lines = text.split("\n")
    try:
        return ["ok", tokenize(lines, generate_label_map(lines))]
    except GoError as e:
        return ["err", str(e)]


def corpus():
    import misaka_net_amd as mk
    from tisgen import mutated_program, random_program

    progs = [mk.networks.EXAMPLE_MISAKA1, mk.networks.EXAMPLE_MISAKA2, mk.networks.SAMPLE_ROUTER,
             mk.networks.DIGITS, mk.networks.COUNTDOWN, mk.networks.pipeline_program(3, 8, 64), "", "\n\n"]
    forms = ["NOP", "SWP", "SAV", "NEG", "MOV 1, ACC", "MOV -7, NIL", "MOV 3, a:R2", "MOV R1, ACC", "MOV ACC, b:R0",
             "ADD 5", "SUB -5", "ADD R3", "SUB ACC", "JMP L", "JEZ l", "JNZ L", "JGZ L", "JLZ L", "JRO -2", "JRO R0",
             "PUSH 4, s", "PUSH ACC, s", "POP s, ACC", "POP s, NIL", "IN ACC", "IN NIL", "OUT 9", "OUT R2",
             "# comment", "L:", "l: NOP"]
    r = random.Random(20261017)
    ws = [" ", "  ", "\t", "\f", "\r", "\v", "", " "]
    for _ in range(1500):
        lines = []
        for _ in range(r.randint(1, 6)):
            f = r.choice(forms)
            if r.random() < 0.5:  # whitespace around and inside, some of it not \s in RE2
                f = r.choice(ws) + f.replace(" ", r.choice(ws + [" "]), r.randint(0, 2)) + r.choice(ws)
            if r.random() < 0.2:
                f = f.replace(",", r.choice([",", " ,", ",,", ""]), 1)
            if r.random() < 0.1:
                f = f.lower() if r.random() < 0.5 else f + " # x"
            if r.random() < 0.1:
                f = r.choice(["L: ", "l:", "x_1:\t", "9: "]) + f
            lines.append(f)
        progs.append("\n".join(lines))
    progs += [mutated_program(s) for s in range(1000)]
    rr = random.Random(12)
    progs += [random_program(rr, ["a", "b"], ["s"], ["ghost"]) for _ in range(300)]
    return progs


if __name__ == "__main__":
    vecs = [[p, load_program(p)] for p in corpus()]
    out = os.path.join(HERE, "front", "tokenizer_reference_regex.json")
    with open(out, "w") as f:
        json.dump({"source": "tests/golden/make_tokenizer_golden.py over internal/tis/tokenizer.go's patterns",
                   "vectors": vecs}, f, separators=(",", ":"))
    ok = sum(1 for _, r in vecs if r[0] == "ok")
    print(f"{len(vecs)} programs ({ok} accepted) -> {out}")
