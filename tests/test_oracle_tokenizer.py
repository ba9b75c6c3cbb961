"""Known-answer tests of the oracle's restatement of internal/tis/tokenizer.go.

Hand-derived from the reference regexes (tokenizer.go:12,34,44-99) under Go
RE2 semantics (\\s = [\\t\\n\\f\\r ], \\w = [0-9A-Za-z_]) -- the reference
ships no tests, so these are the pinning cases.
"""
import pytest

from oracle import pyoracle as po


def tok(p):
    return po.tokenize(p)


def err(p):
    with pytest.raises(po.OracleParseError) as e:
        po.tokenize(p)
    return str(e.value)


def test_example_programs_trailing_newline_is_nop():
    # docker-compose.yml:35-40 keeps a trailing "\n" -> 6 lines, last one NOP
    t = tok("IN ACC\nADD 1\nMOV ACC, misaka2:R0\nMOV R0, ACC\nOUT ACC\n")
    assert t == [
        ["IN", "ACC"],
        ["ADD_VAL", "1"],
        ["MOV_SRC_NETWORK", "ACC", "misaka2:R0"],
        ["MOV_SRC_LOCAL", "R0", "ACC"],
        ["OUT_SRC", "ACC"],
        ["NOP"],
    ]


@pytest.mark.parametrize(
    "line,tokens",
    [
        ("NOP", ["NOP"]),
        ("SWP  ", ["SWP"]),
        ("SAV\t", ["SAV"]),
        ("NEG\r", ["NEG"]),  # CRLF files: \r is in \s
        ("MOV 1, ACC", ["MOV_VAL_LOCAL", "1", "ACC"]),
        ("MOV -5 ,\tNIL", ["MOV_VAL_LOCAL", "-5", "NIL"]),
        ("MOV 007, ACC", ["MOV_VAL_LOCAL", "007", "ACC"]),
        ("MOV 3, a_1:R3", ["MOV_VAL_NETWORK", "3", "a_1:R3"]),
        ("MOV R2, NIL", ["MOV_SRC_LOCAL", "R2", "NIL"]),
        ("MOV ACC, ACC:R0", ["MOV_SRC_NETWORK", "ACC", "ACC:R0"]),
        ("MOV NIL,  x:R1  ", ["MOV_SRC_NETWORK", "NIL", "x:R1"]),
        ("ADD -9223372036854775808", ["ADD_VAL", "-9223372036854775808"]),
        ("SUB 99999999999999999999", ["SUB_VAL", "99999999999999999999"]),  # Atoi fails only at run time
        ("ADD ACC", ["ADD_SRC", "ACC"]),
        ("SUB R3", ["SUB_SRC", "R3"]),
        ("JRO -3", ["JRO_VAL", "-3"]),
        ("JRO R1", ["JRO_SRC", "R1"]),
        ("PUSH 4, stk", ["PUSH_VAL", "4", "stk"]),
        ("PUSH R0, ACC", ["PUSH_SRC", "R0", "ACC"]),
        ("POP stk, NIL", ["POP", "stk", "NIL"]),
        ("IN NIL", ["IN", "NIL"]),
        ("OUT -1", ["OUT_VAL", "-1"]),
        ("OUT R0", ["OUT_SRC", "R0"]),
        ("", ["NOP"]),
        ("   ", ["NOP"]),
        ("# comment ### x", ["NOP"]),
        ("  #", ["NOP"]),
        ("L1:", ["NOP"]),
        ("  L1:   NOP", ["NOP"]),
        ("L1:# c", ["NOP"]),
        ("L1:MOV 1, ACC", ["MOV_VAL_LOCAL", "1", "ACC"]),
    ],
)
def test_accept(line, tokens):
    assert tok(line) == [tokens]


@pytest.mark.parametrize(
    "line",
    [
        "MOV 1,ACC",  # \s+ required after the comma
        "mov 1, ACC",  # opcodes are case-sensitive
        "ADD +1",  # -?\d+ has no '+'
        "ADD 1 # c",  # comments only as a whole line
        "ADD 1 // c",
        "MOV 1, acc",
        "MOV R4, ACC",
        "MOV 1, a:R4",
        "MOV 1, a :R0",
        "MOV BAK, ACC",  # BAK is never an operand
        "POP stk, R0",
        "IN R0",
        "\vNOP",  # \v is not in Go's \s
        "NOP\v",
        "NOPE",
        "JRO",
        "PUSH 1 , s x",
        "OUT 1, ACC",
        "L1 : NOP",
    ],
)
def test_reject_not_valid(line):
    assert err(line) == f"line 0, '{line.lstrip(' ')}' not a valid instruction"


def test_reject_error_text_uses_stripped_instruction_and_line_index():
    assert err("NOP\n  L:  ADD  1 # c") == "line 1, 'ADD  1 # c' not a valid instruction"


def test_undeclared_label_is_uppercased():
    assert err("NOP\nJMP nowhere") == "line 1, label 'NOWHERE' was not declared"


def test_labels_case_insensitive_and_uppercased():
    assert tok("loop: NOP\nJMP Loop") == [["NOP"], ["JMP", "LOOP"]]
    assert po.label_map("a: NOP\n  b:\nNOP\nc_9:") == {"A": 0, "B": 1, "C_9": 3}


def test_duplicate_labels():
    assert err("a:\nA: NOP") == "Cannot repeat label"


def test_label_map_before_tokenize_error():
    # GenerateLabelMap runs first (program.go:180), so its error wins
    assert err("MOV 1,ACC\na:\na:") == "Cannot repeat label"


def test_first_error_in_line_order():
    assert err("JMP X\nbad") == "line 0, label 'X' was not declared"
    assert err("bad\nJMP X") == "line 0, 'bad' not a valid instruction"


def test_empty_program_is_one_nop():
    assert tok("") == [["NOP"]]


@pytest.mark.parametrize(
    "s,v",
    [("0", 0), ("-0", 0), ("007", 7), ("+5", 5), ("9223372036854775807", 2**63 - 1),
     ("-9223372036854775808", -(2**63))],
)
def test_go_atoi_accepts(s, v):
    assert po.go_atoi(s) == v


@pytest.mark.parametrize("s", ["", "+", "-", " 1", "1 ", "0x10", "1_000", "9223372036854775808",
                               "-9223372036854775809", "1e3"])
def test_go_atoi_rejects(s):
    with pytest.raises(ValueError):
        po.go_atoi(s)
