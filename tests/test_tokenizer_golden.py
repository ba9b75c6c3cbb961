"""The front end against golden vectors pinned to the reference's own
regexes (tests/golden/make_tokenizer_golden.py reads the RE2 table of
internal/tis/tokenizer.go and evaluates it; the fixture holds only programs
and results): token vectors, accept / reject, and the Go error text, for the
product parser (csrc/tis_front.cpp through the C ABI) and the oracle."""
import json
import os

import misaka_net_amd as mk
from oracle import pyoracle as po

VECS = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "front", "tokenizer_reference_regex.json")))["vectors"]


def _run(fn, err, program):
    try:
        return ["ok", [list(t) for t in fn(program)]]
    except err as e:
        return ["err", str(e)]


def test_fixture_covers_both_outcomes():
    kinds = [r[0] for _, r in VECS]
    assert len(VECS) > 2500 and kinds.count("ok") > 500 and kinds.count("err") > 500


def test_product_parser_matches_reference_regexes():
    bad = [(p, r, got) for p, r in VECS if (got := _run(mk.tokenize, mk.TisParseError, p)) != r]
    assert not bad, bad[:3]


def test_check_library_front_end_matches_reference_regexes():
    # the same parser built into the CPU check library (and, under
    # tests/test_sanitized.py, its ASan + UBSan build)
    import schedcheck as sc

    bad = [(p, r, got) for p, r in VECS if (got := _run(sc.tokenize, mk.TisParseError, p)) != r]
    assert not bad, bad[:3]


def test_oracle_matches_reference_regexes():
    bad = [(p, r, got) for p, r in VECS if (got := _run(po.tokenize, po.OracleParseError, p)) != r]
    assert not bad, bad[:3]
