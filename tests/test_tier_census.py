"""Tier census: which executor tier every network lands
on -- 1,000 tisgen.random_network seeds and the crafted classes of
tisgen.census_classes -- as the product decides it (check library mkc_tier:
schedule compiler, then the native generator and its bounds; no hiprtc).
Prints the table; the assertions pin the classes' tiers so a change shows."""
import collections

import numpy as np
import pytest

from oracle import pyoracle as po
import schedcheck as sc
from tisgen import census_classes, random_network


def test_random_network_census(capsys):
    counts = collections.Counter()
    reasons = collections.Counter()
    for seed in range(1000):
        t, why = sc.tier(random_network(seed))
        counts[t] += 1
        reasons[(t, why.split(" (")[0][:60])] += 1
    with capsys.disabled():
        print("\nrandom_network census over 1000 seeds:", dict(counts))
        for (t, why), n in reasons.most_common(12):
            print(f"  {t:9s} {n:5d}  {why}")
    assert sum(counts.values()) == 1000
    assert counts["native"] >= 995, counts  # the native tier takes (almost) everything


@pytest.mark.parametrize("cls", sorted(census_classes()))
def test_crafted_class_tiers(cls, capsys):
    for label, nodes, gen in census_classes()[cls]:
        t, why = sc.tier(nodes)
        with capsys.disabled():
            print(f"\n{cls:32s} {label:12s} tier={t} ({why[:80]})")
        # every class runs, on some tier, bit-exact with the oracle (host model of tier 2 where it compiles)
        xs = po.gen_inputs(11, 300, **gen)
        ref = po.OracleNet(nodes).compute_batch(xs)
        assert (ref[1] & po.ST_HAS_OUTPUT).any()
        if t != "interp":
            got = sc.emulate(nodes, xs)
            assert np.array_equal(got[0], ref[0]) and np.array_equal(got[1], ref[1]) and np.array_equal(got[2], ref[2])
