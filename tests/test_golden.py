"""Committed golden vectors (tests/golden/*.json, made by make_golden.py):
the oracle must keep reproducing them; the compiled schedule (host model)
and both GPU tiers must match them bit for bit."""
import glob
import json
import os

import numpy as np
import pytest

import misaka_net_amd as mk
from oracle import pyoracle as po
import schedcheck as sc

FILES = sorted(glob.glob(os.path.join(os.path.dirname(__file__), "golden", "*.json")))
IDS = [os.path.basename(f)[:-5] for f in FILES]


def load(path):
    with open(path) as f:
        g = json.load(f)
    return [tuple(r) for r in g["network"]], g


def check(got, g):
    out, st, sp = got
    assert np.asarray(out).tolist() == g["out"]
    assert np.asarray(st).tolist() == g["status"]
    assert np.asarray(sp).tolist() == g["steps"]


def test_fixtures_present():
    assert len(FILES) >= 9


@pytest.mark.parametrize("path", FILES, ids=IDS)
def test_oracle_reproduces_golden(path):
    nodes, g = load(path)
    check(po.OracleNet(nodes).compute_batch(g["inputs"], **g["options"]), g)


@pytest.mark.parametrize("path", FILES, ids=IDS)
def test_compiled_schedule_reproduces_golden(path):
    nodes, g = load(path)
    check(sc.emulate(nodes, g["inputs"], **g["options"])[:3], g)


@pytest.mark.gpu
@pytest.mark.parametrize("interp", [False, True], ids=["compiled", "interp"])
@pytest.mark.parametrize("path", FILES, ids=IDS)
def test_gpu_reproduces_golden(gpu, path, interp):
    nodes, g = load(path)
    r = mk.Network(nodes).compute_batch(g["inputs"], interp=interp, **g["options"])
    check((r.out, r.status, r.steps), g)
