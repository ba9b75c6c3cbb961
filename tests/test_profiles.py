"""The committed PMC profiles (profiles/pmc_<workload>.json) price bench.py's
roofline only when their module is the one the bench runs (bench.py
measured_profile matches the kernel hash).  A code-generator change that
alters a module's source silently turns its line's issue roofline into the
"no PMC profile" fallback; this check makes that change visible on the CPU
(the modules compile here with hiprtc; nothing runs)."""
import json
import os
import re
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
import misaka_net_amd as mk  # noqa: E402


@pytest.mark.parametrize("cfg", ["c2", "c3", "c4", "c4d256", "c4d1024", "c5", "t2_dyn_depth", "t1_two_stacks",
                                 "t_jro_heavy"])
def test_committed_profile_matches_the_module(cfg):
    workload, factory = bench.WORKLOADS[cfg][:2]
    path = os.path.join(ROOT, "profiles", f"pmc_{workload}.json")
    prof = json.load(open(path))
    want = re.search(r"kernel=(\S+)", prof["executor"]).group(1)
    got = re.search(r"kernel=(\S+)", mk.Network(factory()).plan()).group(1)
    assert got == want, f"{cfg}: module {got}, profile {want} (re-run tools/gpu_pmc_all.sh + tools/pmc_profile.py)"
