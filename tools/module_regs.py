#!/usr/bin/env python3
"""Registers of the native tier's modules, on the CPU (no GPU needed).

For each bench workload: load the network, ask for its plan (mk_net_plan
compiles the module with the process's hiprtc -- this ROCm's, as long as the
script does not import torch first), dump the code object (MK_JIT_DUMP) and
read its kernel metadata: VGPRs, AGPRs, SGPRs, spills, scratch, LDS.

  python tools/module_regs.py [config ...] [--src DIR]   (default: every config)

The same compiler builds the module on the GPU box (mk_exec.hip hiprtc_run),
so these are the counts the kernel runs with there.
"""
from __future__ import annotations

import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"
FIELDS = ("vgpr_count", "agpr_count", "sgpr_count", "vgpr_spill_count", "sgpr_spill_count",
          "private_segment_fixed_size", "group_segment_fixed_size")


def kernel_meta(co_path: str) -> dict:
    notes = subprocess.run([READELF, "--notes", co_path], capture_output=True, text=True, check=True).stdout
    meta = {}
    for f in FIELDS:
        m = re.search(rf"\.{f}:\s+(\d+)", notes)
        meta[f] = int(m.group(1)) if m else None
    return meta


def configs():
    import misaka_net_amd as mk

    nets = {
        "c2": mk.networks.example_network,
        "c3": mk.networks.sample_network,
        "c4": lambda: mk.networks.pipeline_network(64),
        "c4d256": lambda: mk.networks.pipeline_network(256),
        "c4d1024": lambda: mk.networks.pipeline_network(1024),
        "c5": mk.networks.countdown_network,
    }
    cc = mk.networks.census_classes()
    nets["t2_dyn_depth"] = lambda: cc["data_dependent_stack_depth"][0][1]
    nets["t1_two_stacks"] = lambda: cc["two_stacks_independent_depths"][0][1]
    nets["t_jro_heavy"] = lambda: cc["jro_heavy"][0][1]
    nets["t_ring16"] = lambda: cc["sixteen_nodes"][0][1]
    return nets


def module_of(name: str, factory, src_dir: str | None = None) -> dict:
    import misaka_net_amd as mk

    with tempfile.TemporaryDirectory() as td:
        co = os.path.join(td, f"{name}.co")
        os.environ["MK_JIT_DUMP"] = co
        try:
            plan = mk.Network(factory()).plan()
        finally:
            del os.environ["MK_JIT_DUMP"]
        rec = {"config": name, "plan": " ".join(w for w in plan.split() if not w.startswith("knobs="))}
        if os.path.exists(co):
            rec.update(kernel_meta(co))
            if src_dir:
                os.makedirs(src_dir, exist_ok=True)
                os.replace(co + ".hip", os.path.join(src_dir, f"{name}.hip"))
                os.replace(co, os.path.join(src_dir, f"{name}.co"))
    return rec


def main(argv):
    src_dir = None
    if "--src" in argv:
        i = argv.index("--src")
        src_dir = argv[i + 1]
        argv = argv[:i] + argv[i + 2:]
    nets = configs()
    for name in argv or list(nets):
        r = module_of(name, nets[name], src_dir)
        shape = dict(w.split("=", 1) for w in r["plan"].split() if "=" in w).get("shape")
        print(f"{name:14s} shape={shape!s:22s} vgpr={r.get('vgpr_count')} agpr={r.get('agpr_count')} "
              f"sgpr={r.get('sgpr_count')} spill={r.get('vgpr_spill_count')}/{r.get('sgpr_spill_count')} "
              f"scratch={r.get('private_segment_fixed_size')} lds={r.get('group_segment_fixed_size')}")


if __name__ == "__main__":
    main(sys.argv[1:])
