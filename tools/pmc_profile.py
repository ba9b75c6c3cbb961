"""Fold a tools/gpu_pmc_all.sh run into profiles/pmc_<workload>.json:

  python tools/pmc_profile.py TAG CONFIG [CONFIG ...]

Per executor dispatch (mk_jit_exec / tis_* kernels; the first two of each run
are compile / warm-up launches and are skipped):
  * HBM bytes: FETCH_SIZE and WRITE_SIZE (KiB, summed over the XCD rows) from
    separate passes.  gfx950 correction (MI355X_MICROARCH.md section HBM):
    FETCH_SIZE reports half the bytes of wide coalesced streaming reads, so it
    is doubled; WRITE_SIZE is taken as is.  Calibrated for the stack slots'
    own pattern too (tools/probe/pmc_calib.hip, profiles/r03g_pmc_calib.json:
    4 GiB moved by wave-blocked 4-byte buffer loads read FETCH_SIZE = 0.500x,
    the 16-byte streaming loads 0.500x, 4-byte buffer stores WRITE_SIZE =
    1.000x), so one factor serves every workload here.  These are L2 <-> fabric bytes
    (Infinity-Cache hits included), i.e. what left the XCDs' L2s.
  * SQ counters (one pass of 8 SQ + GRBM_GUI_ACTIVE): VALU / SALU wave-
    instructions, VALU lane cycles, waves, vector memory instructions.
  * LDS counters (a fourth pass): LDS wave-instructions, bank-conflict and
    LDS-array cycles (bench.py's LDS bound for stacks kept in LDS).
The bench line's retired node-instructions per launch comes from the same
runs (node_instr_per_lane x lanes)."""
import collections
import csv
import glob
import json
import os
import sys

tag, cfgs = sys.argv[1], sys.argv[2:]


def per_dispatch(d, tuned=False):
    rows = collections.defaultdict(lambda: collections.defaultdict(float))
    grid = {}
    for p in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(p)):
            k = r["Kernel_Name"]
            if not (k.startswith("mk_jit_exec") or "tis_" in k):
                continue
            rows[r["Counter_Name"]][int(r["Dispatch_Id"])] += float(r["Counter_Value"])
            grid[int(r["Dispatch_Id"])] = int(r["Grid_Size"])
    # a kernel whose grid is measured (mk_exec.hip GridTune, grid_tuned= in
    # the plan) runs its first launches at 3/4, 1/2 and all of the resident
    # grid, then at the one it keeps: the launches at the grid most ran
    keep = collections.Counter(grid[i] for i in sorted(grid)[2:]).most_common(1)
    out = {}
    for c, by in rows.items():
        ids = [i for i in sorted(by)[2:] if not tuned or grid[i] == keep[0][0]]
        out[c] = sum(by[i] for i in ids) / max(1, len(ids))
        out[c + "_dispatches"] = len(ids)
    return out


def bench_line(path):
    for line in open(path):
        if line.startswith("{"):
            return json.loads(line)
    return None


for cfg in cfgs:
    d = os.path.join("gpurun_out", tag, cfg)
    rec = bench_line(os.path.join(d, "SQ.log"))
    tuned = "grid_tuned=" in rec["config"]["executor"]
    fetch = per_dispatch(os.path.join(d, "FETCH_SIZE"), tuned)
    write = per_dispatch(os.path.join(d, "WRITE_SIZE"), tuned)
    sq = per_dispatch(os.path.join(d, "SQ"), tuned)
    lds = per_dispatch(os.path.join(d, "LDS"), tuned) if os.path.isdir(os.path.join(d, "LDS")) else {}
    workload = rec["config"]["workload"]
    lanes = rec["config"]["lanes_per_gpu"]
    retired = rec["node_instr_per_lane"] * lanes
    alg = rec["roofline_hbm"]["bytes_per_launch"]
    # a heavy kernel with HBM slots takes ceil(lanes / chunk) dispatches per
    # step (mk_net_plan's chunk=); the counters above are per dispatch
    plan = dict(w.split("=", 1) for w in rec["config"]["executor"].split() if "=" in w)
    per_step = -(-lanes // int(plan["chunk"])) if "chunk" in plan else 1
    for d in (fetch, write, sq, lds):
        for k in list(d):
            if not k.endswith("_dispatches"):
                d[k] *= per_step
    hbm = int(2 * fetch["FETCH_SIZE"] * 1024 + write["WRITE_SIZE"] * 1024)
    out = {
        "workload": workload,
        "source": f"gpurun_out/{tag}/{cfg} (rocprofv3 --kernel-trace --pmc: FETCH_SIZE | WRITE_SIZE | SQ group, "
                  f"separate passes; tools/gpu_pmc_all.sh + tools/pmc_profile.py)",
        "executor": rec["config"]["executor"],
        "dispatches_per_launch": per_step,
        "fetch_kib_raw": fetch["FETCH_SIZE"],
        "write_kib_raw": write["WRITE_SIZE"],
        "correction": "read bytes = 2 x FETCH_SIZE x 1024 (gfx950; calibrated for 16-byte streaming and 4-byte "
                      "buffer loads, profiles/r03g_pmc_calib.json); write bytes = WRITE_SIZE x 1024 (4-byte stores 1.000x)",
        "hbm_bytes_per_launch": hbm,
        "algorithmic_bytes_per_launch": alg,
        "traffic_over_algorithmic": hbm / alg,
        "retired_per_launch": retired,
        "sq": {k: v for k, v in sq.items() if not k.endswith("_dispatches")},
        "sq_dispatches": sq.get("SQ_INSTS_VALU_dispatches"),
        "lds": {k: v for k, v in lds.items() if not k.endswith("_dispatches")},
    }
    s = out["sq"]
    if s.get("SQ_INSTS_VALU"):
        out["valu_lane_ops_per_instr"] = s["SQ_INSTS_VALU"] * 64 / retired
        out["salu_per_instr"] = s.get("SQ_INSTS_SALU", 0) / retired
        if s.get("SQ_ACTIVE_INST_VALU"):
            # active lanes per issued VALU wave-instruction (rocprof's VALU
            # utilisation): C2 / C4, whose lanes never diverge, read 0.96-1.0
            out["valu_lane_util"] = s["SQ_THREAD_CYCLES_VALU"] / (s["SQ_ACTIVE_INST_VALU"] * 64)
    with open(os.path.join("profiles", f"pmc_{workload}.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))
